// Adjoint (reverse) executor on the CPU: every node update is re-run with Dual<double,K>
// reals; the local Jacobian is contracted with the adjoint of the stage outputs and
// scattered to the adjoint of the loaded inputs (AdRec::scatter, atomics), the
// Objective's derivative is added with weight ctx->obj_weight.
// Replaces the reference's Tapenade-generated Run_b() kernels
// (src/LatticeAccess.inc.cpp.Rt:349-361 adjoint push, tools/makeAD).
#pragma once
#include <utility>
#include <omp.h>
#include "ad.hpp"

namespace tclb {
namespace exec {

template <class Model, int K, int STG>
inline void ad_stage(const Launch& L) {
  typedef Dual<double, K> D;
  constexpr int NG = Model::NGLOBALS_;
  constexpr int NSUM = Model::NSUMGLOBALS_;
  AdCtx* ctx = (AdCtx*)L.ext[5];
#pragma omp parallel
  {
#pragma omp for collapse(2) schedule(static)
    for (int z = L.zlo; z < L.zhi; z++)
      for (int y = L.ylo; y < L.yhi; y++)
        for (int x = L.xlo; x < L.xhi; x++) {
          if constexpr (has_rev<typename Model::template NodeT<double, double, true>>::value) {
            // a node with a hand-written reverse sweep (Model.set_reverse; Launch.next[5] = 1
            // when no setting is seeded): one reverse pass instead of the dual numbers
            if (L.next[5] == 1) {
              double gd[NG];
              for (int i = 0; i < NG; i++) gd[i] = 0.0;
              typename Model::template NodeT<double, double, true> nr(L, x, y, z, gd);
              if (nr.template rev_ok<STG>()) {
                nr.template rev_stage<STG>(*ctx);
                continue;
              }
            }
          }
          D g[NG];
          for (int i = 0; i < NG; i++) g[i] = i < NSUM ? D(0.0) : D(-1e30);
          typename Model::template NodeT<D, double, true> n(L, x, y, z, g);
          n.template run_stage<STG>();
          if (ctx != nullptr && ctx->obj_weight != 0.0) n.ad_.scatter(ctx->obj_weight, g[Model::OBJ_]);
        }
  }
}

template <class Model, int K, int... I>
inline int ad_run_impl(const Launch& L, std::integer_sequence<int, I...>) {
  bool found = false;
  ((L.stage == I ? (ad_stage<Model, K, I>(L), found = true) : false), ...);
  return found ? 0 : -2;
}

}  // namespace exec
}  // namespace tclb

#define TCLB_EXPORT_AD(NAME, MODEL, K)                                                       \
  extern "C" int tclb_##NAME##_adjoint(const tclb::Launch* L) {                              \
    return tclb::exec::ad_run_impl<MODEL, K>(*L, std::make_integer_sequence<int, MODEL::NSTAGES_>{}); \
  }                                                                                          \
  extern "C" int tclb_##NAME##_ad_tangents() { return K; }                                   \
  extern "C" int tclb_##NAME##_sizeof_launch() { return (int)sizeof(tclb::Launch); }
