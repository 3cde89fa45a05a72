// CPU executor (OpenMP) for the same node code: the "fake device" used for tests and
// for the CPU plumbing configuration (reference CROSS_CPU backend, src/cross.h:185-346).
#pragma once
#include <utility>
#include <vector>
#include <omp.h>
#include "core.hpp"

namespace tclb {
namespace exec {

template <class Model, class R, class S, int STG, bool GLOB>
inline void cpu_stage(const Launch& L) {
  constexpr int NG = GLOB ? Model::NGLOBALS_ : 1;
  constexpr int NSUM = Model::NSUMGLOBALS_;
  std::vector<double> acc(NG, 0.0);
  for (int i = NSUM; i < NG; i++) acc[i] = -1e300;
  typedef typename Model::template NodeT<R, S, GLOB> N;
  typedef typename N::G_ G;
#pragma omp parallel
  {
    G g[NG];
    for (int i = 0; i < NG; i++) g[i] = i < NSUM ? G(0) : G(-1e30);
#pragma omp for collapse(2) schedule(static)
    for (int z = L.zlo; z < L.zhi; z++)
      for (int y = L.ylo; y < L.yhi; y++)
        for (int x = L.xlo; x < L.xhi; x++) {
          N n(L, x, y, z, g);
          n.template run_stage<STG>();
        }
    if (GLOB) {
#pragma omp critical
      for (int i = 0; i < NG; i++) {
        if (i < NSUM) acc[i] += (double)g[i];
        else acc[i] = acc[i] > (double)g[i] ? acc[i] : (double)g[i];
      }
    }
  }
  if (GLOB) {
    for (int i = 0; i < NG; i++) {
      if (i < NSUM) L.globals[i] += acc[i];
      else L.globals[i] = L.globals[i] > acc[i] ? L.globals[i] : acc[i];
    }
  }
}

template <class Model, class R, class S, bool G, int... I>
inline int cpu_run_impl(const Launch& L, std::integer_sequence<int, I...>) {
  bool found = false;
  ((L.stage == I ? (cpu_stage<Model, R, S, I, G>(L), found = true) : false), ...);
  return found ? 0 : -2;
}

template <class Model, class R, class S>
inline int run_stage(const Launch& L) {
  using Seq = std::make_integer_sequence<int, Model::NSTAGES_>;
  if (L.glob) return cpu_run_impl<Model, R, S, true>(L, Seq{});
  return cpu_run_impl<Model, R, S, false>(L, Seq{});
}

template <class Model, class R, class S>
inline int run_quantity(const Launch& L) {
  const int nc = L.reserved0 > 0 ? L.reserved0 : 1;
#pragma omp parallel for collapse(2) schedule(static)
  for (int z = L.zlo; z < L.zhi; z++)
    for (int y = L.ylo; y < L.yhi; y++)
      for (int x = L.xlo; x < L.xhi; x++) {
        typename Model::template NodeT<R, S, false>::G_ g[1];
        typename Model::template NodeT<R, S, false> n(L, x, y, z, g);
        n.pop();
        R o[3] = {R(0), R(0), R(0)};
        n.get_quantity(L.quantity, o);
        const long long idx = (long long)(x - L.xlo) + L.qsy * (y - L.ylo) + L.qsz * (z - L.zlo);
        R* out = (R*)L.aux;
        for (int c = 0; c < nc; c++) out[idx + (long long)c * L.qcomp] = o[c] * R(L.qscale);
      }
  return 0;
}

template <class Model, class R, class S>
inline int run_sample(const Launch& L, const SamplePlan& P) {
  if (P.np <= 0 || P.row < 0 || P.row >= P.rows) return 0;
  for (int p = 0; p < P.np; p++) {
    const int* c = P.points + 3 * p;
    typename Model::template NodeT<R, S, false>::G_ g[1];
    typename Model::template NodeT<R, S, false> n(L, c[0], c[1], c[2], g);
    sample_node(n, P, P.out + ((long long)P.row * P.np + p) * P.width);
  }
  return 0;
}

}  // namespace exec
}  // namespace tclb

#define TCLB_EXPORT_MODEL(NAME, MODEL)                                                       \
  TCLB_EXPORT_COMMON(NAME, MODEL)                                                            \
  extern "C" int tclb_##NAME##_device() { return 0; }
