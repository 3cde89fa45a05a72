// CPU side of the native multi-rank loop (tclb_rt/dist_loop.hpp), for the OpenMP
// executor: the same loop and halo plan as the GPU build, with two transports —
//   * transport 0: this rank is its own neighbour, the plan's sends and receives are
//     paired in order and copied (memcpy);
//   * transport 2: a callback executes one stage's ops (tclb_amd/parallel/native.py runs
//     them as torch.distributed gloo isend/irecv between CPU ranks).
// The executor's launches are synchronous, so an exchange completes inside start().
#include <string.h>

#include "tclb_rt/dist_loop.hpp"

namespace {

typedef int (*xchg_fn)(void* user, void* base, const tclb::HaloOp* ops, int nops);

struct CpuX {
  int transport;
  int rank;
  xchg_fn cb;
  void* user;
  int start(char* base, const tclb::HaloOp* ops, int nops) {
    if (transport == 2) return cb ? cb(user, base, ops, nops) : -4;
    return tclb::dist_self_pairs(base, ops, nops, rank, [](char* d, const char* s, long long b) {
      memcpy(d, s, (size_t)b);
      return 0;
    });
  }
  int finish() { return 0; }
};

}  // namespace

extern "C" {

int tclb_dist_iterate_cpu(const tclb::Launch* L, int prec, int nsteps, int glob_last, const tclb::DistPlan* P,
                          int transport, int rank, xchg_fn cb, void* user, tclb::run_fn run,
                          tclb::sample_fn sample, const tclb::SamplePlan* sp) {
  CpuX x{transport, rank, cb, user};
  return tclb::dist_iterate(*L, prec, nsteps, glob_last, *P, x, run, sample, sp);
}

int tclb_dist_sizeof_plan_cpu() { return (int)sizeof(tclb::DistPlan); }
int tclb_dist_sizeof_op_cpu() { return (int)sizeof(tclb::HaloOp); }

}  // extern "C"
