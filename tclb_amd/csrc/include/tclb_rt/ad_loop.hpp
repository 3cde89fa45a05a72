// Native reverse sweep of one checkpoint segment of an unsteady adjoint: the adjoint
// steps t = end-1 .. base of a single-stage action in one C++ call.
//
// Reference: Lattice::IterateTill / Iteration_Adj run the recorded primal and the
// Tapenade Run_b kernels per iteration in C++ (src/Lattice.cu.Rt:542-613,843-890).
// Here each step is: zero the incoming-adjoint buffer, then the AD executor's launch(es)
// for the step's input state — the model's reverse sweep (mode 1) and the dual-number
// windows over the nodes it does not cover (mode 2), or dual windows alone (mode 0).  The
// two adjoint buffers ping-pong (the output adjoint of one step is the input of the next)
// and each parity has its own executor context (tclb_amd/adjoint.py _ad_stage prepares
// both on the segment's first, sizing, call).  The AD kernel library is the model's
// libtclb_<model>_ad(hip).so; `run` is its tclb_<model>_adjoint.
#pragma once
#include "tclb/core.hpp"

namespace tclb {

struct AdSegPlan {
  int nsteps;
  int par0;              // parity of the first step's output-adjoint buffer
  int dual_count;        // mode 1: nodes recorded for the dual windows (launch when > 0)
  int mode;              // 0 dual windows only; 1 reverse sweep + dual windows (GPU, two
                         // launches); 2 one launch, reverse or dual per node (CPU executor)
  const long long* states;   // [nsteps] input state of each step (addresses)
  const int* iters;          // [nsteps] iteration of each step
  void* abuf[2];             // adjoint ping-pong buffers
  void* ctx[2];              // executor context of each parity (Launch.ext[5])
  long long abytes;          // bytes of one adjoint buffer
};

typedef int (*ad_run_fn)(const Launch*);

// Z: int zero(void* p, long long bytes) on the launch stream
template <class Zero>
inline int ad_segment(const Launch& L, const AdSegPlan& P, ad_run_fn run, Zero zero) {
  int r;
  for (int i = 0; i < P.nsteps; i++) {
    const int par = P.par0 ^ (i & 1);
    if ((r = zero(P.abuf[1 - par], P.abytes)) != 0) return r;
    Launch Q = L;
    Q.in = (const void*)P.states[i];
    Q.iter = P.iters[i];
    Q.ext[5] = P.ctx[par];
    if (P.mode == 1) {
      Q.next[5] = 1;
      Q.qcomp = 1;                     // the dual nodes are already recorded
      if ((r = run(&Q)) != 0) return r;
      if (P.dual_count > 0) {
        Q.next[5] = 2;
        Q.qcomp = P.dual_count;
        if ((r = run(&Q)) != 0) return r;
      }
    } else {
      Q.next[5] = P.mode == 2 ? 1 : 0;
      if ((r = run(&Q)) != 0) return r;
    }
  }
  return 0;
}

}  // namespace tclb
