// Native multi-rank iteration loop (one rank = one GPU, or one CPU process in tests).
//
// Reference: every MPI rank runs Lattice::Iterate in C++ — border kernel, MPIStream_A
// (device->host copy of the margins), interior kernel, MPIStream_B (MPI Isend/Irecv,
// host->device copy into the next snapshot's margin blocks) — src/Lattice.cu.Rt:466-533,
// 900-989, 327-389, 439-456.
//
// Here the n steps of an action run in one native call for a slab-decomposed lattice:
//   1. the two border launches (planes [0,g) and [n-g,n) of the split axis);
//   2. the transport starts the halo exchange of the stage's saved fields — on the GPU an
//      event on the compute stream, then on the (high-priority) comm stream a grouped
//      ncclSend of each field's border planes STRAIGHT FROM the output snapshot and an
//      ncclRecv of each field's ghost planes STRAIGHT INTO the output snapshot (a field's
//      planes are contiguous in the [field][z][y][x] layout, so there is no pack or
//      unpack kernel and no staging buffer);
//   3. the interior launch [g, n-g) on the compute stream, concurrent with the exchange;
//   4. the compute stream waits for the exchange before the next stage / step.
// The halo plan (which bytes go to / come from which rank) is built once per action on
// the host (tclb_amd/parallel/native.py) as a list of HaloOp.  Sends and receives between
// a pair of ranks are matched in issue order (NCCL semantics; tags are for transports that
// match by tag), which the plan keeps identical on every rank: [sends of fields read from
// below, to next] [sends of fields read from above, to prev] [receives from prev]
// [receives from next], fields ascending.
#pragma once
#include "tclb/core.hpp"

namespace tclb {

struct HaloOp {
  long long off;    // byte offset from the output snapshot's base
  long long bytes;  // message size
  int kind;         // 0 = send, 1 = receive
  int peer;         // rank in the communicator
  int tag;          // identical on both ends of a message (RCCL ignores it)
  int reserved;
};

constexpr int DIST_MAX_STAGES = 32;

struct DistPlan {
  int axis;         // 1 = y slab (2-D lattices: a row of a field is contiguous), 2 = z slab
  int n, g;         // interior extent along the split axis, ghost depth
  int overlap;      // border / exchange / interior split (else: whole box, then exchange)
  int nstages;
  int stage[DIST_MAX_STAGES];
  int op0[DIST_MAX_STAGES];    // first op of stage k in ops[]
  int nops[DIST_MAX_STAGES];   // 0: the stage saves no halo field, no exchange
  const HaloOp* ops;
};

typedef int (*run_fn)(const Launch*, int);
typedef int (*sample_fn)(const Launch*, int, const SamplePlan*);

inline void dist_set_range(Launch& L, int axis, int a, int b) {
  if (axis == 2) {
    L.zlo = a;
    L.zhi = b;
  } else {
    L.ylo = a;
    L.yhi = b;
  }
}

// In-order matching of the plan's sends and receives addressed to this rank itself (the
// loopback transports): the k-th receive from `self` gets the k-th send to `self`.
// Calls copy(dst, src, bytes) per pair; returns -3 when the plan does not pair up.
template <class Copy>
inline int dist_self_pairs(char* base, const HaloOp* ops, int nops, int self, Copy copy) {
  int si = 0;
  for (int r = 0; r < nops; r++) {
    if (ops[r].kind != 1 || ops[r].peer != self) continue;
    while (si < nops && !(ops[si].kind == 0 && ops[si].peer == self)) si++;
    if (si >= nops || ops[si].bytes != ops[r].bytes) return -3;
    const int e = copy(base + ops[r].off, base + ops[si].off, ops[si].bytes);
    if (e != 0) return e;
    si++;
  }
  return 0;
}

// The loop.  X is the transport: int start(char* base, const HaloOp*, int) begins the
// exchange of one stage's halo (ordered after the launches already issued), int finish()
// makes later launches wait for it.  L.in / L.out hold the current / other snapshot.
template <class X>
inline int dist_iterate(Launch L, int prec, int nsteps, int glob_last, const DistPlan& P, X& x, run_fn run,
                        sample_fn sample, const SamplePlan* sp) {
  const void* cur = L.in;
  void* nxt = L.out;
  const int gflags = L.glob & ~1;
  const int n = P.n, g = P.g, ax = P.axis;
  int r;
  for (int s = 0; s < nsteps; s++) {
    for (int k = 0; k < P.nstages; k++) {
      L.in = k == 0 ? cur : nxt;
      L.out = nxt;
      L.stage = P.stage[k];
      L.glob = (glob_last && s == nsteps - 1) ? (1 | gflags) : 0;
      const HaloOp* ops = P.ops + P.op0[k];
      const int no = P.nops[k];
      if (no == 0) {
        dist_set_range(L, ax, 0, n);
        if ((r = run(&L, prec)) != 0) return r;
      } else if (P.overlap && n > 2 * g) {
        dist_set_range(L, ax, 0, g);
        if ((r = run(&L, prec)) != 0) return r;
        dist_set_range(L, ax, n - g, n);
        if ((r = run(&L, prec)) != 0) return r;
        if ((r = x.start((char*)nxt, ops, no)) != 0) return r;
        dist_set_range(L, ax, g, n - g);
        if ((r = run(&L, prec)) != 0) return r;
        if ((r = x.finish()) != 0) return r;
      } else {
        dist_set_range(L, ax, 0, n);
        if ((r = run(&L, prec)) != 0) return r;
        if ((r = x.start((char*)nxt, ops, no)) != 0) return r;
        if ((r = x.finish()) != 0) return r;
      }
    }
    dist_set_range(L, ax, 0, n);
    L.iter += 1;
    L.reserved1 += 1;
    void* t = (void*)cur;
    cur = nxt;
    nxt = t;
    if (sp != nullptr && sample != nullptr && sp->np > 0 && sp->row + s < sp->rows) {
      Launch Q = L;
      Q.in = cur;
      Q.out = nxt;
      Q.glob = 0;
      Q.reserved1 = L.reserved1 > 2 ? L.reserved1 - 1 : 1;   // quantity averaging count
      SamplePlan Sp = *sp;
      Sp.row = sp->row + s;
      if ((r = sample(&Q, prec, &Sp)) != 0) return r;
    }
  }
  return 0;
}

}  // namespace tclb
