// Native action loop: the n steps of an action in one C++ call, for every kind of
// lattice the runtime steps — one rank or many, slab or Y x Z process grid, with the
// stage kinds and per-step services of the reference's Lattice::Iterate.
//
// Reference: every MPI rank runs Lattice::Iterate in C++ (src/Lattice.cu.Rt:900-989):
// per stage RunBorder -> MPIStream_A -> RunInterior -> MPIStream_B (:466-533, 327-389),
// particle stages bracketed by CopyInParticles / CopyOutParticles and the RFI exchange
// (:392-437), fixed-point stages swept in place (:484), the zone index of the time series
// advanced per iteration (:473-477), the samplers filled after each iteration (:1376-1389).
//
// Per stage k of the action (StagePlan.mode):
//   0 plain      slab: the two border launches, whose stores of the exchanged fields
//                also land in one packed send buffer per direction (MirrorSpec ->
//                core.hpp mirror_store), then the halo exchange of the stage starts on the
//                transport (GPU: high-priority comm stream; ONE message per neighbour and
//                direction, then one copy launch unpacking the received buffers into the
//                ghost planes — a field's g planes are contiguous in the [field][z][y][x]
//                layout), then the interior launch concurrent with it; the compute stream
//                waits for the exchange only before the next stage.  Y x Z grid: the four
//                border boxes (the two z boxes mirrored), then the two-phase exchange (z
//                planes packed as above, then y rows over the ghost-inclusive z extent —
//                which also fills the edge ghosts — packed into the staging buffer), then
//                the interior box.  One rank without ghosts: one launch.
//   1 out of place  a stage that reads (through a stencil) a field it writes: launch into
//                the scratch snapshot, copy the saved fields back, exchange (the reference
//                runs it in place, an order-dependent race; tools/race_check.py).
//   2 fixed point   `sweeps` Jacobi sweeps of mode 1 (reference: 100 in-place sweeps).
// StagePlan.particle: zero the force accumulator and build the solid container before
// the stage, all-reduce / NaN-guard the forces after it and (SimplePart) integrate the
// rigid bodies — all on the device, no host round trip (services part_pre / part_post).
//
// Before each step the zonal time series write their active entries (and slopes) into the
// device zonal table (services series); after each step every sampler records a row.
//
// The halo plan (which bytes go to / come from which rank) is built once per action on
// the host (tclb_amd/parallel/native.py) as lists of HaloOp, SegOp, MirrorSpec and PackOp.
// Sends and receives between a pair of ranks are matched in issue order (NCCL semantics;
// tags are for transports that match by tag), which the plan keeps identical on every
// rank: [send up (fields read from below), to next] [send down (fields read from above),
// to prev] [receive from prev] [receive from next]
// (tests/test_distributed.py test_native_plan_pairs_by_issue_order).  The IPC transport
// has no messages: each rank pulls its neighbours' send buffers (SegOp dir 2 / 3) between
// counter waits (csrc/device/dist.hip xstart_ipc).
//
// The services object S supplies the device side (csrc/device/dist.hip GPU, csrc/runtime/
// dist_cpu.cpp OpenMP):
//   int run(Launch&)                               one stage launch (the model library)
//   int sample(Launch&, const SamplePlan&)         one sampler row
//   int copy_runs(void* dst, const void* src, const LoopPlan&, const StagePlan&)
//   int xstart(char* snap, const LoopPlan&, const StagePlan&, int mirrored)   start the
//                                                  exchange (mirrored: the send buffers
//                                                  are already filled by the borders)
//   int xfinish()                                  later launches wait for it
//   void* fork()                                   the comm stream, ordered after the work
//                                                  queued so far (overlap 2 borders)
//   int series(const LoopPlan&, int iter)          active series entries -> zonal table
//   int part_pre(Launch&, const LoopPlan&), part_post(Launch&, const LoopPlan&, int step)
#pragma once
#include "tclb/core.hpp"

namespace tclb {

struct HaloOp {
  long long off;    // byte offset from the output snapshot's base (buf 0) or staging (buf 1)
  long long bytes;  // message size
  int kind;         // 0 = send, 1 = receive
  int peer;         // rank in the communicator
  int tag;          // identical on both ends of a message (RCCL ignores it)
  int buf;          // 0 = snapshot, 1 = staging buffer (the grid's packed y rows)
};

// one packed block of the grid's y phase: fields [field0, field0 + nfield), rows
// [y0, y0 + ny) of planes [z0, z0 + nz) (snapshot coordinates, ghosts included), all px
// columns, to / from staging + boff laid out [field][z][y][x]
struct PackOp {
  long long boff;
  int field0, nfield;
  int y0, ny, z0, nz;
  int unpack;       // 0: snapshot -> staging (before the sends), 1: staging -> snapshot
  int reserved;
};

// one contiguous copy of the packed phase A (a field's g halo planes are contiguous in
// the [field][z][y][x] layout): dir 0 packs snapshot + src -> staging + dst (before the
// sends, when the border launches did not mirror their stores), dir 1 unpacks staging +
// src -> snapshot + dst (after the receives); IPC transport: dir 2 pulls a neighbour's
// packed send buffer (LoopPlan.peer_stg[peer] + src, mapped from the other process) into
// snapshot + dst, dir 3 into staging + dst (the grid's y rows, unpacked by PackOps)
struct SegOp {
  long long dst, src, bytes;
  int dir;
  int peer;
};

// the halo mirror of one border launch (core.hpp mirror_store): the stores of the fields
// with slot[f] >= 0 also land in staging + boff, packed [slot][g planes]
struct MirrorSpec {
  long long boff;
  long long mfs, msy, msz;
  int moy, moz;
  signed char slot[TCLB_MIRROR_FIELDS];
};

constexpr int DIST_MAX_STAGES = 32;

struct StagePlan {
  int stage;        // model stage index
  int mode;         // 0 plain, 1 out of place, 2 fixed point
  int sweeps;       // mode 2
  int particle;     // particle hooks around the stage
  int op0, nops;    // exchange ops of the stage (phase A, then phase B of a grid)
  int opb0, nopsb;
  int pk0, npk;     // pack ops (phase B)
  int run0, nruns;  // saved-field runs [runs[2i], runs[2i+1]) (copy-back of modes 1, 2)
  int seg0;         // phase A segments: npack packs, then nunpack unpacks / pulls
  int npack, nunpack;
  int mir_lo, mir_hi;  // MirrorSpec of the low / high border launch (-1: none)
  int yseg0, nyseg;    // IPC transport: the grid y phase's pulls (dir 3 segments)
  int mirror;          // 1: the border launches fill the send buffers (no pack segments);
                       // 0 for split stages, whose class-0 nodes store nothing
  int reserved;
};

struct SeriesEntry {
  int idx;          // zonal table slot of the value
  int dtidx;        // slot of its time derivative
  int len;          // series length (entry iter % len is active)
  int off;          // first value in svals / sslopes
};

// particle records of the device-resident particle system (tclb_amd/particles/system.py)
struct PartPlan {
  double* P;                 // [n][PART_STRIDE]
  double* acc;               // [n][6] force / moment accumulator
  const double* m;           // [n] masses
  const unsigned char* free_;  // [n] not fixed
  int n;
  int container;             // 0 none (every node scans every particle), 1 grid, 2 tree
  int* grid;                 // container buffer (Launch.ext[4])
  long long grid_n;          // its int32 elements
  int gdim[3], cell, ncell;  // grid container
  int nl;                    // tree: leaves (power of two)
  double mscale;             // tree: Morton quantisation scale
  void* tmp;                 // scratch of the container build (sort keys / values / temp)
  long long tmp_bytes;
  double a[3];               // SimplePart: constant acceleration
  double period[3];
  int periodic;              // bit d: periodic along axis d
  int integrate;             // 1: SimplePart rigid step after the stage (not in Init)
  int allreduce;             // 1: sum the accumulator over the ranks after the stage
  int nslots;                // accumulator copies (core.hpp particle_acc; GPU), summed after
  void* accbuf;              // IPC transport: this rank's shared copy of the accumulator
  const double* const* accs; // and every rank's, mapped (device array of nranks pointers)
};

struct LoopPlan {
  int axis;         // 0 one rank without ghosts, 1 y slab, 2 z slab, 3 Y x Z grid
  int n, g;         // slab: interior extent and ghost depth along the split axis
  int ny, nz, gy, gz;  // grid: interior extents and ghost depths
  int overlap;      // border / exchange / interior split (2: the border launches and the
                    // exchange on the comm stream, concurrent with the interior launch)
  int nstages;
  StagePlan st[DIST_MAX_STAGES];
  const HaloOp* ops;
  const PackOp* packs;
  const int* runs;
  const SegOp* segs;       // phase A segments (host)
  const SegOp* dsegs;      // the same on the device (GPU copy kernels)
  const MirrorSpec* mirrors;
  void* scratch;    // scratch snapshot (modes 1, 2)
  void* staging;    // staging buffer of the grid's y phase
  long long fs_bytes;  // bytes between field planes of a snapshot
  int nseries;
  int nsamplers;
  const SeriesEntry* series;
  const double* svals;     // series values (device)
  const double* sslopes;   // and slopes
  double* zonal;           // device zonal table (Launch.zonal)
  SamplePlan* samplers;    // host array of nsamplers plans (device buffers inside)
  PartPlan* part;          // null: no particles
  // IPC transport: the neighbours' staging buffers mapped into this process (peer 0 / 1:
  // below / above along the slab axis or the grid's z, 2 / 3: the grid's y) and their ranks
  const void* peer_stg[4];
  int ipc_peer[4];
};

typedef int (*run_fn)(const Launch*, int);
typedef int (*sample_fn)(const Launch*, int, const SamplePlan*);

inline void loop_set_range(Launch& L, int axis, int a, int b) {
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
inline int dist_self_pairs(char* base, char* staging, const HaloOp* ops, int nops, int self, Copy copy) {
  int si = 0;
  for (int r = 0; r < nops; r++) {
    if (ops[r].kind != 1 || ops[r].peer != self) continue;
    while (si < nops && !(ops[si].kind == 0 && ops[si].peer == self)) si++;
    if (si >= nops || ops[si].bytes != ops[r].bytes) return -3;
    char* d = (ops[r].buf ? staging : base) + ops[r].off;
    const char* s = (ops[si].buf ? staging : base) + ops[si].off;
    const int e = copy(d, s, ops[si].bytes);
    if (e != 0) return e;
    si++;
  }
  return 0;
}

// a border launch whose stores of the exchanged fields also land in the packed send
// buffer (MirrorSpec m of the plan; m < 0: a plain launch)
template <class S>
inline int loop_run_mirrored(S& sv, Launch& L, const LoopPlan& P, int m) {
  if (m < 0 || P.mirrors == nullptr) return sv.run(L);
  const MirrorSpec& M = P.mirrors[m];
  L.mbase = (char*)P.staging + M.boff;
  L.mfs = M.mfs, L.msy = M.msy, L.msz = M.msz, L.moy = M.moy, L.moz = M.moz;
  for (int i = 0; i < TCLB_MIRROR_FIELDS; i++) L.mslot[i] = M.slot[i];
  const int r = sv.run(L);
  L.mbase = nullptr;
  return r;
}

// one launch over the whole local box
template <class S>
inline int loop_full(S& sv, Launch& L, const LoopPlan& P, int nx) {
  L.xlo = 0;
  L.xhi = nx;
  if (P.axis == 3) {
    L.ylo = 0, L.yhi = P.ny, L.zlo = 0, L.zhi = P.nz;
  } else if (P.axis == 1 || P.axis == 2) {
    loop_set_range(L, P.axis, 0, P.n);
  }
  return sv.run(L);
}

// the border launches of a stage: on the compute stream before the interior (overlap 1),
// or on the comm stream (overlap 2) — forked after the work already queued, so they, the
// exchange that follows them and the interior launch run concurrently; the next stage
// waits for both (xfinish).  Returns the stream the interior launch goes to.
template <class S>
inline void* loop_borders_begin(S& sv, Launch& L, const LoopPlan& P) {
  void* ks = L.stream;
  if (P.overlap == 2) L.stream = sv.fork();
  return ks;
}

// launch + exchange of one stage in place (mode 0)
template <class S>
inline int loop_stage_plain(S& sv, Launch& L, const LoopPlan& P, const StagePlan& st, char* out, int nx) {
  int r;
  const bool xch = (st.nops + st.nopsb + st.nunpack) > 0;
  if (!xch) return loop_full(sv, L, P, nx);
  if (P.axis == 3) {
    const int ny = P.ny, nz = P.nz, gy = P.gy, gz = P.gz;
    if (P.overlap && ny > 2 * gy && nz > 2 * gz) {
      const int box[4][4] = {{0, ny, 0, gz}, {0, ny, nz - gz, nz}, {0, gy, gz, nz - gz}, {ny - gy, ny, gz, nz - gz}};
      const int mir[4] = {st.mir_lo, st.mir_hi, -1, -1};
      void* ks = loop_borders_begin(sv, L, P);
      for (int b = 0; b < 4; b++) {
        L.ylo = box[b][0], L.yhi = box[b][1], L.zlo = box[b][2], L.zhi = box[b][3];
        if ((r = loop_run_mirrored(sv, L, P, mir[b])) != 0) return r;
      }
      L.stream = ks;
      if ((r = sv.xstart(out, P, st, st.mirror)) != 0) return r;
      L.ylo = gy, L.yhi = ny - gy, L.zlo = gz, L.zhi = nz - gz;
      if ((r = sv.run(L)) != 0) return r;
      return sv.xfinish();
    }
    if ((r = loop_full(sv, L, P, nx)) != 0) return r;
    if ((r = sv.xstart(out, P, st, 0)) != 0) return r;
    return sv.xfinish();
  }
  const int n = P.n, g = P.g, ax = P.axis;
  if (P.overlap && n > 2 * g) {
    void* ks = loop_borders_begin(sv, L, P);
    loop_set_range(L, ax, 0, g);
    if ((r = loop_run_mirrored(sv, L, P, st.mir_lo)) != 0) return r;
    loop_set_range(L, ax, n - g, n);
    if ((r = loop_run_mirrored(sv, L, P, st.mir_hi)) != 0) return r;
    L.stream = ks;
    if ((r = sv.xstart(out, P, st, st.mirror)) != 0) return r;
    loop_set_range(L, ax, g, n - g);
    if ((r = sv.run(L)) != 0) return r;
    return sv.xfinish();
  }
  if ((r = loop_full(sv, L, P, nx)) != 0) return r;
  if ((r = sv.xstart(out, P, st, 0)) != 0) return r;
  return sv.xfinish();
}

// launch into the scratch snapshot, copy the saved fields back, exchange (modes 1, 2)
template <class S>
inline int loop_stage_oop(S& sv, Launch& L, const LoopPlan& P, const StagePlan& st, char* out, int nx) {
  int r;
  L.in = out;
  L.out = P.scratch;
  if ((r = loop_full(sv, L, P, nx)) != 0) return r;
  if ((r = sv.copy_runs(out, P.scratch, P, st)) != 0) return r;
  if (st.nops + st.nopsb + st.nunpack > 0) {
    if ((r = sv.xstart(out, P, st, 0)) != 0) return r;
    if ((r = sv.xfinish()) != 0) return r;
  }
  L.out = out;
  return 0;
}

// The loop.  L.in / L.out hold the current / other snapshot; nx = L.nx.  `init`: the
// action is Init (particles are not integrated after its particle stage, as the
// reference's Init does not advance the integrator).
template <class S>
inline int action_loop(S& sv, Launch L, int nsteps, int glob_last, const LoopPlan& P, int init) {
  const void* cur = L.in;
  void* nxt = L.out;
  const int gflags = L.glob & ~1;
  const int nx = L.nx;
  int r;
  for (int s = 0; s < nsteps; s++) {
    if (P.nseries > 0 && (r = sv.series(P, L.iter)) != 0) return r;
    for (int k = 0; k < P.nstages; k++) {
      const StagePlan& st = P.st[k];
      L.in = k == 0 ? cur : nxt;
      L.out = nxt;
      L.stage = st.stage;
      L.glob = (glob_last && s == nsteps - 1) ? (1 | gflags) : 0;
      const bool part = st.particle && P.part != nullptr;
      if (part && (r = sv.part_pre(L, P)) != 0) return r;
      if (st.mode == 0 || k == 0) {
        r = loop_stage_plain(sv, L, P, st, (char*)nxt, nx);
      } else {
        const int sweeps = st.mode == 2 ? st.sweeps : 1;
        r = 0;
        for (int w = 0; w < sweeps && r == 0; w++) r = loop_stage_oop(sv, L, P, st, (char*)nxt, nx);
      }
      if (r != 0) return r;
      if (part && (r = sv.part_post(L, P, !init)) != 0) return r;
    }
    L.xlo = 0, L.xhi = nx;
    if (P.axis == 3) {
      L.ylo = 0, L.yhi = P.ny, L.zlo = 0, L.zhi = P.nz;
    } else if (P.axis == 1 || P.axis == 2) {
      loop_set_range(L, P.axis, 0, P.n);
    }
    L.iter += 1;
    L.reserved1 += 1;
    void* t = (void*)cur;
    cur = nxt;
    nxt = t;
    for (int q = 0; q < P.nsamplers; q++) {
      const SamplePlan& sp = P.samplers[q];
      if (sp.np <= 0 || sp.row + s >= sp.rows) continue;
      Launch Q = L;
      Q.in = cur;
      Q.out = nxt;
      Q.glob = 0;
      Q.reserved1 = L.reserved1 > 2 ? L.reserved1 - 1 : 1;   // quantity averaging count
      SamplePlan Sp = sp;
      Sp.row = sp.row + s;
      if ((r = sv.sample(Q, Sp)) != 0) return r;
    }
  }
  return 0;
}

}  // namespace tclb
