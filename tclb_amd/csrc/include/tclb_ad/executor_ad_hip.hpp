// Adjoint (reverse) executor on the GPU (gfx950).  Same scheme as the CPU executor
// (csrc/include/tclb/executor_ad.hpp): every node update is re-run with dual numbers,
// the local Jacobian is contracted with the adjoint of the stage outputs and scattered to
// the adjoint of the loaded inputs with device fp64 atomics — the reference's adjoint
// push (src/LatticeAccess.inc.cpp.Rt:349-361, Tapenade Run_b kernels, src/Lattice.cu.Rt
// :542-613).
//
// GPU shape: a node reads up to TCLB_AD_K distinct inputs (populations, stencil fields,
// seeded settings), but carrying K tangents per value would put every value of the node
// code in scratch (K+1 doubles each).  Instead each thread re-runs its node in passes of
// TCLB_AD_WINDOW tangents: pass p seeds only the inputs whose first-read index falls in
// [p W, (p+1) W).  The first-read order is the same in every pass (identical primal
// values, identical branches), so the passes partition the Jacobian columns.
#pragma once
#include <hip/hip_runtime.h>
#include <utility>
#include "tclb/ad.hpp"

#ifndef TCLB_AD_WINDOW
// d3q19_adj 128^3 (profiles/r02o): W = 4 10.2 ms per adjoint step (268 B/lane of spills),
// W = 3 11.9 ms (no scratch), W = 2 14.3, W = 1 15.1; W = 5 spills 752 B/lane
#define TCLB_AD_WINDOW 4
#endif

namespace tclb {

// first-read keys of a thread's inputs live in LDS, interleaved across the 64 threads of
// a k_ad block (key j of thread t at [j * 64 + t]: conflict-free).  Kept in the node
// object, their runtime-indexed array would pin the whole node (populations, settings,
// the Launch fields it copies) in scratch: SROA cannot split an object that has a
// variable-offset access.
constexpr int AD_BLOCK = 64;
__device__ inline long long* ad_key_slot() {
  __shared__ long long keys[TCLB_AD_K * AD_BLOCK];
  return keys + threadIdx.x;
}

template <class T, int C>
struct AdRec<Dual<T, C>> {
  static constexpr int KMAX = TCLB_AD_K;
  typedef Dual<T, C> D;
  AdCtx* ctx;
  long long fs, zp;
  int n, base;
  long long* key;        // first-read order of the inputs: kind<<60 | field<<44 | index (LDS)
  TCLB_FN void init(const Launch& L) {
    key = ad_key_slot();
    ctx = (AdCtx*)L.ext[5];
    fs = L.fs;
    zp = L.nzones;
    n = 0;
    base = L.reserved2;
    for (int c = 0; c < C; c++) acc[c] = 0.0;
  }
  TCLB_FN static long long mk(int kind, int f, long long i) {
    return ((long long)kind << 60) | ((long long)f << 44) | i;
  }
  TCLB_FN D mark(double v, int j) const {
    D r(v);
    for (int c = 0; c < C; c++) r.d[c] = (j - base == c) ? T(1) : T(0);   // no runtime index
    return r;
  }
  TCLB_FN int find(long long k) const {
    for (int j = 0; j < n; j++)
      if (key[j * AD_BLOCK] == k) return j;
    return -1;
  }
  TCLB_FN D seed(double v, long long k) {
    const int j = find(k);
    if (j >= 0) return mark(v, j);
    if (n < KMAX) {
      key[n * AD_BLOCK] = k;
      return mark(v, n++);
    }
    ctx->overflow = 1;
    return D(v);
  }
  TCLB_FN D load(double v, int f, long long i) { return ctx ? seed(v, mk(0, f, i)) : D(v); }
  TCLB_FN D setting(int i, D v) {
    return (ctx && ctx->set_mask && ctx->set_mask[i]) ? seed(v.v, mk(1, i, 0)) : v;
  }
  TCLB_FN D zonal(int i, int zone, D v) {
    return (ctx && ctx->zon_mask && ctx->zon_mask[i]) ? seed(v.v, mk(2, i, zone)) : v;
  }
  // the stage outputs' adjoints are contracted with this pass's tangents in registers
  // (acc[c] = sum over stores of aout * d out / d input_(base+c)) and pushed with one
  // atomic per input at the end of the pass (flush), instead of one atomic per
  // (output, input) pair of the local Jacobian
  double acc[C];
  TCLB_FN void scatter(double a, const D& val) {
    if (a == 0.0) return;
    for (int c = 0; c < C; c++) acc[c] += a * (double)val.d[c];
  }
  TCLB_FN void flush() {
    for (int c = 0; c < C; c++) {
      const int j = base + c;
      const double d = acc[c];
      acc[c] = 0.0;
      if (j >= n || d == 0.0) continue;
      const long long k = key[j * AD_BLOCK];
      const int kind = (int)(k >> 60), f = (int)((k >> 44) & 0xffff);
      const long long i = k & ((1LL << 44) - 1);
      double* dst = kind == 0 ? ctx->ain + (long long)f * fs + i
                              : (kind == 1 ? ctx->gset + f : ctx->gzon + (long long)f * zp + i);
      unsafeAtomicAdd(dst, d);
    }
  }
  TCLB_FN void store(int f, long long node, const D& val) {
    if (ctx) scatter(ctx->aout[(long long)f * fs + node], val);
  }
};

namespace exec {

// One launch per tangent window (L.reserved2 = first input of the window, set by the
// host loop in ad_hip_impl).  Passes as separate launches rather than a loop in the
// kernel: inside one kernel the compiler keeps the primal values of every pass live
// and the d3q19_adj node spills 636 B/lane at W = 3; one pass per launch needs no
// scratch at W = 3 (268 B/lane of spills at the default W = 4).  Every node runs the
// passes of the launch; after the first call of a stage the host covers only the
// largest input count seen (adjoint.py), not all K.
//
// Models with hand-written reverse sweeps (Model.set_reverse) split the work by launch
// mode (Launch.next[5]) so a wave never mixes the two kinds of node (a 64-wide x row
// holding one boundary node would otherwise run the whole dual pass):
//   0  dual passes over the launch box (no reverse sweeps);
//   1  reverse sweeps over the box (kernel k_rev, its own register budget: the dual
//      path's would cut its occupancy to one wave); the nodes without one are appended to
//      the dual-node list in Launch.aux (int: [0] count, then box-linear node indices),
//      recorded while Launch.qcomp == 0 (the first call of a stage);
//   2  dual passes over the Launch.qcomp listed nodes, every window in one launch
//      (grid.y = window: a few boundary planes of nodes alone cannot fill the GPU).
// (aux / qcomp are the quantity-launch fields, unused by stage launches.)
template <class Model, int STG>
__global__ void __launch_bounds__(256) k_rev(const Launch L) {
  constexpr int NG = Model::NGLOBALS_;
  const int x = L.xlo + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int y = L.ylo + (int)(blockIdx.y * blockDim.y + threadIdx.y);
  const int z = L.zlo + (int)blockIdx.z;
  if (x >= L.xhi || y >= L.yhi) return;
  if constexpr (has_rev<typename Model::template NodeT<double, double, true>>::value) {
    AdCtx* ctx = (AdCtx*)L.ext[5];
    double gd[NG > 0 ? NG : 1];
    for (int i = 0; i < NG; i++) gd[i] = 0.0;
    typename Model::template NodeT<double, double, true> nr(L, x, y, z, gd);
    if (nr.template rev_ok<STG>()) {
      nr.template rev_stage<STG>(*ctx);
    } else if (L.qcomp == 0) {
      const int w = L.xhi - L.xlo, h = L.yhi - L.ylo;
      int* list = (int*)L.aux;
      const int k = atomicAdd(list, 1);
      list[1 + k] = (x - L.xlo) + w * ((y - L.ylo) + h * (z - L.zlo));
    }
  }
}

// occupancy floor of k_ad (diagnostic build variants, -DTCLB_AD_WAVES=W): W = 2 keeps the
// kernel within 256 registers (no AGPRs: spills go to scratch instead)
#ifndef TCLB_AD_WAVES
#define TCLB_AD_WAVES 0
#endif
template <class Model, int STG>
#if TCLB_AD_WAVES > 0
__global__ void __launch_bounds__(AD_BLOCK) __attribute__((amdgpu_waves_per_eu(TCLB_AD_WAVES)))
#else
__global__ void __launch_bounds__(AD_BLOCK)
#endif
k_ad(const Launch L) {
  typedef Dual<double, TCLB_AD_WINDOW> D;
  constexpr int NG = Model::NGLOBALS_;
  constexpr int NSUM = Model::NSUMGLOBALS_;
  const int mode = (int)L.next[5];
  const int w = L.xhi - L.xlo, h = L.yhi - L.ylo;
  int x, y, z;
  bool active;
  if (mode == 2) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    active = i < L.qcomp;
    const int lin = active ? ((const int*)L.aux)[1 + i] : 0;
    x = L.xlo + lin % w;
    y = L.ylo + (lin / w) % h;
    z = L.zlo + lin / (w * h);
  } else {
    x = L.xlo + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    y = L.ylo + (int)blockIdx.y;
    z = L.zlo + (int)blockIdx.z;
    active = x < L.xhi;
  }
  AdCtx* ctx = (AdCtx*)L.ext[5];
  // mode 2: window of this block row (no setting is seeded in mode 2, so the window base
  // can be set after the node constructor, before its loads seed the inputs)
  const int wbase = mode == 2 ? L.reserved2 + (int)blockIdx.y * TCLB_AD_WINDOW : L.reserved2;
  int n = 0;
  if (active) {
    D g[NG];
    for (int i = 0; i < NG; i++) g[i] = i < NSUM ? D(0.0) : D(-1e30);
    typename Model::template NodeT<D, double, true> nd(L, x, y, z, g);
    nd.ad_.base = wbase;
    nd.template run_stage<STG>();
    if (ctx->obj_weight != 0.0) nd.ad_.scatter(ctx->obj_weight, g[Model::OBJ_]);
    nd.ad_.flush();
    n = nd.ad_.n;
  }
  // first pass: the largest input count of the launch (ctx->reserved), from which the
  // host sizes the passes of later calls of this stage (AdCtx.reserved, adjoint.py)
  if (wbase == 0) {
    for (int off = AD_BLOCK / 2; off > 0; off >>= 1) n = max(n, __shfl_xor(n, off));
    if (threadIdx.x == 0 && n > 0) atomicMax(&ctx->reserved, n);
  }
}

template <class Model, int... I>
inline int ad_hip_impl(const Launch& L, std::integer_sequence<int, I...>) {
  const int w = L.xhi - L.xlo, h = L.yhi - L.ylo, d = L.zhi - L.zlo;
  if (w <= 0 || h <= 0 || d <= 0) return 0;
  const int mode = (int)L.next[5];
  dim3 grid((w + AD_BLOCK - 1) / AD_BLOCK, h, d);
  const dim3 block(AD_BLOCK, 1, 1);
  hipStream_t s = (hipStream_t)L.stream;
  // windows [L.reserved2, L.reserved0) of the input list (reserved0 = 0: all TCLB_AD_K)
  const int end = (L.reserved0 > 0 && L.reserved0 < TCLB_AD_K) ? L.reserved0 : TCLB_AD_K;
  if (mode == 1) {            // reverse sweeps: one launch, stage-kernel block shape
    const int bx = w >= 128 ? 128 : 64, by = 256 / bx;
    const dim3 rgrid((w + bx - 1) / bx, (h + by - 1) / by, d), rblock(bx, by, 1);
    bool found = false;
    ((L.stage == I ? (k_rev<Model, I><<<rgrid, rblock, 0, s>>>(L), found = true) : false), ...);
    return found ? (int)hipGetLastError() : -2;
  }
  if (mode == 2) {            // listed nodes, every window in one launch
    if (L.qcomp <= 0) return 0;
    const int nwin = (end - L.reserved2 + TCLB_AD_WINDOW - 1) / TCLB_AD_WINDOW;
    if (nwin <= 0) return 0;
    grid = dim3((L.qcomp + AD_BLOCK - 1) / AD_BLOCK, nwin, 1);
    bool found = false;
    ((L.stage == I ? (k_ad<Model, I><<<grid, block, 0, s>>>(L), found = true) : false), ...);
    return found ? (int)hipGetLastError() : -2;
  }
  for (int base = L.reserved2; base < end; base += TCLB_AD_WINDOW) {
    Launch Lb = L;
    Lb.reserved2 = base;
    bool found = false;
    ((L.stage == I ? (k_ad<Model, I><<<grid, block, 0, s>>>(Lb), found = true) : false), ...);
    if (!found) return -2;
  }
  return (int)hipGetLastError();
}

}  // namespace exec
}  // namespace tclb

// ctx: device copy of the AdCtx (aout/ain/gset/gzon/masks are device pointers)
#define TCLB_EXPORT_AD_HIP(NAME, MODEL)                                                      \
  extern "C" int tclb_##NAME##_adjoint(const tclb::Launch* L) {                              \
    return tclb::exec::ad_hip_impl<MODEL>(*L, std::make_integer_sequence<int, MODEL::NSTAGES_>{}); \
  }                                                                                          \
  extern "C" int tclb_##NAME##_ad_tangents() { return TCLB_AD_K; }                           \
  extern "C" int tclb_##NAME##_ad_window() { return TCLB_AD_WINDOW; }                        \
  extern "C" int tclb_##NAME##_ad_device() { return 1; }                                     \
  extern "C" int tclb_##NAME##_sizeof_launch() { return (int)sizeof(tclb::Launch); }
