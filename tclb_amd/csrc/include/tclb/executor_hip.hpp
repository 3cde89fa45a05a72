// GPU executor for gfx950 (MI355X): one thread per lattice node, wave64 rows.
//
// Replaces the reference's Kernel<InteriorExecutor/BorderExecutor> (reference:
// src/LatticeContainer.inc.cpp.Rt:201-287; block 32x4 with WARPSIZE=32 even on HIP)
// with CDNA4-shaped launches: blocks are (BX x BY) with BX a multiple of 64 so that
// every wavefront covers 64 consecutive x-nodes (one fully coalesced 512 B fp64 row
// segment per population); the border/interior split is expressed by the caller as a
// z- (or y-) range of the same kernel so it can run on separate HIP streams.
// Globals are reduced wave64 -> LDS -> one atomic per block and global
// (reference: per-warp(32) reduce + atomics, src/cuda.cu.Rt:93-179).
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <mutex>
#include <utility>
#include <vector>
#include "core.hpp"

namespace tclb {
namespace exec {

template <class R>
__device__ __forceinline__ R wave_sum(R v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <class R>
__device__ __forceinline__ R wave_max(R v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    R w = __shfl_xor(v, o, 64);
    v = v > w ? v : w;
  }
  return v;
}

__device__ __forceinline__ void atomic_max_double(double* addr, double v) {
  unsigned long long* a = (unsigned long long*)addr;
  unsigned long long old = __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (__longlong_as_double(old) < v) {
    unsigned long long assumed = old;
    old = atomicCAS(a, assumed, (unsigned long long)__double_as_longlong(v));
    if (old == assumed) break;
  }
}

// Globals of a block: the nodes add into the block-shared LDS accumulators acc[NG]
// (core.hpp glob_add/glob_max: a wave reduction and one LDS atomic per AddTo call), then
// after the barrier thread i adds acc[i] into slot (block % TCLB_GSLOTS) of dst (device,
// double; core.hpp TCLB_GSLOTS): one atomic per block and global, spread over 64 addresses
// per global (with every block adding into the same 8 bytes the L2 serialises ~10^5-10^6
// atomics per global and launch; profiles/README.md r03).  The accumulators are not
// per-thread registers, so the GLOB instantiation needs about the VGPRs of the plain one.
#ifndef TCLB_GLOB_LDS
#define TCLB_GLOB_LDS 1
#endif
// build variant "gregs" (TCLB_GLOB_LDS=0): the previous scheme, per-thread accumulators
// g[NG] kept in registers through the node and reduced wave64 -> LDS at the end
template <int NG, int NSUM, class R>
__device__ __forceinline__ void block_globals_regs(R* g, double* dst) {
  __shared__ double part[NG][16];
  const int tid = threadIdx.x + blockDim.x * threadIdx.y;
  const int lane = tid & 63, wid = tid >> 6;
  const int nw = (blockDim.x * blockDim.y + 63) >> 6;
#pragma unroll
  for (int i = 0; i < NG; i++) {
    R v = i < NSUM ? wave_sum(g[i]) : wave_max(g[i]);
    if (lane == 0) part[i][wid] = (double)v;
  }
  __syncthreads();
  if (tid < NG) {
    const unsigned b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    dst += (b % TCLB_GSLOTS) * (unsigned)gstride(NG);
    double acc = part[tid][0];
    for (int w = 1; w < nw; w++) acc = tid < NSUM ? acc + part[tid][w] : (acc > part[tid][w] ? acc : part[tid][w]);
    if (tid < NSUM) {
      if (acc != 0.0) unsafeAtomicAdd(dst + tid, acc);
    } else {
      atomic_max_double(dst + tid, acc);
    }
  }
}

template <int NG, int NSUM, class R>
__device__ __forceinline__ void block_globals_init(R* acc) {
  const int tid = threadIdx.x + blockDim.x * threadIdx.y;
  const int nt = blockDim.x * blockDim.y;
  for (int i = tid; i < NG; i += nt) acc[i] = i < NSUM ? R(0) : R(-1e30);
  __syncthreads();
}
template <int NG, int NSUM, class R>
__device__ __forceinline__ void block_globals_flush(const R* acc, double* dst) {
  __syncthreads();
  const int tid = threadIdx.x + blockDim.x * threadIdx.y;
  const int nt = blockDim.x * blockDim.y;
  const unsigned b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  dst += (b % TCLB_GSLOTS) * (unsigned)gstride(NG);
  for (int i = tid; i < NG; i += nt) {
    const double a = (double)acc[i];
    if (i < NSUM) {
      if (a != 0.0) unsafeAtomicAdd(dst + i, a);
    } else {
      atomic_max_double(dst + i, a);
    }
  }
}

// Block -> tile map.  The hardware deals work-groups round-robin over the 8 XCDs (b and
// b+8 share an L2; MI355X_MICROARCH.md, Workgroup dispatch) and in linear order in time,
// so with the identity map every resident wave of the chip works in ONE narrow window of
// the lattice: 27 read + 27 written field planes, each 2^k bytes apart, hit the HBM
// channels and banks at the same offsets at once, and the speed of a dispatch then depends
// on where the snapshot pages landed (tools/direction_probe.py: 9.5-11.8 ms per d3q27
// fp64 512^3 step from one allocation to the next, the same kernel).  With
// L.tile_split = k > 0 the linear block id b is remapped so that block b works in window
// (b mod 2^k), one of 2^k contiguous tile ranges (z-ranges): 2^k x 54 streams spread over
// the lattice, and with 2^k = 8 each XCD owns one window, so x-neighbouring tiles (which
// share the partial 128-B lines of the x-shifted pulls) and y/z neighbours of stencil
// stages meet in the same L2.  Speed only: any map gives the same result.
__device__ __forceinline__ unsigned tile_linear(const Launch& L, unsigned b, unsigned T) {
  const unsigned k = (unsigned)L.tile_split;
  if (k > 0u && k < 16u && (T & ((1u << k) - 1u)) == 0u) b = (b & ((1u << k) - 1u)) * (T >> k) + (b >> k);
  return b;
}
__device__ __forceinline__ uint3 tile_id(const Launch& L) {
  const unsigned gx = gridDim.x, gy = gridDim.y;
  if (L.tile_split <= 0) return make_uint3(blockIdx.x, blockIdx.y, blockIdx.z);
  const unsigned b = tile_linear(L, blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
  return make_uint3(b % gx, (b / gx) % gy, b / (gx * gy));
}

// CLS: node class of a split stage (DSL add_stage(split=True), Node::node_class_): 1 / 2
// run only the nodes of that class, each kernel compiled with that class's path alone;
// 0 = every node (the stages that are not split)
// Deferring split stages: the node list of the CLS 3 pass, dq = [count][node ids] (id: the
// node's linear index in the launch box).  The lanes of a wave that deferred reserve their
// slots with one atomic (ballot + prefix count).
__device__ __forceinline__ void defer_record(unsigned* dq, bool d, unsigned id) {
  const unsigned long long m = __ballot(d);
  if (m == 0ull) return;
  const int lane = __lane_id();
  const int leader = __ffsll((long long)m) - 1;
  unsigned base = 0;
  if (lane == leader) base = atomicAdd(dq, (unsigned)__popcll(m));
  base = __shfl(base, leader, 64);
  if (d) dq[1 + base + (unsigned)__popcll(m & ((1ull << lane) - 1ull))] = id;
}
__device__ __forceinline__ unsigned box_id(const Launch& L, int x, int y, int z) {
  return ((unsigned)(z - L.zlo) * (unsigned)(L.yhi - L.ylo) + (unsigned)(y - L.ylo)) * (unsigned)(L.xhi - L.xlo) +
         (unsigned)(x - L.xlo);
}
// dq (class-1 kernels of a deferring stage, k_stage_defer): where the nodes handed to the
// CLS 3 pass (Node::defer_heavy) are recorded
template <class Model, class R, class S, int STG, bool GLOB, int CLS = 0>
__device__ __forceinline__ void stage_tile(const Launch& L, const uint3 t, unsigned* dq = nullptr) {
  typedef typename Model::template NodeCls<R, S, GLOB, CLS> N;
  typedef typename N::G_ G;   // fp64 accumulators, also in fp32-compute builds (core.hpp glob_acc)
  const int x = L.xlo + (int)(t.x * blockDim.x + threadIdx.x);
  // blockDim.x is a multiple of 64 (launch_shape), so a wave covers 64 x of one row:
  // y is wave-uniform.  In the row-form instantiations (N::ROWA_, the globals kernels)
  // readfirstlane tells the compiler, which then keeps the row bases of every field in
  // SGPRs (core.hpp row_at); the flat-form plain kernels leave y in VGPRs, the form that
  // measured fastest on the headline (profiles/README.md r04c).  -DTCLB_UNIFORM_Y=0: never.
#ifndef TCLB_UNIFORM_Y
#define TCLB_UNIFORM_Y 1
#endif
  const int y0 = L.ylo + (int)(t.y * blockDim.y + threadIdx.y);
  const int y = (TCLB_UNIFORM_Y && N::ROWA_) ? __builtin_amdgcn_readfirstlane(y0) : y0;
  const int z = L.zlo + (int)t.z;
  if constexpr (GLOB && !TCLB_GLOB_LDS) {
    constexpr int NG = Model::NGLOBALS_ > 0 ? Model::NGLOBALS_ : 1;
    G g[NG];
#pragma unroll
    for (int i = 0; i < NG; i++) g[i] = i < Model::NSUMGLOBALS_ ? G(0) : G(-1e30);
    if (x < L.xhi && y < L.yhi) {
      N n(L, x, y, z, g);
      n.template run_stage<STG>();
      if constexpr (CLS == 1 && Model::defer_stage(STG)) {
        if (dq) defer_record(dq, n.deferred_, box_id(L, x, y, z));
      }
    }
    block_globals_regs<NG, Model::NSUMGLOBALS_>(g, L.globals);
  } else if constexpr (GLOB) {
    constexpr int NG = Model::NGLOBALS_ > 0 ? Model::NGLOBALS_ : 1;
    __shared__ G acc[NG];
    block_globals_init<NG, Model::NSUMGLOBALS_>(acc);
    if (x < L.xhi && y < L.yhi) {
      N n(L, x, y, z, acc);
      n.template run_stage<STG>();
      if constexpr (CLS == 1 && Model::defer_stage(STG)) {
        if (dq) defer_record(dq, n.deferred_, box_id(L, x, y, z));
      }
    }
    block_globals_flush<NG, Model::NSUMGLOBALS_>(acc, L.globals);
  } else {
    G g[1] = {G(0)};
    if (x < L.xhi && y < L.yhi) {
      N n(L, x, y, z, g);
      n.template run_stage<STG>();
      if constexpr (CLS == 1 && Model::defer_stage(STG)) {
        if (dq) defer_record(dq, n.deferred_, box_id(L, x, y, z));
      }
    }
  }
}
template <class Model, class R, class S, int STG, bool GLOB, int CLS = 0>
__device__ __forceinline__ void stage_body(const Launch& L) {
  stage_tile<Model, R, S, STG, GLOB, CLS>(L, tile_id(L));
}
// a launch over a list of tiles (linear ids of the stage's tile grid, gx x gy x depth)
__device__ __forceinline__ uint3 list_tile(const Launch& L, const unsigned* list, unsigned n, unsigned gx,
                                           unsigned gy) {
  const unsigned i = tile_linear(L, blockIdx.x, n);
  const unsigned b = list ? list[i] : i;   // no list: every tile
  return make_uint3(b % gx, (b / gx) % gy, b / (gx * gy));
}

// Occupancy floor of every stage kernel (build variant "sw2", -DTCLB_STAGE_WAVES=W): a
// kernel just past 256 VGPRs runs at 1 wave/SIMD; the cap trades that for spills (A/B of
// the register-heavy collisions, e.g. the tePSM CHT collide).  0 = no cap (default).
#ifndef TCLB_STAGE_WAVES
#define TCLB_STAGE_WAVES 0
#endif
template <class Model, class R, class S, int STG, bool GLOB, int CLS = 0>
#if TCLB_STAGE_WAVES > 0
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TCLB_STAGE_WAVES)))
#else
__global__ void __launch_bounds__(256)
#endif
k_stage(const Launch L) {
  stage_body<Model, R, S, STG, GLOB, CLS>(L);
}

// Narrow-storage occupancy floor (build variant, -DTCLB_NARROW_WAVES=N): with fp32/fp16
// storage each load moves half (a quarter) of the bytes, so a register-heavy kernel that
// keeps HBM busy at 2 waves/SIMD in fp64 needs more waves in flight (Little's law);
// amdgpu_waves_per_eu caps the VGPRs of the narrow-storage instantiations only.
#ifdef TCLB_NARROW_WAVES
template <class Model, class R, class S, int STG, bool GLOB>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TCLB_NARROW_WAVES)))
k_stage_narrow(const Launch L) {
  stage_body<Model, R, S, STG, GLOB>(L);
}
#endif

// Occupancy floor of the globals-integrating instantiations: the GLOB=true kernel keeps
// the globals accumulators live through the whole node, which can push it past 256 VGPRs
// into 1 wave/SIMD (pf_velocity mixed-shift: 266 VGPRs, 2.3x the plain step;
// profiles/README.md r03j/r03k).  amdgpu_waves_per_eu(W) caps it, W = the model's
// GLOB_WAVES_ (DSL Model.glob_waves; 0 = no cap, for kernels far above 256 VGPRs where a
// cap would spill heavily); -DTCLB_GLOB_WAVES=W overrides it for A/B builds.
#ifndef TCLB_GLOB_WAVES
#define TCLB_GLOB_WAVES -1
#endif
template <class Model>
constexpr int glob_waves() { return TCLB_GLOB_WAVES >= 0 ? TCLB_GLOB_WAVES : Model::GLOB_WAVES_; }

template <class Model, class R, class S, int STG, int W, int CLS = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W))) k_stage_glob(const Launch L) {
  stage_body<Model, R, S, STG, true, CLS>(L);
}

// Occupancy floor of the class-1 kernel of a split stage (A/B knob, build variant flag
// -DTCLB_SPLIT_WAVES=n; 0 = none)
#ifndef TCLB_SPLIT_WAVES
#define TCLB_SPLIT_WAVES 0
#endif
// A/B of the split itself (build variant nosplit): the stage as one kernel over all nodes
#ifndef TCLB_NO_SPLIT
#define TCLB_NO_SPLIT 0
#endif
template <class Model, class R, class S, int STG, bool GLOB, int W, int CLS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W))) k_stage_w(const Launch L) {
  stage_body<Model, R, S, STG, GLOB, CLS>(L);
}

// ---------------------------------------------------------------- class tile lists
// A split stage runs one kernel per node class over the whole tile grid, each node skipping
// the other class; the kernel of a class that holds no node of a tile still dispatches its
// waves, at about 1 ns per wave for the chip: 1.07 ms of the 7.7 ms pf384 mixed-shift step
// for a class-2 kernel with no class-2 node at all (profiles/README.md r05l).  So the
// classes present in each tile are found once per node-type identity and launch geometry
// (k_classify, Launch.flags_gen), and each class kernel runs over the list of its tiles
// only (none: no launch; every tile: the plain grid).
template <class Model, class R, class S, int STG>
__global__ void __launch_bounds__(256) k_classify(const Launch L, unsigned char* out) {
  typedef typename Model::template NodeCls<R, S, false, 1> N;
  __shared__ int bits;
  if (threadIdx.x == 0 && threadIdx.y == 0) bits = 0;
  __syncthreads();
  const int x = L.xlo + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int y = L.ylo + (int)(blockIdx.y * blockDim.y + threadIdx.y);
  const int z = L.zlo + (int)blockIdx.z;
  if (x < L.xhi && y < L.yhi) {
    typename N::G_ g[1];
    N n(L, x, y, z, g);
    atomicOr(&bits, 1 << n.node_class_(STG));   // class 0: no work in this stage
  }
  __syncthreads();
  if (threadIdx.x == 0 && threadIdx.y == 0) out[blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)] = (unsigned char)bits;
}

struct ClassTiles {
  const void* flags;
  int gen;
  int box[6];
  unsigned bx, by;
  unsigned* list;   // device: the class-1 tiles, then the class-2 tiles
  unsigned* dq;     // deferring stages: [count][class-1 nodes handed to the CLS 3 kernel]
  unsigned n1, n2, total;
  unsigned long long used;
};

// the tile lists of this launch's geometry, built on first use (one synchronising classify
// pass), copied out under the lock (the cache may grow or evict behind a caller's back);
// false if that failed (the caller then runs both classes over the full grid).  An
// evicted entry's list is released with hipFree, which waits for the device.
// Node::node_class_(stage): 1, 2, or 0 for a node the stage leaves alone (on no list)
template <class Model, class R, class S, int STG>
inline bool class_tiles(const Launch& L, dim3 grid, dim3 block, hipStream_t s, ClassTiles& out) {
  static std::vector<ClassTiles> cache;
  static std::mutex mu;
  static unsigned long long clock = 0;
  std::lock_guard<std::mutex> lk(mu);
  const int box[6] = {L.xlo, L.xhi, L.ylo, L.yhi, L.zlo, L.zhi};
  for (auto& c : cache) {
    if (c.flags == L.flags && c.gen == L.flags_gen && c.bx == block.x && c.by == block.y &&
        std::equal(box, box + 6, c.box)) {
      c.used = ++clock;
      out = c;
      return true;
    }
  }
  // entries of an older identity of these node types are stale; keep at most 32 others
  for (size_t i = 0; i < cache.size();) {
    if (cache[i].flags == L.flags && cache[i].gen != L.flags_gen) {
      hipFree(cache[i].list);
      hipFree(cache[i].dq);
      cache.erase(cache.begin() + (long)i);
    } else {
      i++;
    }
  }
  if (cache.size() >= 32) {
    size_t o = 0;
    for (size_t i = 1; i < cache.size(); i++)
      if (cache[i].used < cache[o].used) o = i;
    hipFree(cache[o].list);
    hipFree(cache[o].dq);
    cache.erase(cache.begin() + (long)o);
  }
  const unsigned total = grid.x * grid.y * grid.z;
  unsigned char* d = nullptr;
  if (hipMalloc(&d, total) != hipSuccess) return false;
  std::vector<unsigned char> h(total);
  k_classify<Model, R, S, STG><<<grid, block, 0, s>>>(L, d);
  bool ok = hipGetLastError() == hipSuccess &&
            hipMemcpyAsync(h.data(), d, total, hipMemcpyDeviceToHost, s) == hipSuccess &&
            hipStreamSynchronize(s) == hipSuccess;
  hipFree(d);
  if (!ok) return false;
  std::vector<unsigned> l1, l2;
  for (unsigned b = 0; b < total; b++) {
    if (h[b] & 2) l1.push_back(b);
    if (h[b] & 4) l2.push_back(b);
  }
  ClassTiles c;
  c.flags = L.flags;
  c.gen = L.flags_gen;
  std::copy(box, box + 6, c.box);
  c.bx = block.x;
  c.by = block.y;
  c.n1 = (unsigned)l1.size();
  c.n2 = (unsigned)l2.size();
  c.total = total;
  c.used = ++clock;
  c.list = nullptr;
  c.dq = nullptr;
  // room for every node of the class-1 tiles (4 B per node)
  if (Model::defer_stage(STG) &&
      hipMalloc(&c.dq, ((size_t)l1.size() * block.x * block.y + 1) * sizeof(unsigned)) != hipSuccess)
    return false;
  l1.insert(l1.end(), l2.begin(), l2.end());
  if (!l1.empty()) {
    if (hipMalloc(&c.list, l1.size() * sizeof(unsigned)) != hipSuccess) {
      hipFree(c.dq);
      return false;
    }
    if (hipMemcpy(c.list, l1.data(), l1.size() * sizeof(unsigned), hipMemcpyHostToDevice) != hipSuccess) {
      hipFree(c.list);
      hipFree(c.dq);
      return false;
    }
  }
  cache.push_back(c);
  out = c;
  return true;
}

template <class Model, class R, class S, int STG, bool GLOB, int CLS>
__global__ void __launch_bounds__(256) k_stage_list(const Launch L, const unsigned* list, unsigned n, unsigned gx,
                                                    unsigned gy) {
  stage_tile<Model, R, S, STG, GLOB, CLS>(L, list_tile(L, list, n, gx, gy));
}
template <class Model, class R, class S, int STG, bool GLOB, int W, int CLS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W)))
k_stage_list_w(const Launch L, const unsigned* list, unsigned n, unsigned gx, unsigned gy) {
  stage_tile<Model, R, S, STG, GLOB, CLS>(L, list_tile(L, list, n, gx, gy));
}

// Deferring split stages (DSL add_stage(defer=True)).  The class-1 kernel records every
// node that took Node::defer_heavy (defer_record); the CLS 3 kernel then runs only those,
// one per thread of a grid of at most DEFER_GRID work-groups striding over the list (its
// length is read once, after the class-1 kernel ended: every thread reaches its end).  The
// rare heavy branch is compiled into the CLS 3 kernel alone, so it no longer sets the
// class-1 kernel's register budget (d3q27_tePSM_per: the CHT interface closure, 438 ->
// 254 registers, 1 -> 2 waves/SIMD), and its lanes are all busy (a list of nodes, not of
// tiles: a tile with interface nodes has ~20 of 256).
constexpr unsigned DEFER_GRID = 2048;
template <class Model, class R, class S, int STG, bool GLOB, int W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W > 0 ? W : 1)))
k_stage_defer(const Launch L, const unsigned* list, unsigned n, unsigned gx, unsigned gy, unsigned* dq) {
  stage_tile<Model, R, S, STG, GLOB, 1>(L, list_tile(L, list, n, gx, gy), dq);
}
// the list holds any (x, y, z) per lane: the flat addressing form only (Node::ROWA_ assumes
// a wave-uniform row)
template <class Model, class R, class S, int STG, int W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W > 0 ? W : 1)))
k_stage_deferred(const Launch L, const unsigned* dq) {
  typedef typename Model::template NodeCls<R, S, false, 3> N;
  static_assert(!N::ROWA_, "deferred nodes need the flat addressing form");
  const unsigned cnt = dq[0];
  const unsigned w = (unsigned)(L.xhi - L.xlo), h = (unsigned)(L.yhi - L.ylo);
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x) {
    const unsigned id = dq[1 + i], r = id / w;
    typename N::G_ g[1] = {typename N::G_(0)};
    N nd(L, L.xlo + (int)(id % w), L.ylo + (int)(r % h), L.zlo + (int)(r / h), g);
    nd.template run_stage<STG>();
  }
}

// LDS-staged stencil tiles: csrc/include/tclb_tile/k_tile.hpp (a dependency of the
// libraries of models with LDS-staged stages only, build.py _tile_deps)
#include "tclb_tile/k_tile.hpp"

template <class Model, class R, class S>
__global__ void __launch_bounds__(256) k_quantity(const Launch L) {
  const int x = L.xlo + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int y = __builtin_amdgcn_readfirstlane(L.ylo + (int)(blockIdx.y * blockDim.y + threadIdx.y));
  const int z = L.zlo + (int)blockIdx.z;
  if (x >= L.xhi || y >= L.yhi) return;
  typename Model::template NodeT<R, S, false>::G_ g[1];
  typename Model::template NodeT<R, S, false> n(L, x, y, z, g);
  n.pop();
  R o[3] = {R(0), R(0), R(0)};
  n.get_quantity(L.quantity, o);
  const long long idx = (long long)(x - L.xlo) + L.qsy * (y - L.ylo) + L.qsz * (z - L.zlo);
  R* out = (R*)L.aux;
  const int nc = L.reserved0 > 0 ? L.reserved0 : 1;
  for (int c = 0; c < nc; c++) out[idx + (long long)c * L.qcomp] = o[c] * R(L.qscale);
}

// Sampler probes: one thread per point, every quantity of the plan (core.hpp SamplePlan).
template <class Model, class R, class S>
__global__ void __launch_bounds__(64) k_sample(const Launch L, const SamplePlan P) {
  const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (p >= P.np) return;
  const int* c = P.points + 3 * p;
  typename Model::template NodeT<R, S, false>::G_ g[1];
  typename Model::template NodeT<R, S, false> n(L, c[0], c[1], c[2], g);
  sample_node(n, P, P.out + ((long long)P.row * P.np + p) * P.width);
}

// Default shapes from on-device A/B (profiles/r01_tune_*): fp64 storage 128x2, fp32 256x1.
inline void launch_shape(const Launch& L, dim3& grid, dim3& block, int sbytes = 8) {
  const int w = L.xhi - L.xlo, h = L.yhi - L.ylo, d = L.zhi - L.zlo;
  // a multiple of 64: every wave is one row segment (stage_body's wave-uniform y)
  int bx = L.block_x > 0 ? (L.block_x + 63) / 64 * 64 : 0;
  if (bx == 0) {
    // the widest row segment up to bmax that leaves the fewest idle lanes in the last
    // x tile (384 wide, fp32 storage: 128 instead of 256, whose second tile is half idle)
    const int bmax = sbytes >= 8 ? 128 : 256;
    int best = 64;
    for (int c = 64; c <= bmax; c *= 2) {
      if (c > 64 && c >= 2 * w) break;
      const int idle = (w + c - 1) / c * c - w, bidle = (w + best - 1) / best * best - w;
      if (idle <= bidle) best = c;
    }
    bx = best;
  }
  if (bx > 256) bx = 256;
  int by = L.block_y > 0 ? L.block_y : 256 / bx;
  if (by < 1) by = 1;
  if (bx * by > 256) by = 256 / bx;  // kernels are compiled with __launch_bounds__(256)
  block = dim3(bx, by, 1);
  grid = dim3((w + bx - 1) / bx, (h + by - 1) / by, d);
}

// Occupancy floor of the class-2 (boundary) kernels: 2 waves/SIMD, i.e. at most 256
// VGPRs and no AGPRs.  Without it the d3q27_tePSM_per_NEBB class-2 tile-list kernel of the
// plain (globals-free) step (344 registers, 88 of them AGPRs) stores wrong h populations on
// wall nodes on the MI355X, while the same node code is right as the full-grid kernel, as
// the globals kernel, with this floor, and on the CPU under UBSan (profiles/README.md
// r05m; build variant c2w0 reproduces it).  The class-2 nodes are the few boundary ones,
// so the spills of the floor cost nothing measurable.
#ifndef TCLB_SPLIT_WAVES2
#define TCLB_SPLIT_WAVES2 2
#endif
// one class of a split stage: over the list of its tiles (no class tiles: every tile)
template <class Model, class R, class S, int I, bool G, int CLS>
inline void launch_class(const Launch& L, dim3 grid, dim3 block, hipStream_t s, const ClassTiles* ct) {
  constexpr int W = (G && glob_waves<Model>() > 0) ? glob_waves<Model>()
                                                   : (CLS == 1 ? TCLB_SPLIT_WAVES : TCLB_SPLIT_WAVES2);
  const unsigned n = !ct ? grid.x * grid.y * grid.z : (CLS == 1 ? ct->n1 : ct->n2);
  if (n == 0) return;
  // every tile: no list (the list entry is a dependent load at the start of each
  // work-group, ~0.2 ms per step on the 1-wave tePSM collide)
  const unsigned* list = (!ct || n == ct->total) ? nullptr : ct->list + (CLS == 1 ? 0 : ct->n1);
  if constexpr (W > 0) k_stage_list_w<Model, R, S, I, G, W, CLS><<<dim3(n), block, 0, s>>>(L, list, n, grid.x, grid.y);
  else k_stage_list<Model, R, S, I, G, CLS><<<dim3(n), block, 0, s>>>(L, list, n, grid.x, grid.y);
}

template <class Model, class R, class S, int I, bool G>
inline bool launch_one(const Launch& L, dim3 grid, dim3 block, hipStream_t s) {
  if constexpr (TCLB_LDS_TILES && Model::tile_count(I) > 0) {
    const int w = L.xhi - L.xlo, h = L.yhi - L.ylo, d = L.zhi - L.zlo;
    constexpr int ZC = Model::tile_zc(I);
    const dim3 tg((w + TILE_BX - 1) / TILE_BX, (h + TILE_BY - 1) / TILE_BY, (d + ZC - 1) / ZC);
    k_tile<Model, R, S, I, G><<<tg, dim3(TILE_BX, TILE_BY, 1), 0, s>>>(L);
    return true;
  }
  if constexpr (Model::split_stage(I) && !TCLB_NO_SPLIT) {
    // one kernel per node class (the common interior path, then the rest), each over the
    // tiles that hold nodes of its class
    ClassTiles c;
    const ClassTiles* ct = class_tiles<Model, R, S, I>(L, grid, block, s, c) ? &c : nullptr;
    if constexpr (Model::defer_stage(I)) {
      // class 1 (queueing the deferred tiles), the deferred nodes, then class 2; the
      // queue lives with the tile lists (no lists: nothing to run the stage with)
      if (!ct || !ct->dq) return false;
      if (ct->n1 > 0) {
        constexpr int W = (G && glob_waves<Model>() > 0) ? glob_waves<Model>() : TCLB_SPLIT_WAVES;
        const unsigned* list = ct->n1 == ct->total ? nullptr : ct->list;
        if (hipMemsetAsync(ct->dq, 0, sizeof(unsigned), s) != hipSuccess) return false;
        k_stage_defer<Model, R, S, I, G, W><<<dim3(ct->n1), block, 0, s>>>(L, list, ct->n1, grid.x, grid.y, ct->dq);
        // the heavy path under the class-2 floor (no AGPRs, the form measured right; its
        // spills cost little on the few nodes it runs)
        const unsigned long long cap = (unsigned long long)ct->n1 * block.x * block.y;
        const unsigned dg = (unsigned)((cap + 255) / 256 < DEFER_GRID ? (cap + 255) / 256 : DEFER_GRID);
        k_stage_deferred<Model, R, S, I, TCLB_SPLIT_WAVES2><<<dim3(dg), dim3(256), 0, s>>>(L, ct->dq);
      }
      launch_class<Model, R, S, I, G, 2>(L, grid, block, s, ct);
    } else {
      launch_class<Model, R, S, I, G, 1>(L, grid, block, s, ct);
      launch_class<Model, R, S, I, G, 2>(L, grid, block, s, ct);
    }
    return true;
  }
  if constexpr (G && glob_waves<Model>() > 0) {
    k_stage_glob<Model, R, S, I, glob_waves<Model>()><<<grid, block, 0, s>>>(L);
    return true;
  }
#ifdef TCLB_NARROW_WAVES
  if constexpr (sizeof(S) < sizeof(double)) {
    k_stage_narrow<Model, R, S, I, G><<<grid, block, 0, s>>>(L);
    return true;
  }
#endif
  k_stage<Model, R, S, I, G><<<grid, block, 0, s>>>(L);
  return true;
}

template <class Model, class R, class S, bool G, int... I>
inline int run_stage_impl(const Launch& L, std::integer_sequence<int, I...>) {
  dim3 grid, block;
  launch_shape(L, grid, block, (int)sizeof(S));
  if (grid.x == 0 || grid.y == 0 || grid.z == 0) return 0;
  hipStream_t s = (hipStream_t)L.stream;
  bool found = false;
  ((L.stage == I ? (found = launch_one<Model, R, S, I, G>(L, grid, block, s)) : false), ...);
  if (!found) return -2;
  return (int)hipGetLastError();
}

template <class Model, class R, class S>
inline int run_stage(const Launch& L) {
  using Seq = std::make_integer_sequence<int, Model::NSTAGES_>;
  if (L.glob) return run_stage_impl<Model, R, S, true>(L, Seq{});
  return run_stage_impl<Model, R, S, false>(L, Seq{});
}

template <class Model, class R, class S>
inline int run_quantity(const Launch& L) {
  dim3 grid, block;
  launch_shape(L, grid, block, (int)sizeof(S));
  if (grid.x == 0 || grid.y == 0 || grid.z == 0) return 0;
  k_quantity<Model, R, S><<<grid, block, 0, (hipStream_t)L.stream>>>(L);
  return (int)hipGetLastError();
}

template <class Model, class R, class S>
inline int run_sample(const Launch& L, const SamplePlan& P) {
  if (P.np <= 0 || P.row < 0 || P.row >= P.rows) return 0;
  k_sample<Model, R, S><<<dim3((P.np + 63) / 64), dim3(64), 0, (hipStream_t)L.stream>>>(L, P);
  return (int)hipGetLastError();
}

}  // namespace exec
}  // namespace tclb

// C ABI (precision codes: core.hpp prec_dispatch)
#define TCLB_EXPORT_MODEL(NAME, MODEL)                                                       \
  TCLB_EXPORT_COMMON(NAME, MODEL)                                                            \
  extern "C" int tclb_##NAME##_device() { return 1; }
