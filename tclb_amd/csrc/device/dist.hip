// GPU side of the native action loop (tclb_rt/dist_loop.hpp): a context owning this
// rank's RCCL communicator, a high-priority comm stream and two events, the services of
// action_loop (stage launches, copy-back of out-of-place stages, the zonal time series,
// the particle hooks, the grid's packed y rows) and its transports:
//   * RCCL   — grouped ncclSend/ncclRecv of field planes straight from / into the output
//              snapshot on the comm stream (xGMI peer-to-peer between the GPUs of a node);
//              with one rank the peer is this rank itself (self send/receive), which runs
//              the same code on a single MI355X;
//   * copy   — the same plan with this rank as its own neighbour executed as device-to-
//              device copies on the comm stream (no RCCL; the single-GPU baseline).
// RCCL is dlopen'ed from the library torch already loaded (path given by the caller), so
// the process holds one RCCL instance; its communicator is created from a unique id that
// rank 0 makes and the ranks share through the torch.distributed store
// (tclb_amd/parallel/native.py).  Reference: MPIStream_A / MPIStream_B host-staged MPI
// (src/Lattice.cu.Rt:327-389) — no host staging here.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <thread>

#include "tclb_rt/ad_loop.hpp"
#include "tclb_rt/dist_loop.hpp"

namespace {

// the slice of the NCCL/RCCL C API the loop needs (rccl.h: ncclUniqueId is 128 bytes,
// ncclInt8 = 0, ncclSuccess = 0)
struct UniqueId {
  char internal[128];
};
typedef void* Comm;
typedef int (*fn_get_unique_id)(UniqueId*);
typedef int (*fn_comm_init_rank)(Comm*, int, UniqueId, int);
typedef int (*fn_comm_destroy)(Comm);
typedef int (*fn_send)(const void*, size_t, int, int, Comm, hipStream_t);
typedef int (*fn_recv)(void*, size_t, int, int, Comm, hipStream_t);
typedef int (*fn_group)();
typedef const char* (*fn_error_string)(int);
typedef int (*fn_async_error)(Comm, int*);
typedef int (*fn_all_reduce)(const void*, void*, size_t, int, int, Comm, hipStream_t);
typedef int (*fn_comm_abort)(Comm);

struct Rccl {
  void* h = nullptr;
  fn_get_unique_id get_unique_id = nullptr;
  fn_comm_init_rank comm_init_rank = nullptr;
  fn_comm_destroy comm_destroy = nullptr;
  fn_send send = nullptr;
  fn_recv recv = nullptr;
  fn_group group_start = nullptr, group_end = nullptr;
  fn_error_string error_string = nullptr;
  fn_async_error async_error = nullptr;
  fn_all_reduce all_reduce = nullptr;
  fn_comm_abort comm_abort = nullptr;
};

char g_err[512];

void set_err(const char* what, const char* detail) { snprintf(g_err, sizeof g_err, "%s: %s", what, detail); }

int load_rccl(const char* path, Rccl& R) {
  R.h = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
  if (!R.h) {
    set_err("dlopen", dlerror());
    return -10;
  }
#define SYM(field, name)                                          \
  R.field = (decltype(R.field))dlsym(R.h, name);                  \
  if (!R.field) {                                                 \
    set_err("dlsym", name);                                       \
    return -11;                                                   \
  }
  SYM(get_unique_id, "ncclGetUniqueId")
  SYM(comm_init_rank, "ncclCommInitRank")
  SYM(comm_destroy, "ncclCommDestroy")
  SYM(send, "ncclSend")
  SYM(recv, "ncclRecv")
  SYM(group_start, "ncclGroupStart")
  SYM(group_end, "ncclGroupEnd")
  SYM(error_string, "ncclGetErrorString")
  SYM(async_error, "ncclCommGetAsyncError")
  SYM(all_reduce, "ncclAllReduce")
  SYM(comm_abort, "ncclCommAbort")
#undef SYM
  return 0;
}

// IPC transport signal block: one monotonically increasing counter per word, each on its
// own 128-byte line; A = the slab / grid-z phase, B = the grid's y phase, R = the particle
// force all-reduce; READY: this rank's send data of exchange e is in place, DONE: this rank
// has pulled its neighbours' data of exchange e; ERR: a wait of this rank timed out
enum { SIG_A_READY = 0, SIG_A_DONE, SIG_B_READY, SIG_B_DONE, SIG_R_READY, SIG_R_DONE, SIG_ERR, SIG_WORDS };
constexpr int SIG_STRIDE = 16;   // words between counters
constexpr size_t SIG_BYTES = sizeof(unsigned long long) * SIG_STRIDE * SIG_WORDS;
constexpr int IPC_MAX_RANKS = 64;   // one wave polls every rank's counter

struct Ctx {
  int transport;  // 0 = device copies (loopback), 1 = RCCL, 3 = IPC (peer memory pulls)
  int nranks, rank;
  Rccl R;
  Comm comm = nullptr;
  hipStream_t cs = nullptr;   // comm stream
  hipEvent_t ready = nullptr, done = nullptr;
  hipEvent_t fence = nullptr;   // IPC: a system-scope release before READY is published
  // IPC transport
  unsigned long long* sig = nullptr;              // this rank's signal block (exported)
  unsigned long long* hsig[IPC_MAX_RANKS] = {};   // every rank's, mapped (host table)
  unsigned long long** dsig = nullptr;            // the same table on the device
  unsigned long long seq[3] = {0, 0, 0};          // exchange counters of A, B, R
  long long ticks = 0;                            // wait timeout in wall-clock ticks
};

int rccl_check(Ctx* c, int r, const char* what) {
  if (r == 0) return 0;
  set_err(what, c->R.error_string ? c->R.error_string(r) : "?");
  return 1000 + r;
}

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return 0;
  set_err(what, hipGetErrorString(e));
  return 2000 + (int)e;
}

// pack (unpack = 0) or unpack one block of the grid's y phase: [field][z][y][x] between
// the snapshot and staging + boff; one thread per element
template <class T>
__global__ void __launch_bounds__(256) k_pack(T* snap, T* stg, long long fs, long long sz, long long sy, int px,
                                              int nfield, int ny, int nz, int y0, int z0, int f0, int unpack) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long per = (long long)px * ny * nz;
  if (i >= per * nfield) return;
  const int f = (int)(i / per);
  long long r = i - f * per;
  const int z = (int)(r / ((long long)px * ny));
  r -= (long long)z * px * ny;
  const int y = (int)(r / px), x = (int)(r - (long long)y * px);
  T* a = snap + (long long)(f0 + f) * fs + (long long)(z0 + z) * sz + (long long)(y0 + y) * sy + x;
  if (unpack) *a = stg[i];
  else stg[i] = *a;
}

// the contiguous segments of a packed phase A (tclb_rt/dist_loop.hpp SegOp), one launch
// for all of them: blockIdx.y picks the segment, the x blocks stride over its V words
struct Peers {
  const char* p[4];
};

template <class V>
__global__ void __launch_bounds__(256) k_segcopy(const tclb::SegOp* segs, char* snap, char* stg, Peers peers) {
  const tclb::SegOp o = segs[blockIdx.y];
  char* d;
  const char* s;
  if (o.dir == 0) {
    d = stg + o.dst, s = snap + o.src;
  } else if (o.dir == 1) {
    d = snap + o.dst, s = stg + o.src;
  } else {
    const char* b = o.peer == 0 ? peers.p[0] : o.peer == 1 ? peers.p[1] : o.peer == 2 ? peers.p[2] : peers.p[3];
    d = (o.dir == 2 ? snap : stg) + o.dst, s = b + o.src;
  }
  const long long nv = o.bytes / (long long)sizeof(V);
  const long long step = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += step)
    ((V*)d)[i] = ((const V*)s)[i];
}

// active entries of the zonal time series: zonal[idx] = v[iter % len] (and the slope)
__global__ void k_series(double* zonal, const tclb::SeriesEntry* E, int n, const double* v, const double* dv,
                         int iter) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const tclb::SeriesEntry e = E[i];
  const int k = iter % e.len;
  zonal[e.idx] = v[e.off + k];
  if (e.len > 1) zonal[e.dtidx] = dv[e.off + k];
}

// IPC transport: publish counter value v (after everything earlier on the stream)
__global__ void k_signal(unsigned long long* f, unsigned long long v) {
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// IPC transport: lane r waits until rank r's counter `word` reaches v, for every rank in
// `mask`.  Bounded: after `ticks` of the constant wall clock the lane flags *err and
// leaves (a dead peer ends in an error the host reads, never in a wave that spins
// forever); once *err is set every later wait returns at once.
__global__ void k_wait(unsigned long long* const* tab, unsigned long long mask, int word, unsigned long long v,
                       unsigned long long* err, long long ticks) {
  const int r = threadIdx.x;
  if (r >= 64 || !((mask >> r) & 1ull)) return;
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return;
  const unsigned long long* f = tab[r] + word;
  const long long t0 = wall_clock64();
  while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < v) {
    if (wall_clock64() - t0 > ticks) {
      __hip_atomic_store(err, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(4);
  }
}

// IPC transport: the particle force all-reduce, every rank summing the ranks' shared
// copies in rank order (the same sum, bit for bit, on every rank)
__global__ void __launch_bounds__(256) k_accsum(double* out, const double* const* accs, int nranks, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s = accs[0][i];
  for (int r = 1; r < nranks; r++) s += accs[r][i];
  out[i] = s;
}

__global__ void __launch_bounds__(256) k_nan0(double* a, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && isnan(a[i])) a[i] = 0.0;
}

}  // namespace

extern "C" int tclb_part_build_grid(const double*, int, int*, int, int, int, int, int, void*, long long, void*);
extern "C" int tclb_part_build_tree(const double*, int, int*, int, double, void*, long long, void*);
extern "C" int tclb_part_acc_slots(double*, int, int, void*);
extern "C" int tclb_part_rigid_step(double*, const double*, const double*, const unsigned char*, int, double, double,
                                    double, int, double, double, double, void*);

namespace {

// The services of tclb::action_loop on the GPU.  Launches and copies go to the compute
// stream ks; an exchange is ordered after the work already on ks, runs on the comm stream
// (phase A sends / receives, the grid's y-row packs, phase B, the unpacks) and xfinish
// makes ks wait for it.
struct GpuSvc {
  Ctx* c;
  hipStream_t ks;
  int prec;
  tclb::run_fn runf;
  tclb::sample_fn samplef;
  int es;              // bytes per stored element
  long long fs, sz, sy;
  int px;

  int run(tclb::Launch& L) { return runf(&L, prec); }
  int sample(tclb::Launch& L, const tclb::SamplePlan& P) { return samplef ? samplef(&L, prec, &P) : 0; }

  int copy_runs(void* dst, const void* src, const tclb::LoopPlan& P, const tclb::StagePlan& st) {
    for (int i = 0; i < st.nruns; i++) {
      const int r0 = P.runs[2 * (st.run0 + i)], r1 = P.runs[2 * (st.run0 + i) + 1];
      const long long off = (long long)r0 * P.fs_bytes, b = (long long)(r1 - r0) * P.fs_bytes;
      const int r = hip_check(hipMemcpyAsync((char*)dst + off, (const char*)src + off, (size_t)b,
                                             hipMemcpyDeviceToDevice, ks), "hipMemcpyAsync");
      if (r != 0) return r;
    }
    return 0;
  }

  // RCCL: every message goes as pieces of at most rccl_chunk() bytes, in order (both ends
  // cut an op the same way, and sends / receives between a pair of ranks match in issue
  // order).  With one channel per peer, whole 18.9 MB halves of the 512x512x64 d3q27 slab
  // arrived wrong, deterministically, and 4.7 MB ones right (profiles/README.md r06n-o);
  // the per-peer channel count RCCL picks between two GPUs is not known here, so no
  // message is allowed to be large.
  static size_t rccl_chunk() {
    static const size_t b = [] {
      const char* e = getenv("TCLB_RCCL_CHUNK_MB");
      const double mb = e ? atof(e) : 4.0;
      return mb > 0 ? (size_t)(mb * 1048576.0) : (size_t)0;   // 0: whole messages
    }();
    return b;
  }
  int p2p(char* base, char* stg, const tclb::HaloOp* ops, int nops) {
    if (nops == 0) return 0;
    if (c->transport == 1) {
      int r;
      const size_t chunk = rccl_chunk();
      if ((r = rccl_check(c, c->R.group_start(), "ncclGroupStart")) != 0) return r;
      for (int i = 0; i < nops; i++) {
        const tclb::HaloOp& o = ops[i];
        char* a = (o.buf ? stg : base) + o.off;
        const size_t tot = (size_t)o.bytes;
        for (size_t done = 0; done < tot || (tot == 0 && done == 0);) {
          const size_t b = (chunk == 0 || tot - done <= chunk) ? tot - done : chunk;
          const int e = o.kind == 0 ? c->R.send(a + done, b, 0, o.peer, c->comm, c->cs)
                                    : c->R.recv(a + done, b, 0, o.peer, c->comm, c->cs);
          if (e != 0) {
            c->R.group_end();
            return rccl_check(c, e, o.kind == 0 ? "ncclSend" : "ncclRecv");
          }
          done += b;
          if (tot == 0) break;
        }
      }
      return rccl_check(c, c->R.group_end(), "ncclGroupEnd");
    }
    const int r = tclb::dist_self_pairs(base, stg, ops, nops, c->rank, [&](char* d, const char* s, long long b) {
      return hip_check(hipMemcpyAsync(d, s, (size_t)b, hipMemcpyDeviceToDevice, c->cs), "hipMemcpyAsync");
    });
    if (r == -3) set_err("halo plan", "sends and receives to self do not pair up");
    return r;
  }

  int packs(char* base, char* stg, const tclb::PackOp* pk, int n, int unpack) {
    for (int i = 0; i < n; i++) {
      const tclb::PackOp& o = pk[i];
      if (o.unpack != unpack) continue;
      const long long tot = (long long)o.nfield * o.nz * o.ny * px;
      const unsigned blocks = (unsigned)((tot + 255) / 256);
      if (es == 8)
        k_pack<double><<<blocks, 256, 0, c->cs>>>((double*)base, (double*)(stg + o.boff), fs, sz, sy, px, o.nfield,
                                                  o.ny, o.nz, o.y0, o.z0, o.field0, unpack);
      else if (es == 4)
        k_pack<float><<<blocks, 256, 0, c->cs>>>((float*)base, (float*)(stg + o.boff), fs, sz, sy, px, o.nfield,
                                                 o.ny, o.nz, o.y0, o.z0, o.field0, unpack);
      else
        k_pack<unsigned short><<<blocks, 256, 0, c->cs>>>((unsigned short*)base, (unsigned short*)(stg + o.boff), fs,
                                                          sz, sy, px, o.nfield, o.ny, o.nz, o.y0, o.z0, o.field0,
                                                          unpack);
      const int r = hip_check(hipGetLastError(), "k_pack");
      if (r != 0) return r;
    }
    return 0;
  }

  // one launch over segments [s0, s0 + n) of the plan, on the comm stream
  int segcopy(char* base, char* stg, const tclb::LoopPlan& P, int s0, int n) {
    if (n <= 0) return 0;
    long long align = 0, maxb = 0;
    for (int i = 0; i < n; i++) {
      const tclb::SegOp& o = P.segs[s0 + i];
      align |= o.dst | o.src | o.bytes;
      if (o.bytes > maxb) maxb = o.bytes;
    }
    const int w = (align & 15) == 0 ? 16 : (align & 7) == 0 ? 8 : (align & 3) == 0 ? 4 : (align & 1) == 0 ? 2 : 1;
    long long bx = (maxb / w + 255) / 256;
    if (bx > 1024) bx = 1024;
    if (bx < 1) bx = 1;
    const dim3 grid((unsigned)bx, (unsigned)n);
    const tclb::SegOp* d = P.dsegs + s0;
    Peers pe;
    for (int i = 0; i < 4; i++) pe.p[i] = (const char*)P.peer_stg[i];
    switch (w) {
      case 16: k_segcopy<uint4><<<grid, 256, 0, c->cs>>>(d, base, stg, pe); break;
      case 8: k_segcopy<uint2><<<grid, 256, 0, c->cs>>>(d, base, stg, pe); break;
      case 4: k_segcopy<unsigned><<<grid, 256, 0, c->cs>>>(d, base, stg, pe); break;
      case 2: k_segcopy<unsigned short><<<grid, 256, 0, c->cs>>>(d, base, stg, pe); break;
      default: k_segcopy<unsigned char><<<grid, 256, 0, c->cs>>>(d, base, stg, pe); break;
    }
    return hip_check(hipGetLastError(), "k_segcopy");
  }

  // IPC transport primitives (see k_signal / k_wait)
  int signal(hipStream_t s, int word, unsigned long long v) {
    k_signal<<<1, 64, 0, s>>>(c->sig + word * SIG_STRIDE, v);
    return hip_check(hipGetLastError(), "k_signal");
  }
  int wait(hipStream_t s, unsigned long long mask, int word, unsigned long long v) {
    if (!mask) return 0;
    k_wait<<<1, 64, 0, s>>>(c->dsig, mask, word * SIG_STRIDE, v, c->sig + SIG_ERR * SIG_STRIDE, c->ticks);
    return hip_check(hipGetLastError(), "k_wait");
  }
  static unsigned long long peer_mask(const tclb::LoopPlan& P, int a, int b) {
    unsigned long long m = 0;
    if (P.ipc_peer[a] >= 0) m |= 1ull << P.ipc_peer[a];
    if (P.ipc_peer[b] >= 0) m |= 1ull << P.ipc_peer[b];
    return m;
  }

  // the exchange of one stage over IPC-mapped peer memory, on the comm stream: publish
  // READY, wait for the neighbours' READY, pull their packed send buffers straight into
  // the ghost planes (one copy launch), publish DONE; the grid's y phase the same way
  // through the staging rows; finally wait for the neighbours' DONE, so nothing of this
  // rank's send buffers is rewritten (next stage / step) before they have been read.
  // Reference: MPIStream_A / MPIStream_B (src/Lattice.cu.Rt:327-389), here without MPI
  // or a collective library — a one-sided pull between the processes of one node.
  int xstart_ipc(char* base, const tclb::LoopPlan& P, const tclb::StagePlan& st, int mirrored) {
    int r;
    char* stg = (char*)P.staging;
    if ((r = hip_check(hipEventRecord(c->ready, ks), "hipEventRecord")) != 0) return r;
    if ((r = hip_check(hipStreamWaitEvent(c->cs, c->ready, 0), "hipStreamWaitEvent")) != 0) return r;
    const unsigned long long mA = peer_mask(P, 0, 1), mB = peer_mask(P, 2, 3);
    const unsigned long long e = ++c->seq[0];
    if (!mirrored && (r = segcopy(base, stg, P, st.seg0, st.npack)) != 0) return r;
    // the send buffers were written by kernels of this stream (concurrent borders) or of ks:
    // an event's system-scope release writes every XCD's L2 back before READY goes out, so
    // a peer GPU reading over xGMI sees them (within one device the kernel boundary would do)
    if ((r = hip_check(hipEventRecord(c->fence, c->cs), "hipEventRecord")) != 0) return r;
    if ((r = signal(c->cs, SIG_A_READY, e)) != 0 || (r = wait(c->cs, mA, SIG_A_READY, e)) != 0) return r;
    if ((r = segcopy(base, stg, P, st.seg0 + st.npack, st.nunpack)) != 0) return r;
    if ((r = signal(c->cs, SIG_A_DONE, e)) != 0) return r;
    if (st.npk > 0 || st.nyseg > 0) {
      const unsigned long long eb = ++c->seq[1];
      if ((r = packs(base, stg, P.packs + st.pk0, st.npk, 0)) != 0) return r;
      if ((r = hip_check(hipEventRecord(c->fence, c->cs), "hipEventRecord")) != 0) return r;
      if ((r = signal(c->cs, SIG_B_READY, eb)) != 0 || (r = wait(c->cs, mB, SIG_B_READY, eb)) != 0) return r;
      if ((r = segcopy(base, stg, P, st.yseg0, st.nyseg)) != 0) return r;
      if ((r = packs(base, stg, P.packs + st.pk0, st.npk, 1)) != 0) return r;
      if ((r = signal(c->cs, SIG_B_DONE, eb)) != 0 || (r = wait(c->cs, mB, SIG_B_DONE, eb)) != 0) return r;
    }
    if ((r = wait(c->cs, mA, SIG_A_DONE, e)) != 0) return r;
    return hip_check(hipEventRecord(c->done, c->cs), "hipEventRecord");
  }

  // the exchange of one stage on the comm stream, ordered after the work on ks: phase A
  // (pack unless the border launches mirrored their stores, one send and one receive per
  // neighbour, unpack), then the grid's y phase (row packs, sends / receives, unpacks)
  int xstart(char* base, const tclb::LoopPlan& P, const tclb::StagePlan& st, int mirrored) {
    if (c->transport == 3) return xstart_ipc(base, P, st, mirrored);
    int r;
    char* stg = (char*)P.staging;
    if ((r = hip_check(hipEventRecord(c->ready, ks), "hipEventRecord")) != 0) return r;
    if ((r = hip_check(hipStreamWaitEvent(c->cs, c->ready, 0), "hipStreamWaitEvent")) != 0) return r;
    if (!mirrored && (r = segcopy(base, stg, P, st.seg0, st.npack)) != 0) return r;
    if ((r = p2p(base, stg, P.ops + st.op0, st.nops)) != 0) return r;
    if ((r = segcopy(base, stg, P, st.seg0 + st.npack, st.nunpack)) != 0) return r;
    if (st.nopsb > 0) {
      if ((r = packs(base, stg, P.packs + st.pk0, st.npk, 0)) != 0) return r;
      if ((r = p2p(base, stg, P.ops + st.opb0, st.nopsb)) != 0) return r;
      if ((r = packs(base, stg, P.packs + st.pk0, st.npk, 1)) != 0) return r;
    }
    return hip_check(hipEventRecord(c->done, c->cs), "hipEventRecord");
  }
  int xfinish() { return hip_check(hipStreamWaitEvent(ks, c->done, 0), "hipStreamWaitEvent"); }
  // the comm stream after the work on ks (the border launches of overlap 2 go there)
  void* fork() {
    (void)hipEventRecord(c->ready, ks);
    (void)hipStreamWaitEvent(c->cs, c->ready, 0);
    return (void*)c->cs;
  }

  int series(const tclb::LoopPlan& P, int iter) {
    k_series<<<(P.nseries + 63) / 64, 64, 0, ks>>>(P.zonal, P.series, P.nseries, P.svals, P.sslopes, iter);
    return hip_check(hipGetLastError(), "k_series");
  }

  int part_pre(tclb::Launch& L, const tclb::LoopPlan& P) {
    const tclb::PartPlan& q = *P.part;
    const int k = q.nslots > 1 ? q.nslots : 1;
    int r = hip_check(hipMemsetAsync(q.acc, 0, sizeof(double) * 6 * (size_t)(q.n > 0 ? q.n : 1) * k, ks), "memset");
    if (r != 0) return r;
    if (q.container == 1) r = tclb_part_build_grid(q.P, q.n, q.grid, q.gdim[0], q.gdim[1], q.gdim[2], q.cell, q.ncell,
                                                   q.tmp, q.tmp_bytes, ks);
    else if (q.container == 2) r = tclb_part_build_tree(q.P, q.n, q.grid, q.nl, q.mscale, q.tmp, q.tmp_bytes, ks);
    if (r != 0) {
      set_err("solid container build", hipGetErrorString((hipError_t)(r > 0 ? r : 1)));
      return 3000 + (r < 0 ? -r : r);
    }
    L.ext[2] = q.P;
    L.ext[3] = q.acc;
    L.next[3] = k;
    L.next[2] = q.n;
    L.ext[4] = q.container ? q.grid : nullptr;
    L.next[4] = q.container ? q.grid_n : 0;
    return 0;
  }

  int part_post(tclb::Launch& L, const tclb::LoopPlan& P, int step) {
    const tclb::PartPlan& q = *P.part;
    int r;
    const int na = 6 * q.n;
    if (q.nslots > 1 && na > 0 && (r = tclb_part_acc_slots(q.acc, na, q.nslots, ks)) != 0)
      return hip_check((hipError_t)r, "accumulator copies");
    if (q.allreduce && c->transport == 1 && c->nranks > 1 && na > 0) {
      // ncclFloat64 = 8, ncclSum = 0; on the compute stream, after the stage's kernels
      if ((r = rccl_check(c, c->R.all_reduce(q.acc, q.acc, (size_t)na, 8, 0, c->comm, ks), "ncclAllReduce")) != 0)
        return r;
    }
    if (q.allreduce && c->transport == 3 && c->nranks > 1 && na > 0) {
      // publish a copy, wait for every rank's, sum them in rank order, and wait until
      // every rank has summed before the copy may be rewritten
      const unsigned long long e = ++c->seq[2];
      const unsigned long long all = c->nranks >= 64 ? ~0ull : ((1ull << c->nranks) - 1);
      if ((r = hip_check(hipMemcpyAsync(q.accbuf, q.acc, sizeof(double) * (size_t)na, hipMemcpyDeviceToDevice, ks),
                         "hipMemcpyAsync")) != 0 ||
          (r = hip_check(hipEventRecord(c->fence, ks), "hipEventRecord")) != 0)
        return r;
      if ((r = signal(ks, SIG_R_READY, e)) != 0 || (r = wait(ks, all, SIG_R_READY, e)) != 0) return r;
      k_accsum<<<(na + 255) / 256, 256, 0, ks>>>(q.acc, q.accs, c->nranks, na);
      if ((r = hip_check(hipGetLastError(), "k_accsum")) != 0) return r;
      if ((r = signal(ks, SIG_R_DONE, e)) != 0 || (r = wait(ks, all, SIG_R_DONE, e)) != 0) return r;
    }
    if (na > 0) {
      k_nan0<<<(na + 255) / 256, 256, 0, ks>>>(q.acc, na);
      if ((r = hip_check(hipGetLastError(), "k_nan0")) != 0) return r;
    }
    L.next[2] = 0;
    L.next[3] = 0;
    L.ext[4] = nullptr;
    L.next[4] = 0;
    if (step && q.integrate && q.n > 0) {
      r = tclb_part_rigid_step(q.P, q.acc, q.m, q.free_, q.n, q.a[0], q.a[1], q.a[2], q.periodic, q.period[0],
                               q.period[1], q.period[2], ks);
      if (r != 0) return hip_check((hipError_t)r, "rigid step");
    }
    return 0;
  }
};

}  // namespace

extern "C" {

const char* tclb_dist_last_error() { return g_err; }

int tclb_dist_unique_id(const char* rccl_path, void* out) {
  Rccl R;
  int r = load_rccl(rccl_path, R);
  if (r != 0) return r;
  UniqueId id;
  r = R.get_unique_id(&id);
  if (r != 0) {
    set_err("ncclGetUniqueId", R.error_string(r));
    return 1000 + r;
  }
  memcpy(out, id.internal, sizeof id.internal);
  return 0;
}

// transport 0: device copies (nranks must be 1); 1: RCCL communicator of nranks ranks
void tclb_dist_ctx_destroy(void* ctx);

void* tclb_dist_ctx_create(const char* rccl_path, int transport, int nranks, int rank, const void* uid) {
  Ctx* c = new Ctx();
  c->transport = transport;
  c->nranks = nranks;
  c->rank = rank;
  int lo = 0, hi = 0;
  if (hip_check(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange") != 0 ||
      hip_check(hipStreamCreateWithPriority(&c->cs, hipStreamNonBlocking, hi), "hipStreamCreateWithPriority") != 0 ||
      hip_check(hipEventCreateWithFlags(&c->ready, hipEventDisableTiming), "hipEventCreate") != 0 ||
      hip_check(hipEventCreateWithFlags(&c->done, hipEventDisableTiming), "hipEventCreate") != 0 ||
      hip_check(hipEventCreateWithFlags(&c->fence, hipEventDisableTiming), "hipEventCreate") != 0) {
    delete c;
    return nullptr;
  }
  if (transport == 1) {
    if (load_rccl(rccl_path, c->R) != 0) {
      delete c;
      return nullptr;
    }
    UniqueId id;
    memcpy(id.internal, uid, sizeof id.internal);
    const int r = c->R.comm_init_rank(&c->comm, nranks, id, rank);
    if (r != 0) {
      set_err("ncclCommInitRank", c->R.error_string(r));
      delete c;
      return nullptr;
    }
  } else if (transport == 3) {
    if (nranks > IPC_MAX_RANKS) {
      set_err("tclb_dist_ctx_create", "the IPC transport takes at most 64 ranks");
      delete c;
      return nullptr;
    }
    // the signal block: uncached device memory, so a wave polling a counter of another
    // process (same device or a peer over xGMI) reads memory, never a stale cache line
    if (hipExtMallocWithFlags((void**)&c->sig, SIG_BYTES, hipDeviceMallocUncached) != hipSuccess &&
        hip_check(hipMalloc((void**)&c->sig, SIG_BYTES), "hipMalloc") != 0) {
      delete c;
      return nullptr;
    }
    int khz = 0, dev = 0;
    (void)hipGetDevice(&dev);
    if (hip_check(hipMemset(c->sig, 0, SIG_BYTES), "hipMemset") != 0 ||
        hip_check(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev), "hipDeviceGetAttribute") != 0 ||
        hip_check(hipMalloc((void**)&c->dsig, sizeof(void*) * IPC_MAX_RANKS), "hipMalloc") != 0) {
      tclb_dist_ctx_destroy(c);
      return nullptr;
    }
    const char* t = getenv("TCLB_IPC_TIMEOUT_S");
    const double sec = t ? atof(t) : 120.0;
    c->ticks = (long long)((double)(khz > 0 ? khz : 100000) * 1000.0 * sec);
    c->hsig[rank] = c->sig;
  } else if (nranks != 1) {
    set_err("tclb_dist_ctx_create", "the copy transport is single-rank");
    delete c;
    return nullptr;
  }
  return c;
}

// ---- IPC transport: shared buffers, the signal blocks, the error flag

// device memory another process can map: zeroed, its handle (64 bytes) into handle_out
void* tclb_ipc_alloc(long long bytes, void* handle_out) {
  void* p = nullptr;
  if (hip_check(hipMalloc(&p, (size_t)(bytes > 0 ? bytes : 1)), "hipMalloc") != 0) return nullptr;
  hipIpcMemHandle_t h;
  if (hip_check(hipMemset(p, 0, (size_t)(bytes > 0 ? bytes : 1)), "hipMemset") != 0 ||
      hip_check(hipIpcGetMemHandle(&h, p), "hipIpcGetMemHandle") != 0) {
    (void)hipFree(p);
    return nullptr;
  }
  memcpy(handle_out, &h, sizeof h);
  return p;
}
void tclb_ipc_free(void* p) {
  if (p) (void)hipFree(p);
}
void* tclb_ipc_open(const void* handle) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof h);
  void* p = nullptr;
  if (hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle") != 0) return nullptr;
  return p;
}
void tclb_ipc_close(void* p) {
  if (p) (void)hipIpcCloseMemHandle(p);
}
int tclb_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

int tclb_dist_sig_handle(void* ctx, void* out) {
  Ctx* c = (Ctx*)ctx;
  hipIpcMemHandle_t h;
  const int r = hip_check(hipIpcGetMemHandle(&h, c->sig), "hipIpcGetMemHandle(signals)");
  if (r == 0) memcpy(out, &h, sizeof h);
  return r;
}

// map every other rank's signal block (handles: nranks x 64 bytes, rank order)
int tclb_dist_sig_attach(void* ctx, const char* handles) {
  Ctx* c = (Ctx*)ctx;
  for (int k = 0; k < c->nranks; k++) {
    if (k == c->rank) continue;
    void* p = tclb_ipc_open(handles + (size_t)k * sizeof(hipIpcMemHandle_t));
    if (!p) return -20;
    c->hsig[k] = (unsigned long long*)p;
  }
  return hip_check(hipMemcpy(c->dsig, c->hsig, sizeof(void*) * IPC_MAX_RANKS, hipMemcpyHostToDevice), "hipMemcpy");
}

// 1: a wait of this rank timed out (a peer stopped publishing); reads the flag
// synchronously (call when the rank's queued work has been waited for)
int tclb_dist_ipc_error(void* ctx) {
  Ctx* c = (Ctx*)ctx;
  if (!c || c->transport != 3 || !c->sig) return 0;
  unsigned long long v = 0;
  if (hipMemcpy(&v, c->sig + SIG_ERR * SIG_STRIDE, sizeof v, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return v ? 1 : 0;
}

void tclb_dist_ctx_destroy(void* ctx) {
  Ctx* c = (Ctx*)ctx;
  if (!c) return;
  if (c->cs) (void)hipStreamSynchronize(c->cs);
  if (c->comm) c->R.comm_destroy(c->comm);
  for (int k = 0; k < IPC_MAX_RANKS; k++)
    if (c->hsig[k] && k != c->rank) (void)hipIpcCloseMemHandle(c->hsig[k]);
  if (c->sig) (void)hipFree(c->sig);
  if (c->dsig) (void)hipFree(c->dsig);
  if (c->ready) (void)hipEventDestroy(c->ready);
  if (c->done) (void)hipEventDestroy(c->done);
  if (c->fence) (void)hipEventDestroy(c->fence);
  if (c->cs) (void)hipStreamDestroy(c->cs);
  delete c;
}

// the n steps of an action (tclb_rt/dist_loop.hpp action_loop); run / sample are the
// model library's tclb_<model>_run / tclb_<model>_sample; launches go to L->stream.
// es: bytes per stored element (the grid's pack kernels)
int tclb_loop_iterate(void* ctx, const tclb::Launch* L, int prec, int es, int nsteps, int glob_last, int init,
                      const tclb::LoopPlan* P, tclb::run_fn run, tclb::sample_fn sample) {
  Ctx* c = (Ctx*)ctx;
  GpuSvc sv{c, (hipStream_t)L->stream, prec, run, sample, es, L->fs, L->sz, L->sy, L->px};
  const int r = tclb::action_loop(sv, *L, nsteps, glob_last, *P, init);
  if (r != 0) return r;
  // a communicator that failed while these steps were queued (a dead peer) is reported
  // here, not only by tclb_dist_wait, so loops without a globals wait still raise
  if (c->transport == 1 && c->comm) {
    int ae = 0;
    if (c->R.async_error(c->comm, &ae) == 0 && ae != 0) return rccl_check(c, ae, "RCCL async error");
  }
  return 0;
}

// one exchange outside the loop (the Python step path of the same plan)
int tclb_dist_exchange(void* ctx, void* base, const tclb::HaloOp* ops, int nops, void* stream) {
  Ctx* c = (Ctx*)ctx;
  GpuSvc sv{c, (hipStream_t)stream, 0, nullptr, nullptr, 8, 0, 0, 0, 0};
  tclb::LoopPlan P = {};
  tclb::StagePlan st = {};
  P.ops = ops;
  st.nops = nops;
  int r = sv.xstart((char*)base, P, st, 1);
  return r != 0 ? r : sv.xfinish();
}

// the exchange of stage k of a plan outside the loop (Lattice.exchange on a rank whose
// halos travel through the loop's transport: after set_fields_interior, a restart, ...)
int tclb_loop_exchange(void* ctx, void* base, const tclb::LoopPlan* P, int k, int es, long long fs, long long sz,
                       long long sy, int px, void* stream) {
  Ctx* c = (Ctx*)ctx;
  GpuSvc sv{c, (hipStream_t)stream, 0, nullptr, nullptr, es, fs, sz, sy, px};
  const int r = sv.xstart((char*)base, *P, P->st[k], 0);
  return r != 0 ? r : sv.xfinish();
}

// wait for the work queued on `stream` with the communicator watched: polls the RCCL
// asynchronous error while the stream runs and aborts the communicator on an error or
// after timeout_ms (a dead peer then ends this rank's wait instead of hanging it)
int tclb_dist_wait(void* ctx, void* stream, int timeout_ms) {
  Ctx* c = (Ctx*)ctx;
  hipEvent_t e;
  int r = hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
  if (r != 0) return r;
  if ((r = hip_check(hipEventRecord(e, (hipStream_t)stream), "hipEventRecord")) != 0) {
    (void)hipEventDestroy(e);
    return r;
  }
  const auto t0 = std::chrono::steady_clock::now();
  long long spins = 0;
  for (;;) {
    const hipError_t q = hipEventQuery(e);
    if (q == hipSuccess) break;
    if (q != hipErrorNotReady) {
      r = hip_check(q, "hipEventQuery");
      break;
    }
    if (c->transport == 1 && c->comm) {
      int ae = 0;
      if (c->R.async_error(c->comm, &ae) == 0 && ae != 0) {
        r = rccl_check(c, ae, "RCCL async error");
        c->R.comm_abort(c->comm);
        c->comm = nullptr;
        break;
      }
    }
    std::this_thread::sleep_for(std::chrono::microseconds(20));
    if (timeout_ms > 0 && (++spins & 1023) == 0 &&
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() > timeout_ms) {
      set_err("tclb_dist_wait", "timed out: aborting the communicator");
      if (c->transport == 1 && c->comm) {
        c->R.comm_abort(c->comm);
        c->comm = nullptr;
      }
      r = -110;
      break;
    }
  }
  (void)hipEventDestroy(e);
  if (r == 0 && c->transport == 3 && tclb_dist_ipc_error(c) != 0) {
    set_err("IPC transport", "a wait for a peer's counter timed out (TCLB_IPC_TIMEOUT_S)");
    r = -111;
  }
  return r;
}

// the reverse sweep of one checkpoint segment (tclb_rt/ad_loop.hpp) on the GPU
int tclb_ad_segment(const tclb::Launch* L, const tclb::AdSegPlan* P, tclb::ad_run_fn run) {
  hipStream_t s = (hipStream_t)L->stream;
  return tclb::ad_segment(*L, *P, run, [&](void* p, long long b) {
    return hip_check(hipMemsetAsync(p, 0, (size_t)b, s), "hipMemsetAsync");
  });
}
int tclb_ad_sizeof_seg() { return (int)sizeof(tclb::AdSegPlan); }

int tclb_loop_sizeof_plan() { return (int)sizeof(tclb::LoopPlan); }
int tclb_loop_sizeof_stage() { return (int)sizeof(tclb::StagePlan); }
int tclb_loop_sizeof_part() { return (int)sizeof(tclb::PartPlan); }
int tclb_loop_sizeof_pack() { return (int)sizeof(tclb::PackOp); }
int tclb_loop_sizeof_series() { return (int)sizeof(tclb::SeriesEntry); }
int tclb_dist_sizeof_op() { return (int)sizeof(tclb::HaloOp); }
int tclb_loop_sizeof_seg() { return (int)sizeof(tclb::SegOp); }
int tclb_loop_sizeof_mirror() { return (int)sizeof(tclb::MirrorSpec); }

}  // extern "C"
