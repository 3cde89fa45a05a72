// GPU side of the native multi-rank loop (tclb_rt/dist_loop.hpp): a context owning this
// rank's RCCL communicator, a high-priority comm stream and two events, and the
// transports of dist_iterate:
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
#include <string.h>

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
#undef SYM
  return 0;
}

struct Ctx {
  int transport;  // 0 = device copies (loopback), 1 = RCCL
  int nranks, rank;
  Rccl R;
  Comm comm = nullptr;
  hipStream_t cs = nullptr;   // comm stream
  hipEvent_t ready = nullptr, done = nullptr;
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

// one stage's exchange: ordered after the work already on the compute stream ks, on the
// comm stream; finish() orders the compute stream after it
struct GpuX {
  Ctx* c;
  hipStream_t ks;
  int start(char* base, const tclb::HaloOp* ops, int nops) {
    int r;
    if ((r = hip_check(hipEventRecord(c->ready, ks), "hipEventRecord")) != 0) return r;
    if ((r = hip_check(hipStreamWaitEvent(c->cs, c->ready, 0), "hipStreamWaitEvent")) != 0) return r;
    if (c->transport == 1) {
      if ((r = rccl_check(c, c->R.group_start(), "ncclGroupStart")) != 0) return r;
      for (int i = 0; i < nops; i++) {
        const tclb::HaloOp& o = ops[i];
        const int e = o.kind == 0 ? c->R.send(base + o.off, (size_t)o.bytes, 0, o.peer, c->comm, c->cs)
                                  : c->R.recv(base + o.off, (size_t)o.bytes, 0, o.peer, c->comm, c->cs);
        if (e != 0) {
          c->R.group_end();
          return rccl_check(c, e, o.kind == 0 ? "ncclSend" : "ncclRecv");
        }
      }
      if ((r = rccl_check(c, c->R.group_end(), "ncclGroupEnd")) != 0) return r;
    } else {
      r = tclb::dist_self_pairs(base, ops, nops, c->rank, [&](char* d, const char* s, long long b) {
        return hip_check(hipMemcpyAsync(d, s, (size_t)b, hipMemcpyDeviceToDevice, c->cs), "hipMemcpyAsync");
      });
      if (r != 0) {
        if (r == -3) set_err("halo plan", "sends and receives to self do not pair up");
        return r;
      }
    }
    return hip_check(hipEventRecord(c->done, c->cs), "hipEventRecord");
  }
  int finish() { return hip_check(hipStreamWaitEvent(ks, c->done, 0), "hipStreamWaitEvent"); }
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
void* tclb_dist_ctx_create(const char* rccl_path, int transport, int nranks, int rank, const void* uid) {
  Ctx* c = new Ctx();
  c->transport = transport;
  c->nranks = nranks;
  c->rank = rank;
  int lo = 0, hi = 0;
  if (hip_check(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange") != 0 ||
      hip_check(hipStreamCreateWithPriority(&c->cs, hipStreamNonBlocking, hi), "hipStreamCreateWithPriority") != 0 ||
      hip_check(hipEventCreateWithFlags(&c->ready, hipEventDisableTiming), "hipEventCreate") != 0 ||
      hip_check(hipEventCreateWithFlags(&c->done, hipEventDisableTiming), "hipEventCreate") != 0) {
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
  } else if (nranks != 1) {
    set_err("tclb_dist_ctx_create", "the copy transport is single-rank");
    delete c;
    return nullptr;
  }
  return c;
}

void tclb_dist_ctx_destroy(void* ctx) {
  Ctx* c = (Ctx*)ctx;
  if (!c) return;
  if (c->cs) hipStreamSynchronize(c->cs);
  if (c->comm) c->R.comm_destroy(c->comm);
  if (c->ready) hipEventDestroy(c->ready);
  if (c->done) hipEventDestroy(c->done);
  if (c->cs) hipStreamDestroy(c->cs);
  delete c;
}

// the n steps of an action (tclb_rt/dist_loop.hpp); run / sample are the model library's
// tclb_<model>_run / tclb_<model>_sample; launches go to L->stream
int tclb_dist_iterate(void* ctx, const tclb::Launch* L, int prec, int nsteps, int glob_last,
                      const tclb::DistPlan* P, tclb::run_fn run, tclb::sample_fn sample,
                      const tclb::SamplePlan* sp) {
  Ctx* c = (Ctx*)ctx;
  GpuX x{c, (hipStream_t)L->stream};
  int r = tclb::dist_iterate(*L, prec, nsteps, glob_last, *P, x, run, sample, sp);
  if (r == 0 && c->transport == 1) {
    int ae = 0;
    if (c->R.async_error(c->comm, &ae) == 0 && ae != 0) r = rccl_check(c, ae, "RCCL async error");
  }
  return r;
}

// one exchange outside the loop (the Python step path of the same plan)
int tclb_dist_exchange(void* ctx, void* base, const tclb::HaloOp* ops, int nops, void* stream) {
  Ctx* c = (Ctx*)ctx;
  GpuX x{c, (hipStream_t)stream};
  int r = x.start((char*)base, ops, nops);
  return r != 0 ? r : x.finish();
}

int tclb_dist_sizeof_plan() { return (int)sizeof(tclb::DistPlan); }
int tclb_dist_sizeof_op() { return (int)sizeof(tclb::HaloOp); }

}  // extern "C"
