// CPU side of the native action loop (tclb_rt/dist_loop.hpp), for the OpenMP executor:
// the same loop, stage kinds, per-step services and halo plan as the GPU build, with two
// transports —
//   * transport 0: this rank is its own neighbour, the plan's sends and receives are
//     paired in order and copied (memcpy);
//   * transport 2: callbacks execute one phase's ops and the particle-force all-reduce
//     (tclb_amd/parallel/native.py runs them as torch.distributed gloo operations between
//     CPU ranks).
// The executor's launches are synchronous, so an exchange completes inside xstart().
#include <math.h>
#include <string.h>

#include "tclb_rt/ad_loop.hpp"
#include "tclb_rt/dist_loop.hpp"

extern "C" int tclb_part_build_grid_cpu(const double*, int, int*, int, int, int, int, int);
extern "C" int tclb_part_build_tree_cpu(const double*, int, int*, int, double);
extern "C" void tclb_part_nan_to_zero_cpu(double*, int);
extern "C" void tclb_part_rigid_step_cpu(double*, const double*, const double*, const unsigned char*, int, double,
                                         double, double, int, double, double, double);

namespace {

typedef int (*xchg_fn)(void* user, void* base, void* staging, const tclb::HaloOp* ops, int nops);
typedef int (*allred_fn)(void* user, double* a, long long n);

struct CpuSvc {
  int prec;
  tclb::run_fn runf;
  tclb::sample_fn samplef;
  int transport;
  int rank;
  xchg_fn cb;
  allred_fn ared;
  void* user;
  int es;
  long long fs, sz, sy;
  int px;

  int run(tclb::Launch& L) { return runf(&L, prec); }
  int sample(tclb::Launch& L, const tclb::SamplePlan& P) { return samplef ? samplef(&L, prec, &P) : 0; }

  int copy_runs(void* dst, const void* src, const tclb::LoopPlan& P, const tclb::StagePlan& st) {
    for (int i = 0; i < st.nruns; i++) {
      const int r0 = P.runs[2 * (st.run0 + i)], r1 = P.runs[2 * (st.run0 + i) + 1];
      const long long off = (long long)r0 * P.fs_bytes;
      memcpy((char*)dst + off, (const char*)src + off, (size_t)((long long)(r1 - r0) * P.fs_bytes));
    }
    return 0;
  }

  int p2p(char* base, char* stg, const tclb::HaloOp* ops, int nops) {
    if (nops == 0) return 0;
    if (transport == 2) return cb ? cb(user, base, stg, ops, nops) : -4;
    return tclb::dist_self_pairs(base, stg, ops, nops, rank, [](char* d, const char* s, long long b) {
      memcpy(d, s, (size_t)b);
      return 0;
    });
  }

  void packs(char* base, char* stg, const tclb::PackOp* pk, int n, int unpack) {
    for (int i = 0; i < n; i++) {
      const tclb::PackOp& o = pk[i];
      if (o.unpack != unpack) continue;
      char* b = stg + o.boff;
      const size_t row = (size_t)px * es;
      for (int f = 0; f < o.nfield; f++)
        for (int z = 0; z < o.nz; z++)
          for (int y = 0; y < o.ny; y++) {
            char* a = base + ((long long)(o.field0 + f) * fs + (long long)(o.z0 + z) * sz +
                              (long long)(o.y0 + y) * sy) * es;
            char* q = b + (((long long)f * o.nz + z) * o.ny + y) * row;
            if (unpack) memcpy(a, q, row);
            else memcpy(q, a, row);
          }
    }
  }

  void segcopy(char* base, char* stg, const tclb::LoopPlan& P, int s0, int n) {
    for (int i = 0; i < n; i++) {
      const tclb::SegOp& o = P.segs[s0 + i];
      if (o.dir == 0) memcpy(stg + o.dst, base + o.src, (size_t)o.bytes);
      else memcpy(base + o.dst, stg + o.src, (size_t)o.bytes);
    }
  }

  int xstart(char* base, const tclb::LoopPlan& P, const tclb::StagePlan& st, int mirrored) {
    int r;
    char* stg = (char*)P.staging;
    if (!mirrored) segcopy(base, stg, P, st.seg0, st.npack);
    if ((r = p2p(base, stg, P.ops + st.op0, st.nops)) != 0) return r;
    segcopy(base, stg, P, st.seg0 + st.npack, st.nunpack);
    if (st.nopsb > 0) {
      packs(base, stg, P.packs + st.pk0, st.npk, 0);
      if ((r = p2p(base, stg, P.ops + st.opb0, st.nopsb)) != 0) return r;
      packs(base, stg, P.packs + st.pk0, st.npk, 1);
    }
    return 0;
  }
  int xfinish() { return 0; }
  void* fork() { return nullptr; }      // one synchronous executor: nothing to fork

  int series(const tclb::LoopPlan& P, int iter) {
    for (int i = 0; i < P.nseries; i++) {
      const tclb::SeriesEntry& e = P.series[i];
      const int k = iter % e.len;
      P.zonal[e.idx] = P.svals[e.off + k];
      if (e.len > 1) P.zonal[e.dtidx] = P.sslopes[e.off + k];
    }
    return 0;
  }

  int part_pre(tclb::Launch& L, const tclb::LoopPlan& P) {
    const tclb::PartPlan& q = *P.part;
    memset(q.acc, 0, sizeof(double) * 6 * (size_t)(q.n > 0 ? q.n : 1));
    if (q.container == 1) tclb_part_build_grid_cpu(q.P, q.n, q.grid, q.gdim[0], q.gdim[1], q.gdim[2], q.cell, q.ncell);
    else if (q.container == 2) tclb_part_build_tree_cpu(q.P, q.n, q.grid, q.nl, q.mscale);
    L.ext[2] = q.P;
    L.ext[3] = q.acc;
    L.next[2] = q.n;
    L.ext[4] = q.container ? q.grid : nullptr;
    L.next[4] = q.container ? q.grid_n : 0;
    return 0;
  }

  int part_post(tclb::Launch& L, const tclb::LoopPlan& P, int step) {
    const tclb::PartPlan& q = *P.part;
    const int na = 6 * q.n;
    if (q.allreduce && transport == 2 && na > 0) {
      const int r = ared ? ared(user, q.acc, na) : -4;
      if (r != 0) return r;
    }
    tclb_part_nan_to_zero_cpu(q.acc, na);
    L.next[2] = 0;
    L.ext[4] = nullptr;
    L.next[4] = 0;
    if (step && q.integrate && q.n > 0)
      tclb_part_rigid_step_cpu(q.P, q.acc, q.m, q.free_, q.n, q.a[0], q.a[1], q.a[2], q.periodic, q.period[0],
                               q.period[1], q.period[2]);
    return 0;
  }
};

}  // namespace

extern "C" {

int tclb_loop_iterate_cpu(const tclb::Launch* L, int prec, int es, int nsteps, int glob_last, int init,
                          const tclb::LoopPlan* P, int transport, int rank, xchg_fn cb, allred_fn ared, void* user,
                          tclb::run_fn run, tclb::sample_fn sample) {
  CpuSvc sv{prec, run, sample, transport, rank, cb, ared, user, es, L->fs, L->sz, L->sy, L->px};
  return tclb::action_loop(sv, *L, nsteps, glob_last, *P, init);
}

// the reverse sweep of one checkpoint segment (tclb_rt/ad_loop.hpp), OpenMP AD executor
int tclb_ad_segment_cpu(const tclb::Launch* L, const tclb::AdSegPlan* P, tclb::ad_run_fn run) {
  return tclb::ad_segment(*L, *P, run, [](void* p, long long b) {
    memset(p, 0, (size_t)b);
    return 0;
  });
}
int tclb_ad_sizeof_seg_cpu() { return (int)sizeof(tclb::AdSegPlan); }

int tclb_loop_sizeof_plan_cpu() { return (int)sizeof(tclb::LoopPlan); }
int tclb_loop_sizeof_stage_cpu() { return (int)sizeof(tclb::StagePlan); }
int tclb_loop_sizeof_part_cpu() { return (int)sizeof(tclb::PartPlan); }
int tclb_loop_sizeof_pack_cpu() { return (int)sizeof(tclb::PackOp); }
int tclb_loop_sizeof_series_cpu() { return (int)sizeof(tclb::SeriesEntry); }
int tclb_dist_sizeof_op_cpu() { return (int)sizeof(tclb::HaloOp); }
int tclb_loop_sizeof_seg_cpu() { return (int)sizeof(tclb::SegOp); }
int tclb_loop_sizeof_mirror_cpu() { return (int)sizeof(tclb::MirrorSpec); }

}  // extern "C"
