// tclb_amd — core device/host definitions shared by every model kernel.
//
// One source, two drivers: every model's node code is compiled once by hipcc for
// gfx950 (GPU executor, see executor_hip.hpp) and once by g++ (OpenMP CPU executor,
// see executor_cpu.hpp).  This replaces the reference's cross.h CUDA/HIP/CPU macro
// shim (reference: src/cross.h:57-346) with two explicit executors and no CUDA path.
#pragma once
#include <stdint.h>
#include <math.h>
#include <stddef.h>
#include <type_traits>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define TCLB_FN __host__ __device__ __forceinline__
#define TCLB_DEV __device__ __forceinline__
#define TCLB_GPU 1
#else
#define TCLB_FN inline
#define TCLB_DEV inline
#define TCLB_GPU 0
#endif

#define TCLB_UNROLL _Pragma("unroll")
#define TCLB_MIRROR_FIELDS 128   // halo-mirror slot table size (Launch.mslot); models have <= 109 fields
// Globals accumulate into TCLB_GSLOTS slots of gstride(NG) doubles (one or more 128-B
// lines each): block b adds into slot b % TCLB_GSLOTS, so the per-block atomics of a
// launch spread over 64 addresses per global instead of queueing on one (the host sums
// and max-reduces the slots, lattice.py _reduce_globals; ops/abi.py GSLOTS).
#define TCLB_GSLOTS 64

namespace tclb {

TCLB_FN constexpr int gstride(int ng) { return (ng + 15) / 16 * 16; }

// Work-group of the LDS-tile stage kernel (executor_hip.hpp k_tile): 64 x 4 nodes, one
// wave per row (z planes per work-group: Model::tile_zc)
constexpr int TILE_BX = 64, TILE_BY = 4;

typedef uint32_t flag_t;  // node type word (reference: flag_t 16/32 bit, src/conf.R:620-628)

template <class R>
struct vec3 {
  R x, y, z;
};

// Launch descriptor.  POD, mirrored field-for-field by tclb_amd/ops/abi.py (ctypes).
// Layout of one snapshot: storage_t[nfields][nz+2gz][ny+2gy][px], x fastest (SoA, like
// the reference's field-major margin blocks, src/conf.R:952-957) but with contiguous
// ghost planes on the decomposed axis instead of 27 margin blocks.
// Launch.glob bit: no zone has a nonzero objective weight (<global>InObj), so AddTo<global>
// skips the weighted Objective sum and its per-node zonal-table reads (a scalar branch).
#define TCLB_GLOB_NOOBJ 4
struct Launch {
  const void* in;          // input snapshot base
  void* out;               // output snapshot base
  const void* flags;       // flag_t, same node indexing as one field (incl. ghosts)
  const double* settings;  // [NSETTINGS] global settings
  const double* zonal;     // [NZSETTINGS][nzones]
  double* globals;         // [NGLOBALS] accumulators (atomic)
  void* aux;               // quantity output / misc pointer
  void* stream;            // hipStream_t (GPU) or unused
  long long sy, sz, fs;    // strides: y, z, field (elements)
  int nx, ny, nz, px;      // local interior size + x pitch
  int gy, gz;              // ghost depth along y / z
  int x0, y0, z0;          // global offset of local (0,0,0)
  int gnx, gny, gnz;       // global lattice size
  int xlo, xhi, ylo, yhi, zlo, zhi;  // box of nodes to process (local coords)
  int iter;                // iteration counter (Time)
  int nzones;              // zone pitch of the zonal table
  int stage;               // stage index (see model meta)
  int glob;                // bit 0: integrate globals; bit 2 (TCLB_GLOB_NOOBJ): every
                           // <global>InObj weight is zero, the Objective sum is skipped
  int quantity;            // quantity index for get-quantity launches
  int qcomp;               // component stride of vector quantities (elements)
  double qscale;           // unit scale for quantity output
  long long qsy, qsz;      // quantity buffer strides (box-relative)
  int block_x, block_y;    // launch shape hint (GPU)
  int reserved0, reserved1;
  // extension slots (model services): 0 = synthetic-turbulence modes, 1 = cuts (uint16
  // [26][field]), 2 = particles (double[npart][PART_STRIDE]), 3 = particle forces
  // accumulator (double[npart][6]), 4,5 = model-specific
  const void* ext[6];
  long long next[6];       // element counts of the ext slots
  double time_shift;       // synthetic-turbulence time wave number (Lattice.set_turbulence)
  int storage_shift;       // 1: reduced-precision storage keeps f - shift(field) (see below)
  int reserved2;
  // Halo mirror (border launches of the overlapped slab step, tclb_amd/lattice.py): every
  // stored field fi with mslot[fi] >= 0 is also written to
  // mbase[mslot[fi] * mfs + x + msy * (y + moy) + msz * (z + moz)] — the packed send
  // buffer of the neighbour exchange, or the wrapped ghost planes of this snapshot —
  // so no separate pack kernel reads the border planes back.  mbase = null: off.
  void* mbase;
  long long mfs, msy, msz;
  int moy, moz;
  signed char mslot[TCLB_MIRROR_FIELDS];
  // Tile windows (GPU): log2 of the number of contiguous tile ranges the work-groups are
  // dealt over (executor_hip.hpp tile_id); 0 = the hardware's linear block order
  int tile_split;
  // identity of the node types behind `flags` (process-unique, changed whenever they change:
  // Lattice.flags_version); keys the per-class tile lists of split stages (executor_hip.hpp)
  int flags_gen;
};

// Zonal-table read (reference ZoneSettings, one value per zone): the zone comes from the
// node's flags, so a plain indexed load is a per-lane vector load that each use waits on
// (seen as chains of global_load_dwordx2 + s_waitcnt vmcnt(0) in the pf_velocity
// collision).  On the GPU the value of the zone of the wave's first lane is fetched by a
// scalar load (s_load: constant cache, short latency; a read, the table is never written
// by a kernel); only lanes of another zone issue the vector load, and a wave with a single
// zone (nearly all of them) skips it.  Build variant "zscal" (-DTCLB_ZONAL_SCALAR=1); the
// default keeps the plain load: on pf384 mixed-shift the scalar reads measured 1 % slower
// (profiles/README.md r03j), the zonal loads are not what limits that kernel.
#ifndef TCLB_ZONAL_SCALAR
#define TCLB_ZONAL_SCALAR 0
#endif
TCLB_FN double zonal_read(const Launch& L, int k, int zone) {
#if TCLB_GPU && defined(__HIP_DEVICE_COMPILE__) && TCLB_ZONAL_SCALAR
  const int z0 = __builtin_amdgcn_readfirstlane(zone);
  // the address is wave-uniform by construction (k is a constant of the emitted accessor,
  // z0 and L are uniform); readfirstlane of its halves lets the backend keep it in SGPRs
  // where its divergence analysis cannot tell (e.g. inside the AD node)
  const unsigned long long a = (unsigned long long)(L.zonal + ((long long)k * L.nzones + z0));
  // (readfirstlane returns int: go through unsigned, or a low word >= 2^31 would be
  // sign-extended into the high word)
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)a);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(a >> 32));
  const unsigned long long au = (unsigned long long)lo | ((unsigned long long)hi << 32);
  double r;
  asm("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(au));
  if (zone != z0) r = L.zonal[(long long)k * L.nzones + zone];
  return r;
#else
  return L.zonal[(long long)k * L.nzones + zone];
#endif
}

template <class S>
TCLB_FN void mirror_store(const Launch& L, int fi, int x, int y, int z, S v) {
  const int s = L.mslot[fi];
  if (s >= 0)
    ((S*)L.mbase)[(long long)s * L.mfs + x + L.msy * (long long)(y + L.moy) + L.msz * (long long)(z + L.moz)] = v;
}

// Reduced-precision storage (reference --with-storage=float|half[-shift],
// src/configure.ac:213-233, src/LatticeAccess.inc.cpp.Rt:14-35).  A density is stored as
// f_i - w_i (w_i: the rest equilibrium of its lattice, Model::field_shift) when
// Launch.storage_shift is set, so fp32/fp16 keep the relative precision of the small
// deviation from rest instead of that of f_i ~ w_i.  Applied only when the storage type
// is narrower than double.  half_t: IEEE binary16 (native _Float16 in hipcc; a bit-exact
// round-to-nearest-even software conversion for the g++ CPU executor).
#if TCLB_GPU
typedef _Float16 half_t;
#else
struct half_t {
  uint16_t b;
  half_t() = default;
  half_t(double d) : b(from_float((float)d)) {}
  operator double() const { return (double)to_float(b); }
  static uint16_t from_float(float f) {
    uint32_t x;
    __builtin_memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) return (uint16_t)(sign | 0x7c00u | (ax > 0x7f800000u ? 0x200u : 0u));
    if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);   // rounds to >= 65520: inf
    if (ax < 0x38800000u) {                                     // subnormal half (or zero)
      if (ax < 0x33000000u) return (uint16_t)sign;
      const uint32_t e = ax >> 23, m = (ax & 0x7fffffu) | 0x800000u;
      const uint32_t s = 126u - e;                               // 14..24
      uint32_t h = m >> s;
      const uint32_t rem = m & ((1u << s) - 1u), half = 1u << (s - 1u);
      if (rem > half || (rem == half && (h & 1u))) h++;
      return (uint16_t)(sign | h);
    }
    uint32_t h = ((ax - 0x38000000u) >> 13);
    const uint32_t rem = ax & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return (uint16_t)(sign | h);
  }
  static float to_float(uint16_t h) {
    const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu, x;
    if (e == 0) {
      if (m == 0) x = sign;
      else {
        e = 113;
        while (!(m & 0x400u)) { m <<= 1; e--; }
        x = sign | (e << 23) | ((m & 0x3ffu) << 13);
      }
    } else if (e == 31) x = sign | 0x7f800000u | (m << 13);
    else x = sign | ((e + 112u) << 23) | (m << 13);
    float f;
    __builtin_memcpy(&f, &x, 4);
    return f;
  }
};
#endif

// Periodic wrap helper for non-decomposed axes.
TCLB_FN int wrap(int v, int n) { return v < 0 ? v + n : (v >= n ? v - n : v); }

// ---------------------------------------------------------------------------
// Node addressing.  Offsets inside one field are 32-bit (a field is < 2^31
// elements: 1290^3 nodes); field bases are uniform 64-bit values so that loads
// lower to SGPR-base + VGPR-offset addressing on gfx950.
// ---------------------------------------------------------------------------
struct Addr {
  int x, y, z;  // local coordinates
  int node;     // offset of (x,y,z) inside a field
  int nx, ny, nz, gy, gz, sy, sz;
  TCLB_FN void init(const Launch& L, int x_, int y_, int z_) {
    x = x_; y = y_; z = z_;
    nx = L.nx; ny = L.ny; nz = L.nz; gy = L.gy; gz = L.gz;
    sy = (int)L.sy; sz = (int)L.sz;
    node = x + sy * (y + gy) + sz * (z + gz);
  }
  // x part (lane-varying on the GPU: a wave is 64 consecutive x of one row) and y/z part
  // (wave-uniform there: the executors pass y and z through readfirstlane) of off()
  TCLB_FN int xo(int dx) const {
#ifdef TCLB_DEBUG_NO_XSHIFT
    dx = 0;  // diagnostic build only: aligned-x ceiling of the access pattern (wrong physics)
#endif
    return dx == 0 ? x : wrap(x + dx, nx);
  }
  TCLB_FN int yzo(int dy, int dz) const {
    int yy = y + dy;
    if (dy != 0 && gy == 0) yy = wrap(yy, ny);
    int zz = z + dz;
    if (dz != 0 && gz == 0) zz = wrap(zz, nz);
    return sy * (yy + gy) + sz * (zz + gz);
  }
  TCLB_FN int off(int dx, int dy, int dz) const { return xo(dx) + yzo(dy, dz); }
};

// Element x of a row whose (uniform) start is `row`: on the GPU the row pointer lives in
// SGPRs and the lane's x goes in as a 32-bit zero-extended byte offset, so every access is
// one global_load/store with SGPR base + VGPR offset (saddr form) and the few distinct x
// offsets of a stencil (x-1, x, x+1) are shared by all fields; with the whole offset in a
// sign-extended int each access needed its own 64-bit VGPR address (two VGPRs and a
// v_lshl_add_u64 per load; 84 of them in the pf_velocity collide).  x < 2^28: a row is
// shorter than a field.
// TCLB_FLAT_NODE=1: the emitted node accessors take the flat form (one offset per access)
// in every instantiation, the globals kernels included (the GPU adjoint build defines it,
// build.py _adhip_source; emitter Node::ROWA_)
#ifndef TCLB_FLAT_NODE
#define TCLB_FLAT_NODE 0
#endif
// Which instantiations take the row form (ROW = true; the emitted Node passes ROWA_):
// the globals-integrating (GLOB) stage kernels, where it keeps the accumulators' kernel
// at 2 waves/SIMD (profiles/README.md r03o: +0.9 % instead of +11 % pf384 mixed-shift
// with globals on every step); the plain kernels, the bulk of a run, take the 64-bit
// flat address (row + x), which measured faster on the d3q27 headline (profiles/README.md
// r04b/r04c, two boxes: +0.7-1.5 % fp64, +1.4-2 % mixed-shift).  TCLB_ROW_ADDR=0: flat
// everywhere; TCLB_ROW_ADDR_PLAIN=1: the row form everywhere (the round-3 default).
#ifndef TCLB_ROW_ADDR
#define TCLB_ROW_ADDR 1
#endif
#ifndef TCLB_ROW_ADDR_PLAIN
#define TCLB_ROW_ADDR_PLAIN 0
#endif
template <bool ROW, class T>
TCLB_FN T* row_at(T* row, int x) {
#if TCLB_GPU && defined(__HIP_DEVICE_COMPILE__)
  if constexpr (ROW) {
    typedef typename std::conditional<std::is_const<T>::value, const char, char>::type C;
    return (T*)((C*)row + (unsigned)(x * (int)sizeof(T)));
  }
#endif
  return row + x;
}

// Streaming loads/stores.  Every population is read once and written once per step,
// so non-temporal hints keep the 4 MB/XCD L2 for the x-misaligned neighbour lines.
// Selected at build time (-DTCLB_NT_LOAD=1 / -DTCLB_NT_STORE=1), A/B-tested on MI355X.
#ifndef TCLB_NT_LOAD
#define TCLB_NT_LOAD 0
#endif
#ifndef TCLB_NT_STORE
#define TCLB_NT_STORE 0
#endif
template <class T>
TCLB_FN T load_stream(const T* p) {
#if TCLB_GPU && TCLB_NT_LOAD && defined(__HIP_DEVICE_COMPILE__)
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}
template <class T>
TCLB_FN void store_stream(T* p, T v) {
#if TCLB_GPU && TCLB_NT_STORE && defined(__HIP_DEVICE_COMPILE__)
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

// ---------------------------------------------------------------------------
// Particles coupled to the lattice (reference Particle.hpp / RemoteForceInterface).
// Device record (double): pos[3] vel[3] angvel[3] rad  -> PART_STRIDE = 10, in Launch.ext[2];
// force/moment accumulators double[n][6] in Launch.ext[3] (Launch.next[3] copies on the GPU,
// particle_acc).
// ---------------------------------------------------------------------------
constexpr int PART_STRIDE = 10;

template <class R>
struct ParticleS {
  vec3<R> cvel, diff, force, moment;
  R rad, dist;
  int i;
  TCLB_FN void init(const double* P, int i_, R x, R y, R z) {
    i = i_;
    const double* p = P + (long long)i * PART_STRIDE;
    rad = R(p[9]);
    diff.x = x - R(p[0]); diff.y = y - R(p[1]); diff.z = z - R(p[2]);
    dist = sqrt(diff.x * diff.x + diff.y * diff.y + diff.z * diff.z);
    const R wx = R(p[6]), wy = R(p[7]), wz = R(p[8]);
    cvel.x = R(p[3]) + wy * diff.z - wz * diff.y;
    cvel.y = R(p[4]) + wz * diff.x - wx * diff.z;
    cvel.z = R(p[5]) + wx * diff.y - wy * diff.x;
    force.x = force.y = force.z = R(0);
    moment.x = moment.y = moment.z = R(0);
  }
  TCLB_FN bool in() const { return dist < rad; }
  TCLB_FN void applyForce(vec3<R> f) {
    force.x += f.x; force.y += f.y; force.z += f.z;
    moment.x -= f.y * diff.z - f.z * diff.y;
    moment.y -= f.z * diff.x - f.x * diff.z;
    moment.z -= f.x * diff.y - f.y * diff.x;
  }
};

// A particle is certainly out of reach of node (x, y, z) — farther than its cut-off
// rad + 2 (ParticleLoop / ParticleScan) — by an fp32 squared distance against a cut-off
// widened by 1 % + 1 node: fp32 rounding of the coordinates (|x| < 2^24) cannot flip a
// node inside the exact fp64 test to "far".  The exact test follows for the rest.
TCLB_FN bool particle_far(const double* P, int i, int x, int y, int z) {
  const double* p = P + (long long)i * PART_STRIDE;
  const float dx = (float)x - (float)p[0], dy = (float)y - (float)p[1], dz = (float)z - (float)p[2];
  const float c = (float)p[9] * 1.01f + 3.0f;
  return dx * dx + dy * dy + dz * dz > c * c;
}

// The accumulator copy a node adds into: Launch.next[3] copies of the [n][6] block (0 or 1:
// one), picked by the work-group on the GPU — the nodes a particle covers all add to the
// same 6 doubles, and one copy serialised those atomics (the part256 force stage ran
// 110-140 us of which ~20 us are its stores; profiles/README.md r06).  The copies are
// summed into the first after the stage (tclb_part_acc_slots).
TCLB_FN double* particle_acc(const Launch& L) {
  double* acc = (double*)L.ext[3];
#if TCLB_GPU && defined(__HIP_DEVICE_COMPILE__)
  const long long k = L.next[3];
  if (acc != nullptr && k > 1) {
    const unsigned b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    acc += (long long)(b % (unsigned)k) * L.next[2] * 6;
  }
#endif
  return acc;
}

// Flush one particle's force/moment contribution of this node.  On the GPU, when the
// whole wavefront is active the 6 values are reduced across the wave first (one atomic
// per value per wave, reference WARP_SYNC); otherwise each contributing lane adds.
template <class R>
TCLB_FN void particle_flush(double* acc, const ParticleS<R>& p) {
  double v[6] = {(double)p.force.x, (double)p.force.y, (double)p.force.z,
                 (double)p.moment.x, (double)p.moment.y, (double)p.moment.z};
  double* a = acc + (long long)p.i * 6;
#if TCLB_GPU && defined(__HIP_DEVICE_COMPILE__)
  const unsigned long long act = __ballot(1);
  // wave reduction only when every lane is active on the same particle (grid candidate
  // lists differ between lanes of different cells)
  if (act == ~0ull && __all(p.i == __shfl(p.i, 0, 64))) {
    const int lane = __lane_id();
    TCLB_UNROLL for (int k = 0; k < 6; k++) {
      double s = v[k];
      TCLB_UNROLL for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (lane == 0 && s != 0.0) unsafeAtomicAdd(a + k, s);
    }
  } else {
    TCLB_UNROLL for (int k = 0; k < 6; k++)
      if (v[k] != 0.0) unsafeAtomicAdd(a + k, v[k]);
  }
#else
  for (int k = 0; k < 6; k++)
    if (v[k] != 0.0) {
#pragma omp atomic
      a[k] += v[k];
    }
#endif
}

// Probe plan of the Sampler (reference src/Sampler.cpp:66-80, Lattice::updateAllSamples
// src/Lattice.cu.Rt:1376-1389): after every step the nq quantities are evaluated at np
// points (local coordinates) into out[row][np][width] (double, unit-scaled), so a whole
// callback interval is recorded on the device and copied to the host once.  One launch
// per step covers every point and quantity (the reference launches one per point and
// quantity).
constexpr int SAMPLE_MAXQ = 32;
struct SamplePlan {
  const int* points;   // device int[np][3]
  double* out;         // device double[rows][np][width]
  int np, width;       // points, values per point (sum of ncomp)
  int row, rows;       // row written after the first step of a call / capacity
  int nq;
  int q[SAMPLE_MAXQ], ncomp[SAMPLE_MAXQ], offset[SAMPLE_MAXQ];
  double scale[SAMPLE_MAXQ];
};

// one probe of node n into o[width] (shared by both executors)
template <class NodeT>
TCLB_FN void sample_node(NodeT& n, const SamplePlan& P, double* o) {
  n.pop();
  for (int i = 0; i < P.nq; i++) {
    typename NodeT::real_t v[3] = {0, 0, 0};
    n.get_quantity(P.q[i], v);
    for (int c = 0; c < P.ncomp[i]; c++) o[P.offset[i] + c] = (double)v[c] * P.scale[i];
  }
}

// Multi-step driver: nsteps of one action (stage list) with A/B snapshot swapping and no
// host round trip per step (reference Lattice::Iterate, src/Lattice.cu.Rt:900-989).  Used
// when no halo exchange is needed between stages (one rank, periodic wrap in-kernel);
// globals are integrated on the last step only when glob_last is set.  L.in holds the
// current snapshot and L.out the other one on entry.  With a sample plan the probes of
// every step are recorded (row sp->row + s) after the step.
template <class Run, class Sample>
inline int iterate_action(Launch L, int nsteps, const int* stages, int nstages, int glob_last,
                          const SamplePlan* sp, Run run, Sample sample) {
  const void* cur = L.in;
  void* nxt = L.out;
  const int gflags = L.glob & ~1;
  for (int s = 0; s < nsteps; s++) {
    for (int k = 0; k < nstages; k++) {
      L.in = k == 0 ? cur : nxt;
      L.out = nxt;
      L.stage = stages[k];
      L.glob = (glob_last && s == nsteps - 1) ? (1 | gflags) : 0;
      const int r = run(L);
      if (r != 0) return r;
    }
    L.iter += 1;
    L.reserved1 += 1;
    void* t = (void*)cur;
    cur = nxt;
    nxt = t;
    if (sp != nullptr && sp->np > 0 && sp->row + s < sp->rows) {
      Launch Q = L;
      Q.in = cur;
      Q.out = nxt;
      Q.glob = 0;
      Q.reserved1 = L.reserved1 > 2 ? L.reserved1 - 1 : 1;   // quantity averaging count
      SamplePlan P = *sp;
      P.row = sp->row + s;
      const int r = sample(Q, P);
      if (r != 0) return r;
    }
  }
  return 0;
}

// Precision codes of the C ABI (mirrored by ops/abi.py PREC):
//   0 fp64 compute / fp64 storage (reference default, src/configure.ac:208-211)
//   1 fp32 compute / fp32 storage
//   2 fp64 compute / fp32 storage (reference --with-storage=float[-shift])
//   3 fp32 compute / fp16 storage (reference --with-storage=half[-shift])
// the *-shift variants are the same instantiations with Launch.storage_shift = 1.
template <class R_, class S_>
struct prec_tag {
  typedef R_ R;
  typedef S_ S;
};
template <class F>
inline int prec_dispatch(int prec, F&& f) {
  switch (prec) {
    case 0: return f(prec_tag<double, double>{});
    case 1: return f(prec_tag<float, float>{});
    case 2: return f(prec_tag<double, float>{});
    case 3: return f(prec_tag<float, half_t>{});
    default: return -1;
  }
}

// C exports common to both executors (each defines tclb::exec::run_stage, run_quantity
// and run_sample for its device).
#define TCLB_EXPORT_COMMON(NAME, MODEL)                                                       \
  extern "C" int tclb_##NAME##_run(const tclb::Launch* L, int prec) {                         \
    return tclb::prec_dispatch(prec, [&](auto t) {                                            \
      using T = decltype(t);                                                                  \
      return tclb::exec::run_stage<MODEL, typename T::R, typename T::S>(*L);                  \
    });                                                                                       \
  }                                                                                           \
  extern "C" int tclb_##NAME##_quantity(const tclb::Launch* L, int prec) {                    \
    return tclb::prec_dispatch(prec, [&](auto t) {                                            \
      using T = decltype(t);                                                                  \
      return tclb::exec::run_quantity<MODEL, typename T::R, typename T::S>(*L);               \
    });                                                                                       \
  }                                                                                           \
  extern "C" int tclb_##NAME##_iterate(const tclb::Launch* L, int prec, int n, const int* stages, \
                                        int nstages, int glob_last, const tclb::SamplePlan* sp) { \
    return tclb::prec_dispatch(prec, [&](auto t) {                                            \
      using T = decltype(t);                                                                  \
      return tclb::iterate_action(                                                            \
          *L, n, stages, nstages, glob_last, sp,                                              \
          [](const tclb::Launch& l) { return tclb::exec::run_stage<MODEL, typename T::R, typename T::S>(l); }, \
          [](const tclb::Launch& l, const tclb::SamplePlan& p) {                              \
            return tclb::exec::run_sample<MODEL, typename T::R, typename T::S>(l, p);         \
          });                                                                                 \
    });                                                                                       \
  }                                                                                           \
  extern "C" int tclb_##NAME##_sample(const tclb::Launch* L, int prec, const tclb::SamplePlan* P) { \
    return tclb::prec_dispatch(prec, [&](auto t) {                                            \
      using T = decltype(t);                                                                  \
      return tclb::exec::run_sample<MODEL, typename T::R, typename T::S>(*L, *P);             \
    });                                                                                       \
  }                                                                                           \
  extern "C" int tclb_##NAME##_sizeof_sample_plan() { return (int)sizeof(tclb::SamplePlan); } \
  extern "C" int tclb_##NAME##_sizeof_launch() { return (int)sizeof(tclb::Launch); }

// Globals accumulation of one node (the emitted AddTo<global>).  `g` is the executor's
// accumulator array: per-thread registers on the CPU and in the AD executors; on the GPU
// primal executor a block-shared LDS array (executor_hip.hpp stage_body), so the GLOB
// instantiation keeps no NG-long accumulator live through the node (pf_velocity: 33
// globals = 66 VGPRs, 266 VGPRs in all, 1 wave/SIMD; profiles/README.md r03j).  The LDS
// add is a wave reduction (DPP, -amdgpu-atomic-optimizer-strategy=DPP: correct under
// divergence) and one ds_add/ds_max per wave.  __builtin_amdgcn_is_shared folds at
// compile time once the accumulator's address space is known.
// Accumulator type of the globals (the node's glob_ array): fp64 for the plain compute
// types, so an fp32-compute run sums its globals in double like the reference's
// double-precision reduction; the type itself for the AD dual numbers.
template <class R>
struct glob_acc {
  typedef R type;
};
template <>
struct glob_acc<float> {
  typedef double type;
};

template <class G, class R>
TCLB_FN void glob_add(G* g, int i, R v) {
#if TCLB_GPU && defined(__HIP_DEVICE_COMPILE__)
  if constexpr (std::is_same<G, double>::value || std::is_same<G, float>::value) {
    if (__builtin_amdgcn_is_shared((const void*)g)) {
      __hip_atomic_fetch_add(g + i, G(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return;
    }
  }
#endif
  g[i] += G(v);
}
template <class G, class R>
TCLB_FN void glob_max(G* g, int i, R v) {
#if TCLB_GPU && defined(__HIP_DEVICE_COMPILE__)
  if constexpr (std::is_same<G, double>::value || std::is_same<G, float>::value) {
    if (__builtin_amdgcn_is_shared((const void*)g)) {
      __hip_atomic_fetch_max(g + i, G(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return;
    }
  }
#endif
  const G w = G(v);
  g[i] = g[i] > w ? g[i] : w;
}

template <class T>
TCLB_FN T tmax(T a, T b) { return a > b ? a : b; }
template <class T>
TCLB_FN T tmin(T a, T b) { return a < b ? a : b; }

}  // namespace tclb
