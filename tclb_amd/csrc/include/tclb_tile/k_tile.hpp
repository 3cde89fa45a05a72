// LDS-staged stencil tiles (DSL Stage lds=[fields]; emitter tile tables tile_count /
// tile_field / tile_h / tile_zc).  Included by tclb/executor_hip.hpp inside namespace
// tclb::exec (it uses the block-globals helpers defined there); kept in its own
// directory so that only the libraries of models with LDS-staged stages depend on it
// (build.py _tile_deps).
//
// A stage whose node code reads scalar fields through a 3x3x3 (or wider) stencil issues
// one global load per stencil point: 27+ loads per node per field, served by L1/L2 but
// limited by the TA path at ~2-3 TB/s (profiles/README.md r02f LDS A/B: 1.84 TB/s global
// vs 5.59 TB/s LDS).  k_tile instead marches a 64 x 4 work-group through ZC z planes
// (Model::tile_zc: 16 for stencil-bound stages, 1 for stages that also stream many
// populations): each plane of every staged field is loaded once into an LDS ring of
// (2 hz + 1) planes of (64 + 2 hx) x (4 + 2 hy) elements (about 1.6 global loads per node
// and field), and the node's reads of staged fields (the emitted ld()) come from LDS.
// Reads of other fields and every store stay global.  Results are the same as k_stage's
// (the same node code reading the same values).
//
// The plane loads are software-pipelined: the global loads of plane z + hz + 1 are issued
// into registers before the nodes of plane z run and written to the ring at the start of
// the next step, so their latency hides behind the node code instead of stalling every
// step (the RK stages of pf_velocity_thermo waited 65 % of their time with the
// load -> barrier -> compute order, profiles/README.md r04g).
#ifndef TCLB_LDS_TILES
#define TCLB_LDS_TILES 1
#endif

// occupancy floor of the tile kernels (A/B knob, build variant flag -DTCLB_TILE_WAVES=n)
#ifndef TCLB_TILE_WAVES
#define TCLB_TILE_WAVES 0
#endif
template <class Model, class R, class S, int STG, bool GLOB>
#if TCLB_TILE_WAVES > 0
__global__ void __launch_bounds__(TILE_BX * TILE_BY) __attribute__((amdgpu_waves_per_eu(TCLB_TILE_WAVES)))
#else
__global__ void __launch_bounds__(TILE_BX * TILE_BY)
#endif
k_tile(const Launch L) {
  typedef typename Model::template NodeTile<R, S, GLOB, STG> N;
  typedef typename N::G_ G;
  constexpr int NT = Model::tile_count(STG);
  constexpr int TX = Model::tile_h(STG, 0), TY = Model::tile_h(STG, 1), TZ = Model::tile_h(STG, 2);
  constexpr int W = TILE_BX + 2 * TX, H = TILE_BY + 2 * TY, NP = 2 * TZ + 1;
  constexpr int PLANE = W * H, SLOT = NP * PLANE;
  constexpr int NTH = TILE_BX * TILE_BY;
  constexpr int NL = (PLANE + NTH - 1) / NTH;   // plane elements per thread
  __shared__ S tile[NT * SLOT];
  const int tx = threadIdx.x, ty = threadIdx.y, tid = tx + TILE_BX * ty;
  const uint3 tb = tile_id(L);     // executor_hip.hpp: the block -> tile window map
  const int x0 = L.xlo + (int)tb.x * TILE_BX;
  const int y0 = L.ylo + (int)tb.y * TILE_BY;
  constexpr int ZC = Model::tile_zc(STG);
  const int zb = L.zlo + (int)tb.z * ZC;
  const int ze = zb + ZC < L.zhi ? zb + ZC : L.zhi;
  const int x = x0 + tx;
  const int y = __builtin_amdgcn_readfirstlane(y0 + ty);   // a wave is one row of the tile
  const bool active = x < L.xhi && y < L.yhi;
  const S* in = (const S*)L.in;
  // the (x, y) part of this thread's plane elements, the same for every plane; elements
  // outside the snapshot (beyond a partial block's edge) are zero and never read by an
  // active node
  long long eoff[NL];
  bool eok[NL];
#pragma unroll
  for (int j = 0; j < NL; j++) {
    const int i = tid + j * NTH;
    const int ly = i / W, lx = i - ly * W;
    int xx = x0 - TX + lx, yy = y0 - TY + ly;
    bool ok = i < PLANE && xx < L.nx + TX && xx >= -TX;
    xx = wrap(xx, L.nx);
    if (L.gy == 0) {
      ok = ok && yy >= -TY && yy < L.ny + TY;
      yy = wrap(yy, L.ny);
    } else {
      ok = ok && yy >= -L.gy && yy < L.ny + L.gy;
    }
    eok[j] = ok;
    eoff[j] = (long long)xx + L.sy * (long long)(yy + L.gy);
  }
  S pre[NT][NL];
  // global loads of plane z into registers
  auto fetch = [&](int z) {
    int zz = z;
    bool zok;
    if (L.gz == 0) {
      zok = z >= -L.nz && z < 2 * L.nz;
      zz = wrap(z, L.nz);
    } else {
      zok = z >= -L.gz && z < L.nz + L.gz;
    }
    const long long zo = L.sz * (long long)(zz + L.gz);
#pragma unroll
    for (int j = 0; j < NL; j++)
#pragma unroll
      for (int k = 0; k < NT; k++) {
        const int fi = Model::tile_field(STG, k);
        pre[k][j] = (zok && eok[j]) ? in[(long long)fi * L.fs + eoff[j] + zo] : S(0);
      }
  };
  // the fetched plane z into its ring slot
  auto commit = [&](int z) {
    const int ring = (z - zb + TZ) % NP;
#pragma unroll
    for (int j = 0; j < NL; j++) {
      const int i = tid + j * NTH;
      if (i < PLANE) {
#pragma unroll
        for (int k = 0; k < NT; k++) tile[k * SLOT + ring * PLANE + i] = pre[k][j];
      }
    }
  };
  constexpr int NG = Model::NGLOBALS_ > 0 ? Model::NGLOBALS_ : 1;
  __shared__ G acc[GLOB ? NG : 1];
  if constexpr (GLOB) block_globals_init<NG, Model::NSUMGLOBALS_>(acc);
  G g1[1] = {G(0)};
  for (int z = zb - TZ; z < zb + TZ; z++) {
    fetch(z);
    commit(z);
  }
  fetch(zb + TZ);
  // ZC = 1 (stages whose node code is heavy: a z loop would let the compiler hoist the
  // node's loop-invariant loads, e.g. every setting, and keep them live through the node)
  for (int z = zb; ZC == 1 ? z == zb : z < ze; z++) {
    commit(z + TZ);   // overwrites the slot of plane z - hz - 1, last read in step z - 1
    __syncthreads();
    if (ZC != 1 && z + 1 < ze) fetch(z + 1 + TZ);   // in flight while the nodes run
    if (active) {
      // the LDS accumulators and the private dummy are separate constructions, so the
      // address space of the node's globals pointer stays known (core.hpp glob_add)
      auto run = [&](N& n) {
        n.tile_ = tile;
        n.tix_ = (ty + TY) * W + tx + TX;
#pragma unroll
        for (int d = 0; d < NP; d++) n.tpl_[d] = ((z + d - zb) % NP) * PLANE;
        n.template run_stage<STG>();
      };
      if constexpr (GLOB) {
        N n(L, x, y, z, acc);
        run(n);
      } else {
        N n(L, x, y, z, g1);
        run(n);
      }
    }
    __syncthreads();   // the next commit overwrites a ring slot read here
  }
  if constexpr (GLOB) block_globals_flush<NG, Model::NSUMGLOBALS_>(acc, L.globals);
}
