// LDS A/B for the 27-point stencil reads of the multiphase models (the PhaseF / psi
// gradient and Laplacian stencils of d3q27_pf_velocity calcPhase/calcWall, d3q27_PSM,
// d2q9_ShanChen): one weighted 27-point sum over a periodic n^3 fp64 field.
//
//   mode 0: direct global loads, one thread per node (what the model kernels do; the
//           x+-1 / y+-1 / z+-1 neighbour lines are served by L2)
//   mode 1: LDS tile (BX+2) x (BY+2) per plane, a 3-plane ring marching ZC planes in z
//           per work-group: every element is read from HBM/L2 about (1+2/BY)(1+2/ZC)
//           times instead of through 27 cached loads
//
// Host-side shape checks: n must be a multiple of BX, BY and ZC (returns -1 otherwise).
#include <hip/hip_runtime.h>

namespace {

constexpr int BX = 64, BY = 4, ZC = 16;

__device__ __forceinline__ int wrapi(int v, int n) { return v < 0 ? v + n : (v >= n ? v - n : v); }

// D3Q27 Laplacian-like weights by |c|^2 (values are immaterial for the A/B, but the
// same in both modes so the outputs can be compared)
__device__ __forceinline__ double wgt(int dx, int dy, int dz) {
  const int k = dx * dx + dy * dy + dz * dz;
  return k == 0 ? -3.5 : (k == 1 ? 2.0 / 9.0 : (k == 2 ? 1.0 / 18.0 : 1.0 / 72.0));
}

__global__ void __launch_bounds__(256) k_global(const double* __restrict__ in, double* __restrict__ out, int n) {
  const int x = blockIdx.x * BX + threadIdx.x;
  const int y = blockIdx.y * BY + threadIdx.y;
  const int z = blockIdx.z;
  if (x >= n || y >= n || z >= n) return;
  double s = 0.0;
#pragma unroll
  for (int dz = -1; dz <= 1; dz++) {
    const size_t zo = (size_t)wrapi(z + dz, n) * n;
#pragma unroll
    for (int dy = -1; dy <= 1; dy++) {
      const size_t yo = (zo + wrapi(y + dy, n)) * n;
#pragma unroll
      for (int dx = -1; dx <= 1; dx++) s += wgt(dx, dy, dz) * in[yo + wrapi(x + dx, n)];
    }
  }
  out[((size_t)z * n + y) * n + x] = s;
}

__global__ void __launch_bounds__(256) k_lds(const double* __restrict__ in, double* __restrict__ out, int n) {
  __shared__ double tile[3][BY + 2][BX + 2];
  const int tx = threadIdx.x, ty = threadIdx.y;
  const int tid = ty * BX + tx;
  const int x0 = blockIdx.x * BX, y0 = blockIdx.y * BY, z0 = blockIdx.z * ZC;
  auto load_plane = [&](int slot, int z) {
    const size_t zo = (size_t)wrapi(z, n) * n;
    for (int i = tid; i < (BY + 2) * (BX + 2); i += BX * BY) {
      const int ly = i / (BX + 2), lx = i - ly * (BX + 2);
      tile[slot][ly][lx] = in[(zo + wrapi(y0 + ly - 1, n)) * n + wrapi(x0 + lx - 1, n)];
    }
  };
  load_plane(0, z0 - 1);
  load_plane(1, z0);
  for (int k = 0; k < ZC; k++) {
    load_plane((k + 2) % 3, z0 + k + 1);
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int dz = -1; dz <= 1; dz++) {
      const int slot = (k + 1 + dz) % 3;
#pragma unroll
      for (int dy = -1; dy <= 1; dy++)
#pragma unroll
        for (int dx = -1; dx <= 1; dx++) s += wgt(dx, dy, dz) * tile[slot][ty + 1 + dy][tx + 1 + dx];
    }
    out[((size_t)(z0 + k) * n + (y0 + ty)) * n + (x0 + tx)] = s;
    __syncthreads();   // the next iteration overwrites the plane read here
  }
}

}  // namespace

// mode 0/1 as above; runs `reps` launches on `stream` between two events and returns the
// mean ms per launch in *ms.  0 on success, -1 bad shape, else the HIP error code.
extern "C" int tclb_lds_ab_run(int mode, const double* in, double* out, int n, int reps, void* stream, float* ms) {
  if (n <= 0 || n % BX != 0 || n % BY != 0 || n % ZC != 0 || reps <= 0) return -1;
  hipStream_t s = (hipStream_t)stream;
  const dim3 block(BX, BY, 1);
  const dim3 grid(n / BX, n / BY, mode == 0 ? n : n / ZC);
  hipEvent_t a, b;
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return (int)hipGetLastError();
  hipEventRecord(a, s);
  for (int r = 0; r < reps; r++) {
    if (mode == 0) k_global<<<grid, block, 0, s>>>(in, out, n);
    else k_lds<<<grid, block, 0, s>>>(in, out, n);
  }
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float t = 0.f;
  hipEventElapsedTime(&t, a, b);
  *ms = t / (float)reps;
  hipEventDestroy(a);
  hipEventDestroy(b);
  return (int)hipGetLastError();
}
