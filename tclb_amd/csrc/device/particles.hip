// Per-step particle kernels of the device-resident particle system
// (tclb_amd/particles/system.py): one launch each instead of a chain of small tensor ops
// (a step of the in-process SimplePart was ~20 launches and a host->device copy, and the
// GPU idled between them: part256 ran 0.35 ms/step above its kernel time).
//
// Records: P[n][10] = pos[3] vel[3] angvel[3] radius (core.hpp PART_STRIDE), force/moment
// accumulator acc[n][6].  Reference: simplepart.cpp (explicit rigid-sphere update) and
// the NaN-force guard of src/Lattice.cu.Rt:420-435.
#include <hip/hip_runtime.h>
#include <math.h>

namespace {

__global__ void __launch_bounds__(256) k_nan_to_zero(double* a, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && isnan(a[i])) a[i] = 0.0;
}

// torch.remainder semantics (result has the divisor's sign)
__device__ __forceinline__ double wrap(double x, double L) { return x - floor(x / L) * L; }

// v += F/m + a; x += v; omega += T / (2/5 m r^2); periodic wrap of x; fixed particles stay
__global__ void __launch_bounds__(256) k_rigid_step(double* P, const double* acc, const double* m,
                                                    const unsigned char* free_, int n, double ax, double ay,
                                                    double az, int periodic, double Lx, double Ly, double Lz) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !free_[i]) return;
  double* p = P + (long long)i * 10;
  const double* f = acc + (long long)i * 6;
  const double mi = m[i];
  const double vx = p[3] + (f[0] / mi + ax), vy = p[4] + (f[1] / mi + ay), vz = p[5] + (f[2] / mi + az);
  double x = p[0] + vx, y = p[1] + vy, z = p[2] + vz;
  if ((periodic & 1) && Lx > 0) x = wrap(x, Lx);
  if ((periodic & 2) && Ly > 0) y = wrap(y, Ly);
  if ((periodic & 4) && Lz > 0) z = wrap(z, Lz);
  const double I = 0.4 * mi * (p[9] * p[9]);
  p[6] += f[3] / I;
  p[7] += f[4] / I;
  p[8] += f[5] / I;
  p[0] = x; p[1] = y; p[2] = z;
  p[3] = vx; p[4] = vy; p[5] = vz;
}

}  // namespace

extern "C" {

int tclb_part_nan_to_zero(double* acc, int n, void* stream) {
  if (n <= 0) return 0;
  k_nan_to_zero<<<(n + 255) / 256, 256, 0, (hipStream_t)stream>>>(acc, n);
  return (int)hipGetLastError();
}

int tclb_part_rigid_step(double* P, const double* acc, const double* m, const unsigned char* free_, int n,
                         double ax, double ay, double az, int periodic, double Lx, double Ly, double Lz,
                         void* stream) {
  if (n <= 0) return 0;
  k_rigid_step<<<(n + 255) / 256, 256, 0, (hipStream_t)stream>>>(P, acc, m, free_, n, ax, ay, az, periodic, Lx, Ly,
                                                                  Lz);
  return (int)hipGetLastError();
}

}  // extern "C"
