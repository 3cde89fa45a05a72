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

#include <hipcub/hipcub.hpp>

namespace {

__global__ void __launch_bounds__(256) k_acc_slots(double* a, int n6, int k) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n6) return;
  double s = a[j];
  for (int q = 1; q < k; q++) s += a[(long long)q * n6 + j];
  a[j] = s;
}

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

// -- solid containers (tclb_amd/particles/system.py _build_grid / _build_tree; the same
// layouts, so the node code's finders read either build) ------------------------------

// uniform grid: cell of each particle (floor(x / cell), clamped), key = linear cell id,
// value = particle id; cnt[cid + 1] counts the particles of each cell
__global__ void __launch_bounds__(256) k_grid_cells(const double* P, int n, int gx, int gy, int gz, int cell,
                                                    int* keys, int* vals, int* cnt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* p = P + (long long)i * 10;
  const int g[3] = {gx, gy, gz};
  long long c[3];
  for (int d = 0; d < 3; d++) {
    long long v = (long long)floor(p[d] / (double)cell);
    c[d] = v < 0 ? 0 : (v > g[d] - 1 ? g[d] - 1 : v);
  }
  const int cid = (int)((c[2] * gy + c[1]) * gx + c[0]);
  keys[i] = cid;
  vals[i] = i;
  atomicAdd(cnt + cid + 1, 1);
}

__device__ __forceinline__ long long spread10(long long v) {
  v = (v | (v << 16)) & 0x030000FFLL;
  v = (v | (v << 8)) & 0x0300F00FLL;
  v = (v | (v << 4)) & 0x030C30C3LL;
  return (v | (v << 2)) & 0x09249249LL;
}

// bounding-volume tree: Morton code of each centre (10 bits per axis)
__global__ void __launch_bounds__(256) k_morton(const double* P, int n, double mscale, int* keys, int* vals) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* p = P + (long long)i * 10;
  long long q[3];
  for (int d = 0; d < 3; d++) {
    double v = p[d] * mscale;
    v = v < 0.0 ? 0.0 : (v > 1023.0 ? 1023.0 : v);
    q[d] = (long long)v;
  }
  keys[i] = (int)(spread10(q[0]) | (spread10(q[1]) << 1) | (spread10(q[2]) << 2));
  vals[i] = i;
}

// leaves (sorted ids, -1 = empty) and their boxes: the cut-off sphere r + 2, widened by
// 0.05 so fp32 rounding never drops a candidate
__global__ void __launch_bounds__(256) k_tree_leaves(const double* P, int n, int nl, const int* order, int* ids,
                                                     float* B) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nl) return;
  float* b = B + (long long)(nl - 1 + j) * 6;
  if (j < n) {
    const int o = order[j];
    ids[j] = o;
    const double* p = P + (long long)o * 10;
    const double cut = p[9] + 2.05;
    for (int d = 0; d < 3; d++) {
      b[d] = (float)(p[d] - cut);
      b[3 + d] = (float)(p[d] + cut);
    }
  } else {
    ids[j] = -1;
    for (int d = 0; d < 3; d++) {
      b[d] = INFINITY;
      b[3 + d] = -INFINITY;
    }
  }
}

// one level of the implicit tree: node st + j = union of children 2(st + j) + 1, + 2
__global__ void __launch_bounds__(256) k_tree_level(float* B, int st, int cnt) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= cnt) return;
  const int i = st + j;
  const float* c0 = B + (long long)(2 * i + 1) * 6;
  const float* c1 = B + (long long)(2 * i + 2) * 6;
  float* b = B + (long long)i * 6;
  for (int d = 0; d < 3; d++) {
    b[d] = fminf(c0[d], c1[d]);
    b[3 + d] = fmaxf(c0[3 + d], c1[3 + d]);
  }
}

int bits_for(int v) {
  int b = 1;
  while (b < 31 && (1 << b) <= v) b++;
  return b;
}

// scratch layout: keys, keys_out, vals, vals_out, cnt (aligned 256 B each), hipcub temp
struct PartTmp {
  int *keys, *keys_out, *vals, *vals_out, *cnt;
  void* temp;
  size_t temp_bytes;
};

size_t align256(size_t b) { return (b + 255) / 256 * 256; }

size_t cub_temp_bytes(int n, int ncnt) {
  size_t a = 0, b = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (int*)nullptr, (int*)nullptr, (int*)nullptr, (int*)nullptr, n,
                                           0, 31);
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, b, (int*)nullptr, (int*)nullptr, ncnt);
  return a > b ? a : b;
}

bool part_tmp(void* tmp, long long bytes, int n, int ncnt, PartTmp& t) {
  char* p = (char*)tmp;
  const size_t ni = align256(sizeof(int) * (size_t)(n > 0 ? n : 1));
  t.keys = (int*)p, p += ni;
  t.keys_out = (int*)p, p += ni;
  t.vals = (int*)p, p += ni;
  t.vals_out = (int*)p, p += ni;
  t.cnt = (int*)p, p += align256(sizeof(int) * (size_t)(ncnt > 0 ? ncnt : 1));
  t.temp = p;
  t.temp_bytes = cub_temp_bytes(n, ncnt);
  return (size_t)(p - (char*)tmp) + t.temp_bytes <= (size_t)bytes;
}

}  // namespace

extern "C" {

// scratch bytes of the container builds for n particles and (grid) ncell cells
long long tclb_part_tmp_bytes(int n, int ncell) {
  const int ncnt = ncell + 1;
  return (long long)(4 * align256(sizeof(int) * (size_t)(n > 0 ? n : 1)) +
                     align256(sizeof(int) * (size_t)(ncnt > 0 ? ncnt : 1)) + cub_temp_bytes(n, ncnt) + 256);
}

// grid layout: int header[8] (gx gy gz cell), starts[ncell + 1] (inclusive prefix sum of
// the per-cell counts, starts[0] = 0), ids[n] sorted by cell, ascending id inside a cell
int tclb_part_build_grid(const double* P, int n, int* grid, int gx, int gy, int gz, int cell, int ncell, void* tmp,
                         long long tmp_bytes, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  PartTmp t;
  if (n <= 0) return 0;
  if (!part_tmp(tmp, tmp_bytes, n, ncell + 1, t)) return -20;
  hipError_t e = hipMemsetAsync(t.cnt, 0, sizeof(int) * (size_t)(ncell + 1), s);
  if (e != hipSuccess) return (int)e;
  k_grid_cells<<<(n + 255) / 256, 256, 0, s>>>(P, n, gx, gy, gz, cell, t.keys, t.vals, t.cnt);
  size_t tb = t.temp_bytes;
  if ((e = hipcub::DeviceScan::InclusiveSum(t.temp, tb, t.cnt, grid + 8, ncell + 1, s)) != hipSuccess) return (int)e;
  tb = t.temp_bytes;
  e = hipcub::DeviceRadixSort::SortPairs(t.temp, tb, t.keys, t.keys_out, t.vals, grid + 9 + ncell, n, 0,
                                         bits_for(ncell), s);
  if (e != hipSuccess) return (int)e;
  return (int)hipGetLastError();
}

// tree layout: int header[8] (kind 1 in [4], nl in [5]), leaf ids[nl], float boxes
// [2 nl - 1][6] (lo xyz, hi xyz) of an implicit complete binary tree
int tclb_part_build_tree(const double* P, int n, int* grid, int nl, double mscale, void* tmp, long long tmp_bytes,
                         void* stream) {
  hipStream_t s = (hipStream_t)stream;
  PartTmp t;
  if (n <= 0) return 0;
  if (!part_tmp(tmp, tmp_bytes, n, 0, t)) return -20;
  k_morton<<<(n + 255) / 256, 256, 0, s>>>(P, n, mscale, t.keys, t.vals);
  size_t tb = t.temp_bytes;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(t.temp, tb, t.keys, t.keys_out, t.vals, t.vals_out, n, 0, 30, s);
  if (e != hipSuccess) return (int)e;
  float* B = (float*)(grid + 8 + nl);
  k_tree_leaves<<<(nl + 255) / 256, 256, 0, s>>>(P, n, nl, t.vals_out, grid + 8, B);
  int L = 0;
  while ((1 << (L + 1)) <= nl) L++;            // nl = 2^L
  for (int lvl = L - 1; lvl >= 0; lvl--) {
    const int st = (1 << lvl) - 1, cnt = 1 << lvl;
    k_tree_level<<<(cnt + 255) / 256, 256, 0, s>>>(B, st, cnt);
  }
  return (int)hipGetLastError();
}

// the k accumulator copies of the particle stage (core.hpp particle_acc) summed into the
// first: acc[j] += acc[s * n6 + j], s = 1 .. k-1
int tclb_part_acc_slots(double* acc, int n6, int k, void* stream) {
  if (k <= 1 || n6 <= 0) return 0;
  k_acc_slots<<<(n6 + 255) / 256, 256, 0, (hipStream_t)stream>>>(acc, n6, k);
  return (int)hipGetLastError();
}

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
