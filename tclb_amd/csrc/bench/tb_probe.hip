// Two-step (temporal) blocking probe: does a ring of intermediate planes held in the
// 256 MiB Infinity Cache cut the HBM traffic of a 27-population pull step?
//
//   base: one launch per step, S0 -> S1 (27 fp64 streams per node, 432 B/node)
//   tb  : per z plane p (and y chunk), A(p+1): S0 planes p..p+2 -> ring slot (p+1) % K,
//         then B(p): ring slots p-1..p+1 -> S1 plane p.  Two steps per sweep; HBM sees S0
//         read once and S1 written once per two steps if the ring stays resident.
// Fields 0-8 come from plane z-1, 9-17 from z, 18-26 from z+1 (the d3q27 pull pattern by
// plane).  Timed with events; prints ms per step of each form.
//
//   tb_probe nx ny nz K ychunks reps
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

// src planes: field f of plane z at src + f*fs + z*ps; dst likewise (dfs, dps); the
// z of each field group is given as three plane offsets (already wrapped by the host)
template <bool NT>
__global__ void __launch_bounds__(256) k_plane(const double* __restrict__ src, double* __restrict__ dst,
                                               long long fs, long long zm, long long z0, long long zp,
                                               long long dfs, long long dz, long long off, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long j = off + i;
  double v[27];
#pragma unroll
  for (int f = 0; f < 27; f++) {
    const long long zo = f < 9 ? zm : (f < 18 ? z0 : zp);
    v[f] = src[f * fs + zo + j];
  }
#pragma unroll
  for (int f = 0; f < 27; f++) v[f] = v[f] * 0.999 + 1e-3;
#pragma unroll
  for (int f = 0; f < 27; f++) {
    if (NT) __builtin_nontemporal_store(v[f], dst + f * dfs + dz + j);
    else dst[f * dfs + dz + j] = v[f];
  }
}

// whole-volume step: one launch, the same pattern with z-1/z/z+1 as +-plane offsets
__global__ void __launch_bounds__(256) k_full(const double* __restrict__ src, double* __restrict__ dst,
                                              long long fs, long long ps, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double v[27];
#pragma unroll
  for (int f = 0; f < 27; f++) {
    const long long zo = f < 9 ? -ps : (f < 18 ? 0 : ps);
    long long k = i + zo;
    k = k < 0 ? k + n : (k >= n ? k - n : k);
    v[f] = src[f * fs + k];
  }
#pragma unroll
  for (int f = 0; f < 27; f++) v[f] = v[f] * 0.999 + 1e-3;
#pragma unroll
  for (int f = 0; f < 27; f++) __builtin_nontemporal_store(v[f], dst + f * fs + i);
}

int main(int argc, char** argv) {
  const int nx = argc > 1 ? atoi(argv[1]) : 512, ny = argc > 2 ? atoi(argv[2]) : 512, nz = argc > 3 ? atoi(argv[3]) : 512;
  const int K = argc > 4 ? atoi(argv[4]) : 4, YC = argc > 5 ? atoi(argv[5]) : 1, reps = argc > 6 ? atoi(argv[6]) : 4;
  const int ntring = argc > 7 ? atoi(argv[7]) : 0;
  const long long ps = (long long)nx * ny, fs = ps * nz, n = fs;
  const long long rps = ps / YC;      // ring plane chunk (one y chunk of a plane)
  if (ny % YC || K < 3 || nz < 4) { fprintf(stderr, "bad args\n"); return 2; }
  double *S0, *S1, *R;
  CK(hipMalloc(&S0, 27 * fs * 8));
  CK(hipMalloc(&S1, 27 * fs * 8));
  // ring: [slot][f][plane chunk] for each y chunk (one ring per chunk, chunks in sequence)
  const long long rfs = rps * K;
  CK(hipMalloc(&R, 27 * rfs * 8));
  CK(hipMemset(S0, 0, 27 * fs * 8));
  CK(hipMemset(S1, 0, 27 * fs * 8));
  CK(hipMemset(R, 0, 27 * rfs * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned gfull = (unsigned)((n + 255) / 256);
  auto base = [&](int steps) {
    for (int s = 0; s < steps; s++) {
      k_full<<<gfull, 256>>>(s & 1 ? S1 : S0, s & 1 ? S0 : S1, fs, ps, n);
    }
  };
  const int cn = (int)rps;
  const unsigned gc = (unsigned)((cn + 255) / 256);
  auto wz = [&](long long z) { return ((z % nz) + nz) % nz; };
  auto tb = [&]() {   // two steps, S0 -> S1
    for (int c = 0; c < YC; c++) {
      const long long yoff = c * rps;
      // prologue: A on planes 0 and 1 (ring slots of planes z: z % K)
      for (long long p = -1; p < nz; p++) {
        const long long a = p + 1;   // A(a): S0 planes a-1, a, a+1 -> ring slot a % K
        if (a < nz && ntring)
          k_plane<true><<<gc, 256>>>(S0, R - yoff, fs, wz(a - 1) * ps, wz(a) * ps, wz(a + 1) * ps, rfs, (a % K) * rps, yoff, cn);
        else if (a < nz)
          k_plane<false><<<gc, 256>>>(S0, R - yoff, fs, wz(a - 1) * ps, wz(a) * ps, wz(a + 1) * ps, rfs, (a % K) * rps, yoff, cn);
        if (p >= 1 && p <= nz - 2) {   // B on plane p: ring slots p-1..p+1 (A(p+1) done)
          const long long b = p;
          k_plane<true><<<gc, 256>>>(R - yoff, S1, rfs, ((b - 1 + K) % K) * rps, (b % K) * rps, ((b + 1) % K) * rps, fs,
                               b * ps, yoff, cn);
        }
      }
    }
  };
  base(2);
  tb();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  base(2 * reps);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float mb;
  CK(hipEventElapsedTime(&mb, e0, e1));
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; r++) tb();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float mt;
  CK(hipEventElapsedTime(&mt, e0, e1));
  const double sb = mb / (2 * reps), st = mt / (2 * reps);
  printf("{\"nx\":%d,\"ny\":%d,\"nz\":%d,\"K\":%d,\"ychunks\":%d,\"ntring\":%d,\"ring_MB\":%.1f,\"base_ms\":%.4f,\"tb_ms\":%.4f,"
         "\"base_TBps\":%.3f,\"speedup\":%.3f}\n",
         nx, ny, nz, K, YC, ntring, 27.0 * rfs * 8 / 1e6, sb, st, 432.0 * n / sb / 1e9, sb / st);
  CK(hipFree(S0));
  CK(hipFree(S1));
  CK(hipFree(R));
  return 0;
}
