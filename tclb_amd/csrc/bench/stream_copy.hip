// K-stream copy probe: the memory pattern of the collide-stream kernels without the
// arithmetic and the neighbour shifts.  Thread i copies element i of each of K arrays
// that sit `stride` elements apart (the SoA field planes of a snapshot), with
// non-temporal stores as in the model kernels.  K = 1 over one long array is the plain
// copy ceiling; K = 27 at a 512^3 stride is the d3q27 snapshot pattern (54 concurrent
// streams).  Used by tools/stream_probe.py to tell a box's copy ceiling apart from the
// many-stream ceiling.
#include <hip/hip_runtime.h>
#include <cstdint>

template <typename T, int K>
__global__ void __launch_bounds__(256) k_streams(const T* __restrict__ src, T* __restrict__ dst, int64_t n,
                                                 int64_t stride) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  T v[K];
#pragma unroll
  for (int k = 0; k < K; k++) v[k] = src[k * stride + i];
#pragma unroll
  for (int k = 0; k < K; k++) __builtin_nontemporal_store(v[k], dst + k * stride + i);
}

// read-only and write-only halves of the same pattern (tools/direction_probe.py: which
// side of a snapshot pair is slow on a given placement)
template <typename T, int K>
__global__ void __launch_bounds__(256) k_read(const T* __restrict__ src, T* __restrict__ sink, int64_t n,
                                              int64_t stride) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  T s = 0;
#pragma unroll
  for (int k = 0; k < K; k++) s += src[k * stride + i];
  if (s == (T)-1.2345e30) sink[0] = s;      // never true for the probe's data: keeps the loads
}

template <typename T, int K>
__global__ void __launch_bounds__(256) k_write(T* __restrict__ dst, int64_t n, int64_t stride) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
#pragma unroll
  for (int k = 0; k < K; k++) __builtin_nontemporal_store((T)1, dst + k * stride + i);
}

template <typename T>
static int launch_rw(const void* src, void* dst, int64_t n, int64_t stride, int K, int op, hipStream_t s) {
  const dim3 block(256), grid((unsigned)((n + 255) / 256));
  if (K != 27) return -2;
  if (op == 1) k_read<T, 27><<<grid, block, 0, s>>>(static_cast<const T*>(src), static_cast<T*>(dst), n, stride);
  else k_write<T, 27><<<grid, block, 0, s>>>(static_cast<T*>(dst), n, stride);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <typename T>
static int launch(const void* src, void* dst, int64_t n, int64_t stride, int K, hipStream_t s) {
  const dim3 block(256), grid((unsigned)((n + 255) / 256));
  const T* a = static_cast<const T*>(src);
  T* b = static_cast<T*>(dst);
  switch (K) {
    case 1: k_streams<T, 1><<<grid, block, 0, s>>>(a, b, n, stride); break;
    case 9: k_streams<T, 9><<<grid, block, 0, s>>>(a, b, n, stride); break;
    case 19: k_streams<T, 19><<<grid, block, 0, s>>>(a, b, n, stride); break;
    case 27: k_streams<T, 27><<<grid, block, 0, s>>>(a, b, n, stride); break;
    default: return -2;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int tclb_stream_copy(const void* src, void* dst, int64_t n, int64_t stride, int K, int elem_bytes,
                                void* stream) {
  if (n <= 0 || stride < n || (n + 255) / 256 > 0x7fffffffLL) return -3;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (elem_bytes == 8) return launch<double>(src, dst, n, stride, K, s);
  if (elem_bytes == 4) return launch<float>(src, dst, n, stride, K, s);
  return -4;
}

// op 1: read the K streams of src (dst: a sink of at least one element); op 2: write dst
extern "C" int tclb_stream_rw(const void* src, void* dst, int64_t n, int64_t stride, int K, int elem_bytes, int op,
                              void* stream) {
  if (n <= 0 || stride < n || (n + 255) / 256 > 0x7fffffffLL || (op != 1 && op != 2)) return -3;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (elem_bytes == 8) return launch_rw<double>(src, dst, n, stride, K, op, s);
  if (elem_bytes == 4) return launch_rw<float>(src, dst, n, stride, K, op, s);
  return -4;
}
