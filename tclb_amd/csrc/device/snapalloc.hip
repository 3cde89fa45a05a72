// Snapshot allocator: the A/B population buffers are the only large allocations of a
// lattice (2 x 29 GB for d3q27 fp64 512^3), and where they land in HBM decides how fast
// the collide-stream kernel reads them (tools/direction_probe.py: the same kernel runs
// 9.7 ms or 11.8 ms per dispatch depending on the placement of the buffer it reads).
// The reference pre-allocates every snapshot in one cudaMalloc (src/cross.cu:52-117,
// cudaPreAlloc / cudaAllocFinalize); here the placement is a choice:
//
//   mode 0  hipMalloc                                   (what the torch allocator does)
//   mode 1  hipExtMallocWithFlags(hipDeviceMallocContiguous): one physically contiguous
//           range, so the GPU page tables can use their largest fragments
//   mode 2  virtual memory API: hipMemCreate of the whole size at the recommended
//           granularity, mapped into a range reserved at a 1 GiB-aligned address
//
// None of the modes gives a placement that is fast every time (the same mode ran 9.5 and
// 11.8 ms per dispatch on different allocations), so the lattice ranks several candidates
// by tclb_snap_probe — the streaming read / write speed of each — and keeps the fastest
// pair (tclb_amd/lattice.py _alloc_snapshots).
//
// Each call returns 0 or a HIP error code; tclb_snap_free releases by the same mode.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <mutex>

namespace {

struct VmmRange {
  hipMemGenericAllocationHandle_t handle;
  size_t size;
};

std::mutex g_mu;
std::map<uintptr_t, VmmRange> g_vmm;

int vmm_alloc(void** out, size_t bytes, int device) {
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = device;
  size_t gran = 0;
  hipError_t e = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended);
  if (e != hipSuccess) return (int)e;
  if (gran == 0) gran = 2u << 20;
  const size_t size = (bytes + gran - 1) / gran * gran;
  hipMemGenericAllocationHandle_t h;
  if ((e = hipMemCreate(&h, size, &prop, 0)) != hipSuccess) return (int)e;
  void* p = nullptr;
  const size_t align = size_t(1) << 30;
  if ((e = hipMemAddressReserve(&p, size, align, nullptr, 0)) != hipSuccess) {
    hipMemRelease(h);
    return (int)e;
  }
  if ((e = hipMemMap(p, size, 0, h, 0)) != hipSuccess) {
    hipMemAddressFree(p, size);
    hipMemRelease(h);
    return (int)e;
  }
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  if ((e = hipMemSetAccess(p, size, &acc, 1)) != hipSuccess) {
    hipMemUnmap(p, size);
    hipMemAddressFree(p, size);
    hipMemRelease(h);
    return (int)e;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  g_vmm[(uintptr_t)p] = VmmRange{h, size};
  *out = p;
  return 0;
}

int vmm_free(void* p) {
  VmmRange r;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_vmm.find((uintptr_t)p);
    if (it == g_vmm.end()) return (int)hipErrorInvalidValue;
    r = it->second;
    g_vmm.erase(it);
  }
  hipError_t e = hipMemUnmap(p, r.size);
  if (e == hipSuccess) e = hipMemAddressFree(p, r.size);
  if (e == hipSuccess) e = hipMemRelease(r.handle);
  return (int)e;
}

}  // namespace

namespace {

// streaming probe of one snapshot candidate: K field planes `stride` elements apart read
// (op 1, summed into a sink that is never written for finite data) or written with
// non-temporal stores (op 2) — the memory pattern of the collide-stream kernels
template <class T, int K>
__global__ void __launch_bounds__(256) k_probe(T* buf, T* sink, long long n, long long stride, int op) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (op == 1) {
    T s = 0;
#pragma unroll
    for (int k = 0; k < K; k++) s += buf[k * stride + i];
    if (s == (T)12345) sink[0] = s;
  } else {
#pragma unroll
    for (int k = 0; k < K; k++) __builtin_nontemporal_store((T)0, buf + k * stride + i);
  }
}

template <class T>
int probe(void* buf, void* sink, long long n, long long stride, int K, int op, hipStream_t s) {
  const dim3 b(256), g((unsigned)((n + 255) / 256));
  T* p = (T*)buf;
  T* q = (T*)sink;
  // the nearest unrolled width not above K (the pattern, not every byte, is what is probed);
  // fewer than 9 planes: one stream over all of them
  if (K >= 27) k_probe<T, 27><<<g, b, 0, s>>>(p, q, n, stride, op);
  else if (K >= 19) k_probe<T, 19><<<g, b, 0, s>>>(p, q, n, stride, op);
  else if (K >= 9) k_probe<T, 9><<<g, b, 0, s>>>(p, q, n, stride, op);
  else {
    const long long m = (long long)(K - 1) * stride + n;
    if ((m + 255) / 256 > 0x7fffffffLL) return (int)hipErrorInvalidValue;
    k_probe<T, 1><<<dim3((unsigned)((m + 255) / 256)), b, 0, s>>>(p, q, m, 0, op);
  }
  return (int)hipGetLastError();
}

}  // namespace

// op 1: read / op 2: write (zeros) of K planes of n elements (elem_bytes 8, 4 or 2: the
// half storage modes, probed as 16-bit words), stride apart
extern "C" int tclb_snap_probe(void* buf, void* sink, long long n, long long stride, int K, int elem_bytes, int op,
                               void* stream) {
  if (n <= 0 || K <= 0 || (n + 255) / 256 > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  if (elem_bytes == 8) return probe<double>(buf, sink, n, stride, K, op, (hipStream_t)stream);
  if (elem_bytes == 4) return probe<float>(buf, sink, n, stride, K, op, (hipStream_t)stream);
  if (elem_bytes == 2) return probe<unsigned short>(buf, sink, n, stride, K, op, (hipStream_t)stream);
  return (int)hipErrorInvalidValue;
}

extern "C" int tclb_snap_alloc(void** out, size_t bytes, int mode, int device) {
  if (!out || bytes == 0) return (int)hipErrorInvalidValue;
  *out = nullptr;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return (int)e;
  switch (mode) {
    case 0: e = hipMalloc(out, bytes); break;
    case 1: e = hipExtMallocWithFlags(out, bytes, hipDeviceMallocContiguous); break;
    case 2: return vmm_alloc(out, bytes, device);
    default: return (int)hipErrorInvalidValue;
  }
  return (int)e;
}

extern "C" int tclb_snap_free(void* p, int mode) {
  if (!p) return 0;
  // the buffer may still be read or written by queued kernels of any stream
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return (int)e;
  if (mode == 2) return vmm_free(p);
  return (int)hipFree(p);
}
