// hbm_stream.hip — the box's measured HBM peak for bench.py's roofline
// ("also report the measured STREAM-copy
// peak on the box").  Not part of the IVF-PQ library or its C-ABI: a separate
// libhbmstream.so that bench.py runs before its timed region.
//
// Two streaming kernels over buffers far larger than the 256 MiB Infinity Cache
// (bench.py uses 2 GiB each), 16 B per lane, four loads in flight per thread,
// grid-stride over a grid of 8 workgroups per CU:
//   copy: b[i] = a[i]            (STREAM copy: bytes = read + written)
//   read: x ^= a[i], one store per thread at the end (the scan's read-mostly
//         shape: bytes = read)
// Timed with HIP events on the caller's stream, best of `iters` launches.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
constexpr int kThreads = 256;
constexpr int kUnroll = 4;

__global__ __launch_bounds__(kThreads) void k_stream_copy(const u4* __restrict__ a, u4* __restrict__ b,
                                                          int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  for (; i + (kUnroll - 1) * stride < n; i += kUnroll * stride) {
    u4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; u++) v[u] = __builtin_nontemporal_load(a + i + u * stride);
#pragma unroll
    for (int u = 0; u < kUnroll; u++) __builtin_nontemporal_store(v[u], b + i + u * stride);
  }
  for (; i < n; i += stride) b[i] = a[i];
}

__global__ __launch_bounds__(kThreads) void k_stream_read(const u4* __restrict__ a, int64_t n,
                                                          uint32_t* __restrict__ sink) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  uint32_t x = 0;
  for (; i + (kUnroll - 1) * stride < n; i += kUnroll * stride) {
    u4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; u++) v[u] = __builtin_nontemporal_load(a + i + u * stride);
#pragma unroll
    for (int u = 0; u < kUnroll; u++) x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n; i += stride) x ^= a[i].x ^ a[i].y ^ a[i].z ^ a[i].w;
  sink[(int64_t)blockIdx.x * kThreads + threadIdx.x] = x;  // (keeps the loads; 4 B per thread)
}

int grid_for(int dev) {
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return cus * 8;
}

}  // namespace

extern "C" {

// Best time (ms) of `iters` launches of the copy (src -> dst, `bytes` each, a
// multiple of 16) and of the read (src; `sink` >= grid * 256 * 4 bytes of device
// scratch), on `stream`.  Returns 0, or a hipError_t.
int hbm_stream_measure(const void* src, void* dst, int64_t bytes, void* sink, int64_t sink_bytes, int iters,
                       void* stream, float* copy_ms, float* read_ms) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  const int grid = grid_for(dev);
  if (bytes % 16 != 0 || sink_bytes < (int64_t)grid * kThreads * 4 || iters < 1) return (int)hipErrorInvalidValue;
  const int64_t n = bytes / 16;
  hipStream_t s = (hipStream_t)stream;
  hipEvent_t a, b;
  if ((e = hipEventCreate(&a)) != hipSuccess) return (int)e;
  if ((e = hipEventCreate(&b)) != hipSuccess) return (int)e;
  float best_c = 1e30f, best_r = 1e30f;
  for (int it = 0; it <= iters; it++) {  // (launch 0: warm-up)
    (void)hipEventRecord(a, s);
    hipLaunchKernelGGL(k_stream_copy, dim3(grid), dim3(kThreads), 0, s, (const u4*)src, (u4*)dst, n);
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float t = 0.f;
    (void)hipEventElapsedTime(&t, a, b);
    if (it > 0 && t < best_c) best_c = t;
    (void)hipEventRecord(a, s);
    hipLaunchKernelGGL(k_stream_read, dim3(grid), dim3(kThreads), 0, s, (const u4*)src, n, (uint32_t*)sink);
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&t, a, b);
    if (it > 0 && t < best_r) best_r = t;
  }
  e = hipGetLastError();
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  *copy_ms = best_c;
  *read_ms = best_r;
  return (int)e;
}

}  // extern "C"
