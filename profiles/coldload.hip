// coldload.hip — why do the coarse kernels' first loads take ~18k cycles?
// (profiles/r06_cstamps_*.txt: k_coarse_select's 16 key loads per lane and the
// key/T3 tile fills of k_coarse_gemm each take 17-20k cycles per wave).
// A reader kernel (1024 waves, each 16 x 4-B loads per lane from a 4 MB buffer,
// the select's access pattern) stamps the wave's first-load round trip
// (s_memtime before the loads, after s_waitcnt vmcnt(0)), launched:
//   a: right after a writer kernel that wrote the same 4 MB,
//   b: right after itself (warm),
//   c: right after a writer of another 16 MB buffer,
//   d: right after an empty kernel.
// Build: hipcc --offload-arch=gfx950 -O3 -o profiles/coldload profiles/coldload.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ __launch_bounds__(256) void k_write(float* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = (float)i;
}
__global__ void k_empty() {}
__global__ __launch_bounds__(256) void k_read(const float* __restrict__ keys, int nlist, uint64_t* stamps,
                                              float* sink) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t q = (int64_t)blockIdx.x * 4 + wave;
  const float* row = keys + q * nlist;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  float v[16];
#pragma unroll
  for (int u = 0; u < 16; u++) v[u] = row[u * 64 + lane];
  float m = v[0];
#pragma unroll
  for (int u = 1; u < 16; u++) m = fminf(m, v[u]);
  __builtin_amdgcn_s_waitcnt(0);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) stamps[q] = t1 - t0;
  if (m < -1.f) sink[q] = m;
}

int main() {
  const int nq = 1024, nlist = 1024;
  float *keys, *other, *sink;
  uint64_t* st;
  hipMalloc(&keys, sizeof(float) * nq * nlist);
  hipMalloc(&other, sizeof(float) * 4 * nq * nlist);
  hipMalloc(&sink, sizeof(float) * nq);
  hipMalloc(&st, sizeof(uint64_t) * nq);
  std::vector<uint64_t> h(nq);
  auto report = [&](const char* name) {
    hipDeviceSynchronize();
    hipMemcpy(h.data(), st, sizeof(uint64_t) * nq, hipMemcpyDeviceToHost);
    std::vector<uint64_t> s = h;
    std::sort(s.begin(), s.end());
    printf("%-28s first-load round trip cycles: p10 %6llu p50 %6llu p90 %6llu max %6llu\n", name,
           (unsigned long long)s[nq / 10], (unsigned long long)s[nq / 2], (unsigned long long)s[nq * 9 / 10],
           (unsigned long long)s[nq - 1]);
  };
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(k_write, dim3(1024), dim3(256), 0, 0, keys, (int64_t)nq * nlist);
    hipLaunchKernelGGL(k_read, dim3(nq / 4), dim3(256), 0, 0, keys, nlist, st, sink);
    report("a: after writing it");
    hipLaunchKernelGGL(k_read, dim3(nq / 4), dim3(256), 0, 0, keys, nlist, st, sink);
    report("b: after itself");
    hipLaunchKernelGGL(k_read, dim3(nq / 4), dim3(256), 0, 0, keys, nlist, st, sink);
    hipLaunchKernelGGL(k_write, dim3(1024), dim3(256), 0, 0, other, (int64_t)4 * nq * nlist);
    hipLaunchKernelGGL(k_read, dim3(nq / 4), dim3(256), 0, 0, keys, nlist, st, sink);
    report("c: after writing 16 MB else");
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0);
    hipLaunchKernelGGL(k_read, dim3(nq / 4), dim3(256), 0, 0, keys, nlist, st, sink);
    report("d: after an empty kernel");
  }
  return 0;
}
