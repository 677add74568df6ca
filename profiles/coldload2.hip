// coldload2.hip — what makes the coarse kernels' first loads slow in the search
// (profiles/r06_coarse_stamps.txt: 17-20k cycles per wave for a few loads), when
// profiles/coldload.hip's reader sees 430-1400 cycles for the same select pattern?
// The trace says k_coarse_select takes 5.1 us after a key-only k_coarse_gemm and
// 10.5 us after one that also writes the 16 MB of T3 (profiles/r06_kernel_summary.txt).
//   E1..E3: a writer kernel (keys 4 MB [+ T3 16 MB, plain or nontemporal stores]),
//           then the select-pattern reader of the keys: per-wave first-load cycles
//           and the reader's duration (events);
//   E4:     the key-tile fill pattern of k_coarse_gemm (512 workgroups x 4 waves,
//           32 x 8-B loads per lane of a [128][1040] centroid matrix + 8 KB of
//           query staging and a barrier) after an empty kernel / after the writer.
// Build: hipcc --offload-arch=gfx950 -O3 -o profiles/coldload2 profiles/coldload2.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ __launch_bounds__(256) void k_write(float* keys, int64_t nk, float* t3, int64_t nt, int nontemporal) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nk; i += stride) keys[i] = (float)(i & 1023);
  if (nontemporal)
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nt; i += stride)
      __builtin_nontemporal_store((float)i, t3 + i);
  else
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nt; i += stride) t3[i] = (float)i;
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
// k_coarse_gemm's key-tile fill (d = 128, paired layout): 32 x float2 of centT per
// lane, then the 16 x 128 query tile staged in LDS, a barrier
__global__ __launch_bounds__(256) void k_fill(const float* __restrict__ centT, int ldc, const float* __restrict__ x,
                                              uint64_t* stamps, float* sink) {
  __shared__ float xs[128 * 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nct = 8;
  const int q0 = (blockIdx.x / nct) * 16;
  const int c0 = (blockIdx.x % nct) * 128 + wave * 32;
  const int i16 = lane & 15, k4 = lane >> 4;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  float b[32][2];
  const int cp2 = c0 + 2 * i16;
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const float2 v = *reinterpret_cast<const float2*>(centT + (int64_t)(4 * j + k4) * ldc + cp2);
    b[j][0] = v.x;
    b[j][1] = v.y;
  }
  for (int i = tid; i < 16 * 128; i += 256) {
    const int qq = i >> 7, k = i & 127;
    xs[k * 16 + qq] = x[(int64_t)(q0 + qq) * 128 + k];
  }
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 32; j++) s += b[j][0] * xs[(4 * j + k4) * 16 + i16] + b[j][1];
  if (lane == 0) stamps[blockIdx.x * 4 + wave] = t1 - t0;
  if (s == 12345.f) sink[blockIdx.x] = s;
}

int main() {
  const int nq = 1024, nlist = 1024, ldc = 1040;
  float *keys, *t3, *sink, *centT, *x;
  uint64_t* st;
  hipMalloc(&keys, sizeof(float) * nq * nlist);
  hipMalloc(&t3, sizeof(float) * 4 * nq * nlist);
  hipMalloc(&sink, sizeof(float) * 4096);
  hipMalloc(&st, sizeof(uint64_t) * 4096);
  hipMalloc(&centT, sizeof(float) * 128 * ldc);
  hipMalloc(&x, sizeof(float) * nq * 128);
  hipMemset(centT, 0, sizeof(float) * 128 * ldc);
  hipMemset(x, 0, sizeof(float) * nq * 128);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::vector<uint64_t> h(4096);
  auto report = [&](const char* name, int n) {
    hipDeviceSynchronize();
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h.data(), st, sizeof(uint64_t) * n, hipMemcpyDeviceToHost);
    std::vector<uint64_t> s(h.begin(), h.begin() + n);
    std::sort(s.begin(), s.end());
    printf("%-44s cycles p10 %6llu p50 %6llu p90 %6llu max %6llu | kernel %6.2f us\n", name,
           (unsigned long long)s[n / 10], (unsigned long long)s[n / 2], (unsigned long long)s[n * 9 / 10],
           (unsigned long long)s[n - 1], ms * 1e3);
  };
  const int64_t nk = (int64_t)nq * nlist, nt = 4 * nk;
  for (int rep = 0; rep < 3; rep++) {
    // E2: keys only
    hipLaunchKernelGGL(k_write, dim3(1536), dim3(256), 0, 0, keys, nk, t3, (int64_t)0, 0);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_read, dim3(nq / 4), dim3(256), 0, 0, keys, nlist, st, sink);
    hipEventRecord(e1);
    report("E2 select reader after keys-only writer", nq);
    // E1: keys + 16 MB T3, plain stores
    hipLaunchKernelGGL(k_write, dim3(1536), dim3(256), 0, 0, keys, nk, t3, nt, 0);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_read, dim3(nq / 4), dim3(256), 0, 0, keys, nlist, st, sink);
    hipEventRecord(e1);
    report("E1 select reader after keys + T3 writer", nq);
    // E3: keys + 16 MB T3, nontemporal T3 stores
    hipLaunchKernelGGL(k_write, dim3(1536), dim3(256), 0, 0, keys, nk, t3, nt, 1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_read, dim3(nq / 4), dim3(256), 0, 0, keys, nlist, st, sink);
    hipEventRecord(e1);
    report("E3 select reader after keys + nt-T3 writer", nq);
    // E4: gemm fill pattern
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_fill, dim3(512), dim3(256), 0, 0, centT, ldc, x, st, sink);
    hipEventRecord(e1);
    report("E4a gemm fill after an empty kernel", 2048);
    hipLaunchKernelGGL(k_write, dim3(1536), dim3(256), 0, 0, keys, nk, t3, nt, 0);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_fill, dim3(512), dim3(256), 0, 0, centT, ldc, x, st, sink);
    hipEventRecord(e1);
    report("E4b gemm fill after keys + T3 writer", 2048);
  }
  return 0;
}
