// Microbenchmark of the LUT-gather inner loop variants of the M = 16 list scan
// (no global memory in the timed loop): cycles per 16-step block per wave, with
// 2 workgroups x 4 waves per CU and a 64 KB LUT per workgroup, as in the scan.
//   V0 "rowmajor": [m][j] float4 image, every lane reads sub-table m at step m
//                  (random 16-B slots: ~3-way bank conflicts), 4 v_add (or 2 packed)
//   V1 "skew_cnd": [j][m] image, lane s = l & 15 staggered, keep fma + v_cndmask capture
//   V2 "skew_exec": the same, capture by packed moves under a narrowed exec mask
//   V3 "skew_nocap": skewed gathers + packed fma, no capture (lower bound)
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o gather_micro gather_micro.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float nf2 __attribute__((ext_vector_type(2)));

constexpr uint64_t kRowLane0 = 0x0001000100010001ull;
__device__ __forceinline__ float keep_lanes(uint64_t m) {
  float r;
  asm("v_cndmask_b32_e64 %0, 1.0, 0, %1" : "=v"(r) : "s"(m));
  return r;
}
__device__ __forceinline__ float sel_lanes(uint64_t m, float a, float b) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
  return r;
}
__device__ __forceinline__ void cap2(nf2& f0, nf2& f1, nf2 d0, nf2 d1, uint64_t m) {
  uint64_t sv;
  asm("s_and_saveexec_b64 %[sv], %[m]\n\t"
      "v_pk_mov_b32 %[f0], %[d0], %[d0] op_sel:[0,1]\n\t"
      "v_pk_mov_b32 %[f1], %[d1], %[d1] op_sel:[0,1]\n\t"
      "s_mov_b64 exec, %[sv]"
      : [f0] "+v"(f0), [f1] "+v"(f1), [sv] "=&s"(sv)
      : [d0] "v"(d0), [d1] "v"(d1), [m] "s"(m)
      : "scc");
}

template <int VAR>
__global__ __launch_bounds__(256, 2) void k_gather(const uint32_t* __restrict__ codes, int nblk, float* out,
                                                   uint64_t* cyc) {
  __shared__ f4 lut[4096];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < 4096; i += 256) lut[i] = f4{(float)(i & 255), (float)(i >> 8), 1.f, 2.f};
  __syncthreads();
  // each lane: 16 random code bytes per block, from a small table (cache resident, loaded ahead)
  const uint4* cp = reinterpret_cast<const uint4*>(codes) + (blockIdx.x * 256 + tid) % 4096;
  uint4 w = cp[0];
  const int s = lane & 15;
  uint32_t MO[4];
#pragma unroll
  for (int q = 0; q < 4; q++) {
    uint32_t x = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) x |= (uint32_t)((((4 * q + r) - s) & 15) << 4) << (8 * r);
    MO[q] = x;
  }
  float acc = 0.f;
  nf2 d0{0.f, 0.f}, d1{0.f, 0.f}, f0{0.f, 0.f}, f1{0.f, 0.f};
  float ds[4] = {0.f, 0.f, 0.f, 0.f}, fs[4] = {0.f, 0.f, 0.f, 0.f};
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int b = 0; b < nblk; b++) {
    uint32_t W[4] = {w.x, w.y, w.z, w.w};
    f4 v[16];
    if constexpr (VAR == 0 || VAR == 4) {
#pragma unroll
      for (int m = 0; m < 16; m++) v[m] = lut[m * 256 + ((W[m >> 2] >> (8 * (m & 3))) & 255)];
#pragma unroll
      for (int m = 0; m < 16; m++) {
        if constexpr (VAR == 0) {
          d0 = d0 + v[m].xy;
          d1 = d1 + v[m].zw;
        } else {
#pragma unroll
          for (int g = 0; g < 4; g++) ds[g] = ds[g] + v[m][g];
        }
      }
      f0 = d0;
      f1 = d1;
    } else {
#pragma unroll
      for (int u = 0; u < 16; u++) {
        const int r = u & 3;
        const uint32_t a16 = __builtin_amdgcn_perm(W[u >> 2], MO[u >> 2], 0x0C0C0000u | ((4u + r) << 8) | (uint32_t)r);
        v[u] = *reinterpret_cast<const f4*>(reinterpret_cast<const char*>(lut) + a16);
      }
      uint64_t m0 = kRowLane0;
#pragma unroll
      for (int u = 0; u < 16; u++) {
        asm volatile("" : "+s"(m0));
        const uint64_t m15 = u == 15 ? kRowLane0 : m0 << 1;
        const float keep = keep_lanes(m0);
        if constexpr (VAR == 1) {
#pragma unroll
          for (int g = 0; g < 4; g++) ds[g] = __builtin_fmaf(ds[g], keep, v[u][g]);
#pragma unroll
          for (int g = 0; g < 4; g++) fs[g] = sel_lanes(m15, fs[g], ds[g]);
        } else {
          const nf2 kk{keep, keep};
          d0 = __builtin_elementwise_fma(d0, kk, v[u].xy);
          d1 = __builtin_elementwise_fma(d1, kk, v[u].zw);
          if constexpr (VAR == 2) cap2(f0, f1, d0, d1, m15);
        }
        m0 = m15;
      }
    }
    acc += f0.x + f1.y + fs[0] + fs[3];
    w.x = w.x * 1664525u + 1013904223u;  // next block's codes (ALU, no memory)
    w.y = w.y * 1664525u + 1013904223u;
    w.z = w.z ^ (w.x >> 7);
    w.w = w.w + w.y;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 256 + tid] = acc + d0.y + d1.x + ds[1] + ds[2];
  if (lane == 0) cyc[blockIdx.x * 4 + (tid >> 6)] = t1 - t0;
}

template <int VAR>
void run(const char* name, const uint32_t* dcodes, float* dout, uint64_t* dcyc, int grid, int nblk) {
  hipLaunchKernelGGL(k_gather<VAR>, dim3(grid), dim3(256), 0, 0, dcodes, nblk, dout, dcyc);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_gather<VAR>, dim3(grid), dim3(256), 0, 0, dcodes, nblk, dout, dcyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<uint64_t> c(grid * 4);
  hipMemcpy(c.data(), dcyc, c.size() * 8, hipMemcpyDeviceToHost);
  double mean = 0;
  for (auto x : c) mean += (double)x;
  mean /= c.size();
  const double lookups = (double)grid * 256 * nblk * 16;  // lane-lookups (each serves 4 queries)
  printf("%-12s %8.1f us  %7.0f cycles/block/wave  %6.2f G lane-lookups/s\n", name, ms * 1e3, mean / nblk,
         lookups / (ms * 1e-3) / 1e9);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = 2 * cus, nblk = 2000;
  std::vector<uint32_t> h(4096 * 4);
  uint32_t x = 12345;
  for (auto& v : h) v = (x = x * 1103515245u + 12345u);
  uint32_t* dc;
  float* dout;
  uint64_t* dcyc;
  hipMalloc(&dc, h.size() * 4);
  hipMalloc(&dout, grid * 256 * 4);
  hipMalloc(&dcyc, grid * 4 * 8);
  hipMemcpy(dc, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  printf("grid %d x 256 threads, %d blocks of 16 steps per wave\n", grid, nblk);
  run<0>("rowmajor_pk", dc, dout, dcyc, grid, nblk);
  run<4>("rowmajor_4add", dc, dout, dcyc, grid, nblk);
  run<1>("skew_cnd", dc, dout, dcyc, grid, nblk);
  run<2>("skew_exec", dc, dout, dcyc, grid, nblk);
  run<3>("skew_nocap", dc, dout, dcyc, grid, nblk);
  return 0;
}
