// Kernel-boundary hand-off under concurrent streams ("Batches in
// flight"): the pattern of one batch's list scan -> merge, reduced to two kernels.
//
// Per stream s, iteration it:  W writes buffer B_s (every 4-KB chunk by one
// workgroup, value f(it, i)); R, next on the same stream, reads a different chunk
// per workgroup (so mostly on another XCD than its writer) and counts words that
// are not f(it, i).  S streams run their loops with no host synchronisation, so
// one stream's W and R overlap the other streams' kernels.  The reader's L2 may
// hold lines of B_s from R of iteration it - 1 (it read the same addresses).
//
// argv: streams iterations mode [partial]
//   mode 0: plain loads in R
//   mode 1: R starts with an agent-scope acquire fence in every wave
//   mode 2: R starts with a system-scope acquire fence in every wave
//   mode 3: W ends with an agent-scope release fence in every wave
//   mode 4: W holds its workgroups ~50 us after its stores (dirty lines stay in L2
//           while the other streams' kernels start and end)
//   mode 5: as 4, with agent-scope (sc1, write-through) stores in W
//   mode 6: R pinned by XCD: a reader workgroup on XCD x reads chunks x, x + 8, ... (its
//           XCC_ID hardware register), so every chunk is read on the same XCD every
//           iteration and a line that XCD's L2 kept from the previous read would be hit
//   partial = 1: W writes only the first 40 of every 128 bytes (the rest keeps the
//               previous iteration's values; R checks only those 40 bytes)
// Prints one JSON line: mismatching words per stream.
// Build: hipcc --offload-arch=gfx950 -O2 -o profiles/handoff_streams profiles/handoff_streams.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                           \
    }                                                                                         \
  } while (0)

constexpr int kBlocks = 1024;     // chunks of 1024 words (4 KB) each
constexpr int kWords = kBlocks * 1024;

__device__ __forceinline__ unsigned val(unsigned it, unsigned i) { return (it * 2654435761u) ^ (i * 40503u) ^ 0x5bd1e995u; }

__global__ __launch_bounds__(256) void k_write(unsigned* b, unsigned it, int mode, int partial) {
  const unsigned base = blockIdx.x * 1024u;
  for (unsigned t = threadIdx.x; t < 1024u; t += 256u) {
    const unsigned i = base + t;
    if (!partial || (i & 31u) < 10u) {
      if (mode == 5)
        __hip_atomic_store(b + i, val(it, i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        b[i] = val(it, i);
    }
  }
  if (mode == 3) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  if (mode >= 4) {  // bounded hold: 5000 ticks of the 100 MHz counter
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 5000ull) __builtin_amdgcn_s_sleep(8);
  }
}

__global__ __launch_bounds__(256) void k_read(const unsigned* b, unsigned it, int mode, int partial, unsigned* err) {
  if (mode == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (mode == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  unsigned chunk = (blockIdx.x * 37u + 11u) % kBlocks;  // another workgroup's chunk
  if (mode == 6) {
    const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (3 << 11)) & 7u;  // HW_REG_XCC_ID[3:0]
    chunk = (xcc + 8u * (blockIdx.x / 8u)) % kBlocks;
  }
  const unsigned base = chunk * 1024u;
  unsigned bad = 0;
  for (unsigned t = threadIdx.x; t < 1024u; t += 256u) {
    const unsigned i = base + t;
    if (!partial || (i & 31u) < 10u) bad += b[i] != val(it, i);
  }
  if (bad) atomicAdd(err, bad);
}

int main(int argc, char** argv) {
  const int S = argc > 1 ? std::atoi(argv[1]) : 3;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 2000;
  const int mode = argc > 3 ? std::atoi(argv[3]) : 0;
  const int partial = argc > 4 ? std::atoi(argv[4]) : 0;
  std::vector<hipStream_t> st(S);
  std::vector<unsigned*> buf(S);
  unsigned* err;
  CK(hipMalloc(&err, S * sizeof(unsigned)));
  CK(hipMemset(err, 0, S * sizeof(unsigned)));
  for (int s = 0; s < S; s++) {
    CK(hipStreamCreateWithFlags(&st[s], hipStreamNonBlocking));
    CK(hipMalloc(&buf[s], kWords * sizeof(unsigned)));
    CK(hipMemset(buf[s], 0, kWords * sizeof(unsigned)));
  }
  CK(hipDeviceSynchronize());
  for (int it = 1; it <= iters; it++)
    for (int s = 0; s < S; s++) {
      hipLaunchKernelGGL(k_write, dim3(kBlocks), dim3(256), 0, st[s], buf[s], (unsigned)it, mode, partial);
      hipLaunchKernelGGL(k_read, dim3(kBlocks), dim3(256), 0, st[s], buf[s], (unsigned)it, mode, partial, err + s);
    }
  CK(hipDeviceSynchronize());
  std::vector<unsigned> h(S);
  CK(hipMemcpy(h.data(), err, S * sizeof(unsigned), hipMemcpyDeviceToHost));
  std::printf("{\"streams\": %d, \"iters\": %d, \"mode\": %d, \"partial\": %d, \"bad_words\": [", S, iters, mode, partial);
  for (int s = 0; s < S; s++) std::printf("%s%u", s ? ", " : "", h[s]);
  std::printf("]}\n");
  return 0;
}
