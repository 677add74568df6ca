// Designed checks of the two runtime behaviours the overlapped-batch design
// relies on ("Batches in flight"); not a stress loop.  Each check
// runs once with a bounded spin kernel (~20 ms of s_memrealtime), no fault path.
//
//  1. hipFree while a kernel of another stream is still running: does hipFree
//     wait for it?  (DevBuf::ensure frees and reallocates slot buffers.)
//  2. hipStreamWaitEvent(B, E) followed by a re-record of E (on B itself, as a
//     slot's `done` event is re-recorded by the search that waited on it, or on
//     another stream): does B still wait for the record it was given?
//  3. The same with more streams than hardware queues (GPU_MAX_HW_QUEUES = 4).
//
// Build: hipcc --offload-arch=gfx950 -O2 -o profiles/hip_semantics profiles/hip_semantics.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                \
    }                                                                              \
  } while (0)

// spins `ticks` of the 100 MHz real-time counter, then every lane stores `val`
// into its own flag element (vector stores only)
__global__ void k_spin_then_set(int* flag, long long ticks, int val) {
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
  flag[threadIdx.x] = val;
}

// out[lane] = flag[lane]
__global__ void k_read(const int* flag, int* out) { out[threadIdx.x] = flag[threadIdx.x]; }

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const long long kSpin = 2000000;  // 20 ms at 100 MHz
  int *flag, *out;
  CK(hipMalloc(&flag, 64 * sizeof(int)));
  CK(hipMalloc(&out, 64 * sizeof(int)));
  std::vector<hipStream_t> st(8);
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int h[64];

  // ---- 1. hipFree vs a running kernel on another stream (the kernel never touches the freed buffer)
  {
    void* p;
    CK(hipMalloc(&p, 64 << 20));
    CK(hipMemset(flag, 0, 64 * sizeof(int)));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_spin_then_set, dim3(1), dim3(64), 0, st[0], flag, kSpin, 1);
    const double t0 = now_ms();
    CK(hipFree(p));
    const double t1 = now_ms();
    const hipError_t q = hipStreamQuery(st[0]);
    CK(hipDeviceSynchronize());
    std::printf("{\"check\": \"hipFree_waits_for_running_kernel\", \"free_ms\": %.3f, \"spin_ms\": 20, "
                "\"kernel_done_when_free_returned\": %s}\n",
                t1 - t0, q == hipSuccess ? "true" : "false");
  }
  // ---- 1b. the same for a small allocation (sub-allocated sizes)
  {
    void* p;
    CK(hipMalloc(&p, 4096));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_spin_then_set, dim3(1), dim3(64), 0, st[0], flag, kSpin, 1);
    const double t0 = now_ms();
    CK(hipFree(p));
    const double t1 = now_ms();
    const hipError_t q = hipStreamQuery(st[0]);
    CK(hipDeviceSynchronize());
    std::printf("{\"check\": \"hipFree_small_waits_for_running_kernel\", \"free_ms\": %.3f, "
                "\"kernel_done_when_free_returned\": %s}\n",
                t1 - t0, q == hipSuccess ? "true" : "false");
  }
  // ---- 1c. hipMalloc right after hipFree: same address?
  {
    void *p, *p2;
    CK(hipMalloc(&p, 1 << 20));
    CK(hipFree(p));
    CK(hipMalloc(&p2, 1 << 20));
    std::printf("{\"check\": \"malloc_after_free_same_address\", \"same\": %s}\n", p == p2 ? "true" : "false");
    CK(hipFree(p2));
  }

  // ---- 2. wait on E, then E re-recorded; variant a: re-record on the waiting stream after
  //         a dependent kernel (the slot `done` pattern); b: on an idle third stream
  for (int variant = 0; variant < 2; variant++) {
    hipEvent_t e;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipMemset(flag, 0, 64 * sizeof(int)));
    CK(hipMemset(out, 0xff, 64 * sizeof(int)));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_spin_then_set, dim3(1), dim3(64), 0, st[0], flag, kSpin, 1);
    CK(hipEventRecord(e, st[0]));
    CK(hipStreamWaitEvent(st[1], e, 0));
    if (variant == 1) CK(hipEventRecord(e, st[2]));
    hipLaunchKernelGGL(k_read, dim3(1), dim3(64), 0, st[1], flag, out);
    if (variant == 0) CK(hipEventRecord(e, st[1]));
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
    int ok = 0;
    for (int i = 0; i < 64; i++) ok += h[i] == 1;
    std::printf("{\"check\": \"wait_then_rerecord_%s\", \"reader_saw_producer\": %s}\n",
                variant == 0 ? "on_waiting_stream" : "on_idle_stream", ok == 64 ? "true" : "false");
    CK(hipEventDestroy(e));
  }

  // ---- 3. a chain over 8 streams (more than the 4 hardware queues): step i waits on the one
  //         shared event, reads step i - 1's flag, spins, sets its own and re-records the event
  {
    hipEvent_t e;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    int *vals, *seen;
    CK(hipMalloc(&vals, 16 * 64 * sizeof(int)));
    CK(hipMalloc(&seen, 16 * 64 * sizeof(int)));
    CK(hipMemset(vals, 0, 16 * 64 * sizeof(int)));
    CK(hipMemset(seen, 0xff, 16 * 64 * sizeof(int)));
    CK(hipDeviceSynchronize());
    for (int i = 0; i < 16; i++) {
      hipStream_t s = st[i % 8];
      if (i > 0) {
        CK(hipStreamWaitEvent(s, e, 0));
        hipLaunchKernelGGL(k_read, dim3(1), dim3(64), 0, s, vals + (i - 1) * 64, seen + i * 64);
      }
      hipLaunchKernelGGL(k_spin_then_set, dim3(1), dim3(64), 0, s, vals + i * 64, kSpin / 10, i + 1);
      CK(hipEventRecord(e, s));
    }
    CK(hipDeviceSynchronize());
    std::vector<int> hv(16 * 64);
    CK(hipMemcpy(hv.data(), seen, hv.size() * sizeof(int), hipMemcpyDeviceToHost));
    int ordered = 0;
    for (int i = 1; i < 16; i++) ordered += hv[i * 64] == i;
    std::printf("{\"check\": \"chain_over_8_streams_ordered\", \"steps_that_saw_predecessor\": %d, \"of\": 15}\n",
                ordered);
    CK(hipFree(vals));
    CK(hipFree(seen));
    CK(hipEventDestroy(e));
  }
  for (auto& s : st) CK(hipStreamDestroy(s));
  CK(hipFree(flag));
  CK(hipFree(out));
  return 0;
}
