// Phase-stamp instrumentation of the search kernels (ivfpq_kernels.hip),
// compiled in only by diagnostic builds (profiles/build_variants.sh with
// -DDIAG_STAMPS or -DDIAG_CSTAMPS; read back by profiles/diag_stamps.py and
// profiles/diag_coarse.py through ivfpq_diag_stamps).  In the shipped library
// every macro below is empty.
#pragma once

#if defined(DIAG_STAMPS) || defined(DIAG_CSTAMPS)
namespace chivf {
constexpr int kDiagWG = 1024, kDiagItems = 64, kDiagSlots = 16;
__device__ uint64_t g_diag[kDiagWG * kDiagItems * kDiagSlots];
}  // namespace chivf
#endif

#ifdef DIAG_CSTAMPS  // coarse kernels: stamps per (workgroup, wave) after the wave's memory ops drain
#define CDIAG(slot)                                                                                          \
  do {                                                                                                       \
    __builtin_amdgcn_s_waitcnt(0);                                                                           \
    if (lane == 0 && blockIdx.x < kDiagWG)                                                                   \
      g_diag[((size_t)blockIdx.x * kDiagItems + wave) * kDiagSlots + (slot)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define SDIAG(slot)                                                                                              \
  do {                                                                                                           \
    __builtin_amdgcn_s_waitcnt(0);                                                                               \
    if (lane == 0 && blockIdx.x < kDiagWG)                                                                       \
      g_diag[((size_t)blockIdx.x * kDiagItems + 4 + wave) * kDiagSlots + (slot)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define CDIAG(slot) \
  do {              \
  } while (0)
#define SDIAG(slot) \
  do {              \
  } while (0)
#endif

#ifdef DIAG_STAMPS  // list scan: per-item stamps of workgroup 0's thread 0
#define DIAG(slot, v)                                                                         \
  do {                                                                                        \
    if (tid == 0 && blockIdx.x < kDiagWG && it_no < kDiagItems)                               \
      g_diag[((size_t)blockIdx.x * kDiagItems + it_no) * kDiagSlots + (slot)] = (uint64_t)(v); \
  } while (0)
#define DIAG_ONLY(...) __VA_ARGS__  // statements kept in diagnostic builds only (counters)
#else
#define DIAG(slot, v) \
  do {                \
  } while (0)
#define DIAG_ONLY(...)
#endif
