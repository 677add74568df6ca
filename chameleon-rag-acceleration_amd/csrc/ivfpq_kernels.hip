// gfx950 (MI355X, CDNA4) kernels for IVF-PQ search.
//
// Hot path: coarse probe -> distance LUT -> PQ-code scan
// -> top-k.  The reference runs it in Faiss (IndexIVFPQ::search ->
// IVFPQScanner::scan_list_with_table; faiss-gpu pqScanPrecomputedMultiPass +
// pass1/pass2SelectLists, Chameleon/Faiss_experiments/MICRO_GPU_profiling/
// classify_stages.py:127-136) and on the FPGA (retrieval_accelerator/
// entire_accelerator_final_SIFT_M16/src/{LUT_construction,ADC}.hpp).
//
// Design, four launches per batch (C2):
//  * k_coarse_gemm: the coarse key tiles on the matrix cores
//    (v_mfma_f32_16x16x4_f32, ascending k = the oracle's fmaf chain) and, in
//    the same launch, T3 workgroups (per query and sub-quantizer, Faiss tree
//    order); nlist >= 8192 uses k_coarse_segtop + k_coarse_select_cand instead
//    (no [B x nlist] key matrix);
//  * k_coarse_select: per query the nprobe nearest lists; its epilogue plans
//    the batch: every (query, probe) pair is bucketed under its list, the
//    query's first usable probe as kind 0, the others as kind 1;
//  * k_scan_lists: persistent workgroups that derive their work items (list,
//    up to G pairs, kind 0 first) from the per-list counts; per item the G
//    LUTs (T1[list] - 2 T3[q], or -T3[q] for IP) are formed in LDS (the LUT
//    never touches HBM), the list's PQ codes are streamed coalesced and every
//    code is summed from M LDS lookups per query; top-k is fused into the scan
//    (per-wave candidate queue + DPP wave top-k in registers, admission against
//    the query's running k-th key shared through atomicMin), so no distance is
//    ever written to memory, only each wave's partial top-k;
//  * k_merge_probes (k <= 64) / k_merge_big (k > 64): per query the partial
//    lists of its probes, labels looked up for survivors only.
// Every fp32 operation follows the oracle's order (oracle/ivfpq_oracle.c,
// Faiss 1.7.1 AVX order); the library is compiled with -ffp-contract=off and
// the only FMAs are the explicit fmaf() of the coarse inner product and the
// LUT's T1 + (-2) T3 (exact product, so one rounding either way).
#include <float.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include <hip/hip_runtime.h>

#include "ivfpq_kernels.h"
#include "ivfpq_diag.h"

namespace chivf {

namespace {

constexpr float kInf = __builtin_huge_valf();

enum { K_IP = 0, K_L2 = 1, K_NORM = 2 };

// Faiss-1.7.1 AVX reduction order (see or_tree in oracle/ivfpq_oracle.c).
// fx(t), fy(t) return element t of the two operands.
template <int KIND, class FX, class FY>
__device__ __forceinline__ float tree(FX fx, FY fy, int d) {
  float a8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int i = 0;
  for (; i + 8 <= d; i += 8) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      float p;
      if (KIND == K_IP) {
        p = fx(i + j) * fy(i + j);
      } else if (KIND == K_L2) {
        float t = fx(i + j) - fy(i + j);
        p = t * t;
      } else {
        float v = fx(i + j);
        p = v * v;
      }
      a8[j] = a8[j] + p;
    }
  }
  float a4[4];
#pragma unroll
  for (int j = 0; j < 4; j++) a4[j] = a8[j + 4] + a8[j];
#pragma unroll
  for (int pass = 0; pass < 2; pass++) {
    // pass 0: the 4-wide remainder (d - i >= 4); pass 1: the masked tail
    if (pass == 0 && i + 4 > d) continue;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (i + j < d) {
        float p;
        if (KIND == K_IP) {
          p = fx(i + j) * fy(i + j);
        } else if (KIND == K_L2) {
          float t = fx(i + j) - fy(i + j);
          p = t * t;
        } else {
          float v = fx(i + j);
          p = v * v;
        }
        a4[j] = a4[j] + p;
      }
    }
    if (pass == 0) i += 4;
  }
  float h0 = a4[0] + a4[1];
  float h1 = a4[2] + a4[3];
  return h0 + h1;
}

// Branch-free (bitwise, not short-circuit) so that the networks below compile
// to compare masks and selects instead of divergent branches.
template <class T>
__device__ __forceinline__ bool lexless(float ad, T ai, float bd, T bi) {
  return (ad < bd) | ((ad == bd) & (ai < bi));
}

__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// Cross-lane moves on the VALU (DPP) instead of the LDS crossbar (ds_bpermute):
// wave_shr:1 shifts the whole wave by one lane, lane 0 receiving `old`.
__device__ __forceinline__ int dpp_shr1_i(int old, int v) { return __builtin_amdgcn_update_dpp(old, v, 0x138, 0xf, 0xf, false); }
__device__ __forceinline__ float shr1_f(float old, float v) {
  return __int_as_float(dpp_shr1_i(__float_as_int(old), __float_as_int(v)));
}

// lane ^ J exchange, all on the VALU: DPP for J <= 8, the gfx950 row / half
// swaps for 16 and 32 (v_permlane16_swap / v_permlane32_swap of v with itself:
// the first result holds the partner's value in the odd rows / upper half, the
// second in the even rows / lower half).
template <int CTRL>
__device__ __forceinline__ int dmov(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, false);
}
template <int J>
__device__ __forceinline__ int xor_i(int v) {
  if constexpr (J == 1) return dmov<0xB1>(v);                  // quad_perm [1,0,3,2]
  else if constexpr (J == 2) return dmov<0x4E>(v);             // quad_perm [2,3,0,1]
  else if constexpr (J == 4) return dmov<0x1B>(dmov<0x141>(v));  // row_half_mirror, quad_perm [3,2,1,0]
  else if constexpr (J == 8) return dmov<0x128>(v);            // row_ror:8
  else if constexpr (J == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    return (int)((__lane_id() & 16) ? r[0] : r[1]);
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
    return (int)((__lane_id() & 32) ? r[0] : r[1]);
  }
}
template <int J>
__device__ __forceinline__ float xor_f(float v) { return __int_as_float(xor_i<J>(__float_as_int(v))); }
// v[63 - lane] on the VALU: row_mirror, then the half and row swaps (row r -> 3 - r)
__device__ __forceinline__ int rev64_i(int v) { return xor_i<16>(xor_i<32>(dmov<0x140>(v))); }
__device__ __forceinline__ float rev64_f(float v) { return __int_as_float(rev64_i(__float_as_int(v))); }
// v[lane ^ 15] (reverse inside each row of 16)
__device__ __forceinline__ int rev16_i(int v) { return dmov<0x140>(v); }

// Candidate ids: int64 labels / global positions, or int32 positions inside one
// list (the list scan): half the cross-lane traffic of the top-k network.
__device__ __forceinline__ int64_t id_readlane(int64_t v, int lane) {
  const uint64_t u = (uint64_t)v;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), lane);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int64_t id_shr1(int64_t old, int64_t v) {
  const uint64_t uo = (uint64_t)old, uv = (uint64_t)v;
  const uint32_t lo = (uint32_t)dpp_shr1_i((int)(uint32_t)uo, (int)(uint32_t)uv);
  const uint32_t hi = (uint32_t)dpp_shr1_i((int)(uint32_t)(uo >> 32), (int)(uint32_t)(uv >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
template <int J>
__device__ __forceinline__ int id_xor(int v) { return xor_i<J>(v); }
__device__ __forceinline__ int64_t id_rev64(int64_t v) {
  const uint64_t u = (uint64_t)v;
  const uint32_t lo = (uint32_t)rev64_i((int)(uint32_t)u);
  const uint32_t hi = (uint32_t)rev64_i((int)(uint32_t)(u >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
template <int J>
__device__ __forceinline__ int64_t id_xor(int64_t v) {
  const uint64_t u = (uint64_t)v;
  const uint32_t lo = (uint32_t)xor_i<J>((int)(uint32_t)u);
  const uint32_t hi = (uint32_t)xor_i<J>((int)(uint32_t)(u >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int lane) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shr1_u64(uint64_t old, uint64_t v) {
  const uint32_t lo = (uint32_t)dpp_shr1_i((int)(uint32_t)old, (int)(uint32_t)v);
  const uint32_t hi = (uint32_t)dpp_shr1_i((int)(uint32_t)(old >> 32), (int)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
template <class T>
__device__ __forceinline__ constexpr T id_none() {
  if constexpr (sizeof(T) == 8) return (T)kSentinelId;
  else return (T)INT32_MAX;
}

// A wave's running k best (key, id) pairs, sorted ascending across
// R rows x 64 lanes (logical index r*64 + lane).  Requires k <= 64*R.
template <int R, class T = int64_t>
struct WaveTopK {
  float d[R];
  T id[R];
  float td;  // current k-th best (the admission threshold)
  T ti;
  int krow, klane;

  __device__ __forceinline__ void init(int k) {
#pragma unroll
    for (int r = 0; r < R; r++) {
      d[r] = kInf;
      id[r] = id_none<T>();
    }
    td = kInf;
    ti = id_none<T>();
    krow = (k - 1) >> 6;
    klane = (k - 1) & 63;
  }

  __device__ __forceinline__ void refresh_tau() {
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (r == krow) {
        td = readlane_f(d[r], klane);
        ti = id_readlane(id[r], klane);
      }
    }
  }

  // Insert the candidates (cd, ci) of the lanes set in `mask` (wave-uniform).
  __device__ __forceinline__ void insert(uint64_t mask, float cd, T ci, int lane) {
    while (mask) {
      const int src = __builtin_ctzll(mask);
      mask &= mask - 1;
      const float vd = readlane_f(cd, src);
      const T vi = id_readlane(ci, src);
      if (!lexless(vd, vi, td, ti)) continue;  // overtaken by an earlier insert
      int pos = 0;
#pragma unroll
      for (int r = 0; r < R; r++) pos += __popcll(__ballot(lexless(d[r], id[r], vd, vi)));
#pragma unroll
      for (int r = R - 1; r >= 0; r--) {
        if ((r + 1) * 64 <= pos) continue;  // row entirely before the slot
        float cdd = vd;
        T cii = vi;
        if (r > 0) {
          cdd = readlane_f(d[r - 1], 63);
          cii = id_readlane(id[r - 1], 63);
        }
        const float ud = shr1_f(cdd, d[r]);
        const T ui = id_shr1(cii, id[r]);
        const int idx = r * 64 + lane;
        d[r] = idx > pos ? ud : (idx == pos ? vd : d[r]);
        id[r] = idx > pos ? ui : (idx == pos ? vi : id[r]);
      }
      refresh_tau();
    }
  }
};

// Merge up to 64 candidates (one per lane; (inf, sentinel) = none) into a
// single-row top-k: bitonic sort of the candidates, then the classic
// reverse-min + bitonic merge against the sorted row.  Exchanges at strides
// are VALU lane moves (xor_i).
template <int KK, int J, class T>
__device__ __forceinline__ void bitonic_step(float& cd, T& ci, int lane) {
  const float od = xor_f<J>(cd);
  const T oi = id_xor<J>(ci);
  const bool want_min = ((lane & J) == 0) == ((lane & KK) == 0);
  const bool o_lt = lexless(od, oi, cd, ci);
  const bool c_lt = lexless(cd, ci, od, oi);
  const bool take = (want_min & o_lt) | (!want_min & c_lt);
  cd = take ? od : cd;
  ci = take ? oi : ci;
}
template <int KK, int J, class T>
__device__ __forceinline__ void bitonic_steps(float& cd, T& ci, int lane) {
  if constexpr (J >= 1) {
    bitonic_step<KK, J>(cd, ci, lane);
    bitonic_steps<KK, J / 2>(cd, ci, lane);
  }
}
template <int KK, class T>
__device__ __forceinline__ void bitonic_sort64(float& cd, T& ci, int lane) {
  if constexpr (KK <= 64) {
    bitonic_steps<KK, KK / 2>(cd, ci, lane);
    bitonic_sort64<KK * 2>(cd, ci, lane);
  }
}

template <class T>
__device__ __forceinline__ void bulk_merge_row(WaveTopK<1, T>& tk, float cd, T ci, int lane) {
  bitonic_sort64<2>(cd, ci, lane);
  const float rd = rev64_f(cd);
  const T ri = id_rev64(ci);
  {
    const bool t = lexless(rd, ri, tk.d[0], tk.id[0]);
    tk.d[0] = t ? rd : tk.d[0];
    tk.id[0] = t ? ri : tk.id[0];
  }
  // ascending bitonic merge: KK = 128 keeps every lane "up"
  bitonic_steps<128, 32>(tk.d[0], tk.id[0], lane);
  tk.refresh_tau();
}

// The same into an R-row top-k: the sorted candidates cascade down the rows,
// each row keeping the lower half of (row, carry) and passing the upper half on.
template <int R, class T>
__device__ __forceinline__ void bulk_merge_rows(WaveTopK<R, T>& tk, float cd, T ci, int lane) {
  bitonic_sort64<2>(cd, ci, lane);
#pragma unroll
  for (int r = 0; r < R; r++) {
    const float rd = rev64_f(cd);
    const T ri = id_rev64(ci);
    const bool t = lexless(rd, ri, tk.d[r], tk.id[r]);
    const float lo_d = t ? rd : tk.d[r], hi_d = t ? tk.d[r] : rd;
    const T lo_i = t ? ri : tk.id[r], hi_i = t ? tk.id[r] : ri;
    tk.d[r] = lo_d;
    tk.id[r] = lo_i;
    bitonic_steps<128, 32>(tk.d[r], tk.id[r], lane);
    if (r + 1 < R) {
      cd = hi_d;
      ci = hi_i;
      bitonic_steps<128, 32>(cd, ci, lane);
    }
  }
  tk.refresh_tau();
}

// Merge up to 16 candidates held in lanes 0..15 (others (inf, none)) into a
// single-row top-k with k <= 16: a 16-lane bitonic sort (DPP moves only), the
// reverse-min against lanes 0..15 of the row, a 16-lane bitonic merge.  Only
// lanes 0..15 of the row are kept (the rest are reset to (inf, none)).
template <class T>
__device__ __forceinline__ void row16_merge(WaveTopK<1, T>& tk, float cd, T ci, int lane) {
  bitonic_steps<2, 1>(cd, ci, lane);
  bitonic_steps<4, 2>(cd, ci, lane);
  bitonic_steps<8, 4>(cd, ci, lane);
  bitonic_steps<128, 8>(cd, ci, lane);  // KK = 128: every row ascending
  const float rd = __int_as_float(rev16_i(__float_as_int(cd)));
  T ri;
  if constexpr (sizeof(T) == 8) {
    const uint64_t u = (uint64_t)ci;
    ri = (T)(((uint64_t)(uint32_t)rev16_i((int)(uint32_t)(u >> 32)) << 32) | (uint32_t)rev16_i((int)(uint32_t)u));
  } else {
    ri = (T)rev16_i((int)ci);
  }
  {
    const bool t = lexless(rd, ri, tk.d[0], tk.id[0]);
    tk.d[0] = t ? rd : tk.d[0];
    tk.id[0] = t ? ri : tk.id[0];
  }
  bitonic_steps<128, 8>(tk.d[0], tk.id[0], lane);
  tk.d[0] = lane >= 16 ? kInf : tk.d[0];
  tk.id[0] = lane >= 16 ? id_none<T>() : tk.id[0];
  tk.refresh_tau();
}

// ---- selection when every candidate is known up front ------------------------
// Each lane holds KL (dist, id) entries sorted ascending; the wave emits the k
// smallest overall (k <= 64) into lanes 0..k-1 with a 64-way merge: per output
// one butterfly min across lanes (DPP) and a pop on the owning lane.  No
// per-candidate serial insertion.
template <int KL>
__device__ __forceinline__ void cas_asc(float (&d)[KL], int64_t (&id)[KL], int a, int b) {
  const bool t = lexless(d[b], id[b], d[a], id[a]);
  const float da = d[a], db = d[b];
  const int64_t ia = id[a], ib = id[b];
  d[a] = t ? db : da;
  id[a] = t ? ib : ia;
  d[b] = t ? da : db;
  id[b] = t ? ia : ib;
}

// in-register bitonic sort of KL (power of two) entries, ascending
template <int KL>
__device__ __forceinline__ void lane_sort(float (&d)[KL], int64_t (&id)[KL]) {
#pragma unroll
  for (int kk = 2; kk <= KL; kk <<= 1) {
#pragma unroll
    for (int j = kk >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int i = 0; i < KL; i++) {
        const int pj = i ^ j;
        if (pj > i) {
          if ((i & kk) == 0)
            cas_asc<KL>(d, id, i, pj);
          else
            cas_asc<KL>(d, id, pj, i);
        }
      }
    }
  }
}

template <int J>
__device__ __forceinline__ void min_step(float& d, int64_t& id) {
  const float od = xor_f<J>(d);
  const int64_t oi = id_xor<J>(id);
  const bool t = lexless(od, oi, d, id);
  d = t ? od : d;
  id = t ? oi : id;
}

// lanes' lists sorted ascending -> the k smallest into (out_d, out_id) of lanes 0..k-1
template <int KL>
__device__ __forceinline__ void wave_kway(float (&d)[KL], int64_t (&id)[KL], int k, int lane, float& out_d,
                                          int64_t& out_id) {
  out_d = kInf;
  out_id = kSentinelId;
  for (int t = 0; t < k; t++) {
    float md = d[0];
    int64_t mi = id[0];
    min_step<1>(md, mi);
    min_step<2>(md, mi);
    min_step<4>(md, mi);
    min_step<8>(md, mi);
    min_step<16>(md, mi);
    min_step<32>(md, mi);
    // every lane now holds the minimum; the first lane whose head equals it pops
    const uint64_t own = __ballot(d[0] == md && id[0] == mi);
    if (lane == __builtin_ctzll(own)) {
#pragma unroll
      for (int j = 0; j < KL - 1; j++) {
        d[j] = d[j + 1];
        id[j] = id[j + 1];
      }
      d[KL - 1] = kInf;
      id[KL - 1] = kSentinelId;
    }
    if (lane == t) {
      out_d = md;
      out_id = mi;
    }
  }
}

// k-th smallest (k <= 64) of the wave's 64 values: ascending bitonic sort of
// the values alone (no ids), then a readlane.
__device__ __forceinline__ float wave_kth_smallest(float m, int k, int lane) {
#pragma unroll
  for (int kk = 2; kk <= 64; kk <<= 1) {
#pragma unroll
    for (int j = kk >> 1; j > 0; j >>= 1) {
      float o;
      switch (j) {
        case 1: o = xor_f<1>(m); break;
        case 2: o = xor_f<2>(m); break;
        case 4: o = xor_f<4>(m); break;
        case 8: o = xor_f<8>(m); break;
        case 16: o = xor_f<16>(m); break;
        default: o = xor_f<32>(m); break;
      }
      const bool up = (lane & kk) == 0 || kk == 64;
      const bool lower = (lane & j) == 0;
      m = (lower == up) ? fminf(m, o) : fmaxf(m, o);
    }
  }
  return readlane_f(m, k - 1);
}

// order-preserving int image of a float (signed int compare == float compare),
// for atomicMin on keys that may be negative (IP keys, rounding-negative L2)
__device__ __forceinline__ int f2ord(float f) {
  const int b = __float_as_int(f);
  return b >= 0 ? b : b ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float ord2f(int o) { return __int_as_float(o >= 0 ? o : o ^ 0x7FFFFFFF); }

// ------------------------------------------------------------------ norms
// Eight lanes per row (8 rows per 64-thread workgroup): lane j of a row's group
// holds tree()'s accumulator a8[j] (elements j, j + 8, ... in order), so a 768-d
// row is 96 dependent adds per lane instead of 768 in one thread; the group's
// combine, the 4-wide remainder and the masked tail then follow tree() exactly.
__global__ __launch_bounds__(64) void k_row_norms(const float* __restrict__ x, int64_t n, int d,
                                                  float* __restrict__ out) {
  const int lane = threadIdx.x, j = lane & 7;
  const int64_t i = (int64_t)blockIdx.x * 8 + (lane >> 3);
  const bool ok = i < n;
  const float* xi = x + (ok ? i : 0) * d;
  const int d8 = d & ~7;
  float a = 0.f;
  int t = 0;
  if (ok) {
    for (; t + 32 <= d8; t += 32) {  // four loads in flight per lane, adds in element order
      const float v0 = xi[t + j], v1 = xi[t + 8 + j], v2 = xi[t + 16 + j], v3 = xi[t + 24 + j];
      a = a + v0 * v0;
      a = a + v1 * v1;
      a = a + v2 * v2;
      a = a + v3 * v3;
    }
    for (; t < d8; t += 8) {
      const float v = xi[t + j];
      a = a + v * v;
    }
  }
  const float hi4 = __shfl_down(a, 4, 8);  // a8[j + 4] for j < 4
  float a4 = hi4 + a;                       // a4[j] = a8[j + 4] + a8[j]
  int r = d8;
  if (r + 4 <= d) {  // the 4-wide remainder
    if (ok && j < 4) {
      const float v = xi[r + j];
      a4 = a4 + v * v;
    }
    r += 4;
  }
  if (ok && j < 4 && r + j < d) {  // the masked tail
    const float v = xi[r + j];
    a4 = a4 + v * v;
  }
  const float h = a4 + __shfl_down(a4, 1, 8);  // lane 0: a4[0] + a4[1], lane 2: a4[2] + a4[3]
  const float h1 = __shfl_down(h, 2, 8);
  if (ok && j == 0) out[i] = h + h1;
}

// ------------------------------------------------- coarse key matrix (split path)
// 64 x 64 output tile per 256-thread workgroup, 4 x 4 per thread, K staged in
// LDS 16 at a time.  Each output's inner product is a k-ordered fmaf chain.
constexpr int DT_B = 64;
constexpr int DT_K = 16;

__global__ __launch_bounds__(256) void k_l2_dist(const float* __restrict__ x, const float* __restrict__ xn,
                                                 int64_t nx, const float* __restrict__ c,
                                                 const float* __restrict__ cn, int nc, int d,
                                                 float* __restrict__ out, int ip) {
  __shared__ float xs[DT_K][DT_B + 4];
  __shared__ float cs[DT_K][DT_B + 4];
  const int tid = threadIdx.x;
  const int tx = tid & 15, ty = tid >> 4;
  const int64_t row0 = (int64_t)blockIdx.y * DT_B;
  const int64_t col0 = (int64_t)blockIdx.x * DT_B;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[i][j] = 0.f;

  for (int k0 = 0; k0 < d; k0 += DT_K) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int e = tid + 256 * u;
      const int r = e >> 4, kk = e & 15;
      const bool kin = k0 + kk < d;
      xs[kk][r] = (row0 + r < nx && kin) ? x[(row0 + r) * d + k0 + kk] : 0.f;
      cs[kk][r] = (col0 + r < nc && kin) ? c[(col0 + r) * d + k0 + kk] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < DT_K; kk++) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; i++) av[i] = xs[kk][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; j++) bv[j] = cs[kk][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = __builtin_fmaf(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int64_t r = row0 + ty * 4 + i;
    if (r >= nx) continue;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int64_t cc = col0 + tx * 4 + j;
      if (cc >= nc) continue;
      float dis;
      if (ip) {
        dis = -acc[i][j];
      } else {
        dis = (xn[r] + cn[cc]) - 2.0f * acc[i][j];
        if (dis < 0.f) dis = 0.f;
      }
      out[r * nc + cc] = dis;
    }
  }
}

// ---------------------------------------------------------- planning helpers
// One (query, probe) pair of a batch: kind 0 when it is the query's first
// usable probe, else kind 1; bucketed under its list with the scan's dis0.
__device__ __forceinline__ void plan_pair(const ListPlan& pl, int nloc, int64_t l, int lo, int kind, int pair,
                                          float dis0) {
  const int s = atomicAdd(&pl.cnt[kind * nloc + (int)(l - lo)], 1);
  // a list holds at most one pair per query and kind, so s < cap (deduplicated rows)
  if (s < pl.cap) pl.bucket[((int64_t)(l - lo) * 2 + kind) * pl.cap + s] = make_int2(pair, __float_as_int(dis0));
  pl.pd0[pair] = dis0;  // the same dis0 for a merge that has to rescan the pair (repair_probe)
}

// The query bound tau_q of this batch (an order-preserving int; "no bound" =
// f2ord(inf) when the word still carries an earlier batch's tag).  Agent-scope
// atomic load: other workgroups lower the word while this one runs, so the read
// must not be served from a non-coherent cached copy.
__device__ __forceinline__ int tau_get(const ListPlan& pl, int64_t q) {
  const uint64_t v = __hip_atomic_load(pl.tauq + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // One value for the whole wave.  The lanes' loads of this word are separate
  // requests, and another workgroup's atomicMin can land between them: lanes would
  // then hold different bounds, and every "wave-uniform" branch on the bound
  // (loose / fast admission / queue fills) would diverge -- the wrong-rows failure
  // under concurrent kernels ("Uniform bounds").
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  return hi == ~pl.epoch ? (int)(lo ^ 0x80000000u) : f2ord(kInf);
}
// tau_get in two halves: the agent-scope load (kept in flight as a raw word) and
// its wave-uniform decode at the use
__device__ __forceinline__ uint64_t tau_load(const ListPlan& pl, int64_t q) {
  return __hip_atomic_load(pl.tauq + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int tau_decode(const ListPlan& pl, uint64_t v) {
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));  // (see tau_get)
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  return hi == ~pl.epoch ? (int)(lo ^ 0x80000000u) : f2ord(kInf);
}
// tau_q := min(tau_q, o) within this batch (any k real candidates bound the final k-th key)
__device__ __forceinline__ void tau_lower(const ListPlan& pl, int64_t q, int o) {
  const uint64_t w = ((uint64_t)(~pl.epoch) << 32) | ((uint32_t)o ^ 0x80000000u);
  atomicMin(reinterpret_cast<unsigned long long*>(pl.tauq + q), (unsigned long long)w);
}
// ---- self-identifying partial lists ("Tagged partial lists")
// Every per-wave partial-list entry is one 16-B record {key bits, tag, code
// position (int64)} written by one store; the tag's low 28 bits name the batch
// (the workspace epoch) and the slot, its high 4 bits the XCD of the writer.  A
// reader that finds another tag has read memory this batch's scan did not leave
// there (a lost, late or misdirected store): the merges never use such an entry
// and rescan that probe's list instead (k_merge_probes, repair_probe).
constexpr uint32_t kTagMask = 0x0FFFFFFFu;
__device__ __forceinline__ uint32_t part_tag(uint32_t epoch, int64_t slot) {
  return (epoch * 0x9E3779B1u + (uint32_t)slot) & kTagMask;
}
// this wave's XCD (hwreg XCC_ID bits 3:0) in the tag's top nibble
__device__ __forceinline__ uint32_t xcc_tag() {
  return ((uint32_t)__builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11)) & 15u) << 28;
}
__device__ __forceinline__ uint4 part_rec(float key, uint32_t tag, int64_t pos) {
  return make_uint4(__float_as_uint(key), tag, (uint32_t)(uint64_t)pos, (uint32_t)((uint64_t)pos >> 32));
}
__device__ __forceinline__ bool tag_ok(uint32_t t, uint32_t expect) { return ((t ^ expect) & kTagMask) == 0; }
__device__ __forceinline__ float rec_key(const uint4& r) { return __uint_as_float(r.x); }
__device__ __forceinline__ int64_t rec_pos(const uint4& r) { return (int64_t)(((uint64_t)r.w << 32) | r.z); }

// a code position read back from a partial list, checked against the image
// (counted in pl.err and dropped when outside it: never dereferenced)
__device__ __forceinline__ bool pos_ok(const ScanArgs& a, const ListPlan& pl, int64_t pos) {
  const bool bad = pos >= a.n_codes;
  if (bad) atomicAdd(pl.err, 1);
  return pos >= 0 && !bad;
}

// List-major planning request for the coarse selection's epilogue.
struct CoarsePlan {
  ListPlan pl;
  int on = 0;                         // 0: no planning (nprobe > 64, or not requested)
  const int64_t* list_off = nullptr;
  int lo = 0, hi = 0;
  const float* cent = nullptr;        // [nlist][d] row-major (IP dis0)
};

// ------------------------------------------------------------ row select
template <int R>
__global__ __launch_bounds__(256) void k_select_rows(const float* __restrict__ dist, int64_t nrows, int ncols,
                                                     int n, float* __restrict__ ov, int64_t* __restrict__ oc,
                                                     int neg) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= nrows) return;  // wave-uniform
  WaveTopK<R> tk;
  tk.init(n);
  const float* drow = dist + row * ncols;
  for (int base = 0; base < ncols; base += 64) {
    const int cix = base + lane;
    const bool valid = cix < ncols;
    const float v = valid ? drow[cix] : kInf;
    const bool pass = valid && lexless(v, (int64_t)cix, tk.td, tk.ti);
    const uint64_t mask = __ballot(pass);
    if (!mask) continue;
    if constexpr (R == 1) {
      if (__popcll(mask) > 6) {
        bulk_merge_row(tk, pass ? v : kInf, pass ? (int64_t)cix : kSentinelId, lane);
        continue;
      }
    }
    tk.insert(mask, v, (int64_t)cix, lane);
  }
  const float pad = neg ? -FLT_MAX : FLT_MAX;
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int idx = r * 64 + lane;
    if (idx < n) {
      const bool empty = tk.id[r] == kSentinelId;
      ov[row * n + idx] = empty ? pad : (neg ? -tk.d[r] : tk.d[r]);
      oc[row * n + idx] = empty ? -1 : tk.id[r];
    }
  }
}

// ------------------------------------------------- coarse probe (MFMA path)
// (key, column) packed so that unsigned 64-bit order is (key asc, column asc).
// (-0 is folded into +0 first: the float order has them equal)
__device__ __forceinline__ uint64_t pack_kc(float key, int col) {
  return ((uint64_t)((uint32_t)f2ord(key + 0.0f) ^ 0x80000000u) << 32) | (uint32_t)col;
}
__device__ __forceinline__ float kc_key(uint64_t p) { return ord2f((int)((uint32_t)(p >> 32) ^ 0x80000000u)); }
constexpr uint64_t kKcNone = ~0ull;

template <int J>
__device__ __forceinline__ uint64_t xor_u64(uint64_t v) {
  const uint32_t lo = (uint32_t)xor_i<J>((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)xor_i<J>((int)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
// one compare-exchange step of the bitonic network on packed keys
template <int KK, int J>
__device__ __forceinline__ void kc_step(uint64_t& p, int lane) {
  const uint64_t o = xor_u64<J>(p);
  const bool up = KK >= 64 || (lane & KK) == 0;
  const bool take_min = ((lane & J) == 0) == up;
  p = ((o < p) == take_min) ? o : p;
}
template <int KK, int J>
__device__ __forceinline__ void kc_steps(uint64_t& p, int lane) {
  if constexpr (J >= 1) {
    kc_step<KK, J>(p, lane);
    kc_steps<KK, J / 2>(p, lane);
  }
}
template <int KK = 2>
__device__ __forceinline__ void kc_sort64(uint64_t& p, int lane) {  // ascending across the wave
  if constexpr (KK <= 64) {
    kc_steps<KK, KK / 2>(p, lane);
    kc_sort64<KK * 2>(p, lane);
  }
}
// run (sorted asc) := the 64 smallest of run and p (p sorted asc)
__device__ __forceinline__ void kc_merge64(uint64_t& run, uint64_t p, int lane) {
  const uint32_t lo = (uint32_t)rev64_i((int)(uint32_t)p);
  const uint32_t hi = (uint32_t)rev64_i((int)(uint32_t)(p >> 32));
  const uint64_t rev = ((uint64_t)hi << 32) | lo;
  run = rev < run ? rev : run;  // bitonic: ascending run vs descending p
  kc_steps<128, 32>(run, lane);
}

// Key matrix of the coarse quantizer on the matrix cores: keys[q][c] =
// max(0, (|x_q|^2 + |c|^2) - 2 <x_q, c>) (L2) or -<x_q, c> (IP), where <.,.>
// is accumulated by v_mfma_f32_16x16x4_f32 in ascending k, which rounds like
// the k-ordered fmaf chain of the oracle (checked bit for bit on gfx950).
// Workgroup = 16 queries x 256 centroids (wave w: 4 tiles of 16 centroids).
// Workgroups past the key tiles build T3 [nq][M][256] (Faiss tree order) for
// 16 queries x 1024 entries each, when T3out is set.
constexpr int GQ = 16, GC = 128;

// rows q0..q0+15 of x transposed into xs[dk][16] (k-major; zeros past nq and d)
__device__ __forceinline__ void fill_cols(float* xs, const float* __restrict__ x, int64_t q0, int64_t nq, int d,
                                          int dk, int tid) {
  if ((d & 3) == 0 && d <= 1024) {
    const int nk4 = dk / 4;  // thread k4: elements 4 k4 .. 4 k4 + 3 of the 16 rows
    for (int k4 = tid; k4 < nk4; k4 += 256) {
      float4 r[GQ];
#pragma unroll
      for (int i = 0; i < GQ; i++)
        r[i] = (q0 + i < nq && 4 * k4 < d) ? reinterpret_cast<const float4*>(x + (q0 + i) * d)[k4]
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
      float4* row = reinterpret_cast<float4*>(xs + 4 * k4 * GQ);  // 4 k-rows of 16 floats
#pragma unroll
      for (int i4 = 0; i4 < GQ / 4; i4++) {
        row[0 * 4 + i4] = make_float4(r[4 * i4].x, r[4 * i4 + 1].x, r[4 * i4 + 2].x, r[4 * i4 + 3].x);
        row[1 * 4 + i4] = make_float4(r[4 * i4].y, r[4 * i4 + 1].y, r[4 * i4 + 2].y, r[4 * i4 + 3].y);
        row[2 * 4 + i4] = make_float4(r[4 * i4].z, r[4 * i4 + 1].z, r[4 * i4 + 2].z, r[4 * i4 + 3].z);
        row[3 * 4 + i4] = make_float4(r[4 * i4].w, r[4 * i4 + 1].w, r[4 * i4 + 2].w, r[4 * i4 + 3].w);
      }
    }
  } else {
    for (int e = tid; e < GQ * dk; e += 256) {
      const int i = e / dk, k = e % dk;
      xs[k * GQ + i] = (q0 + i < nq && k < d) ? x[(q0 + i) * d + k] : 0.f;
    }
  }
}

struct CoarseT3 {
  float* out = nullptr;  // [nq][M * 256]
  const float* cb = nullptr;
  int M = 0;
  int nblk = 0;  // T3 workgroups
  // the queries of the tables: the key tiles' own queries, or (the list-range shard
  // step) the whole global batch while the key tiles cover this rank's slice
  const float* x = nullptr;
  int64_t nq = 0;
};

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int NTL = GC / 64;  // 16 x 16 MFMA tiles per wave (32 centroids)

// Stage the A operand of a key tile (rows q0..q0+15 transposed, zero-padded to
// dk) and |x_q|^2 in Faiss tree order into LDS (xs [dk][16], xn [16] + 128
// floats of scratch).  Ends with the block barrier that publishes xs; xn is
// published by the caller's next barrier.
__device__ __forceinline__ void coarse_stage_queries(float* xs, float* xn, const float* __restrict__ x, int64_t q0,
                                                     int64_t nq, int d, int dk, int tid) {
  fill_cols(xs, x, q0, nq, d, dk, tid);
  __syncthreads();
  // with d % 8 == 0 the 8 lane sums of each query are 8 independent sequential
  // chains (threads i * 8 + j), folded by 16 threads
  float* a8 = xn + GQ;  // [GQ][8]
  if (d % 8 == 0) {
    if (tid < GQ * 8) {
      const int i = tid >> 3, j = tid & 7;
      float acc8 = 0.f;
      for (int k = j; k < d; k += 8) {
        const float v = xs[k * GQ + i];
        acc8 = acc8 + v * v;
      }
      a8[i * 8 + j] = acc8;
    }
    __syncthreads();
    if (tid < GQ) {
      const float* r = a8 + tid * 8;
      const float h0 = (r[4] + r[0]) + (r[5] + r[1]);
      const float h1 = (r[6] + r[2]) + (r[7] + r[3]);
      xn[tid] = h0 + h1;
    }
  } else if (tid < GQ) {
    xn[tid] = tree<K_NORM>([&](int t) { return xs[t * GQ + tid]; }, [&](int t) { return xs[t * GQ + tid]; }, d);
  }
}

// acc[t] = the wave's 16 x 16 tiles <x_q, c> for its 16 queries (A rows arow0 ..
// arow0 + 15 of xs [dk][lda]) and centroids c0 + 16 t .. + 15, accumulated by
// v_mfma_f32_16x16x4_f32 in ascending k (rounds like the oracle's k-ordered
// fmaf chain).  B rows past d are clamped to row d - 1: their A entries are 0
// and fma(0, b, acc) == acc for every finite b (acc is never -0).  B rows are
// streamed from global in chunks of KS k-steps, two chunks in flight.
template <int NT = NTL, int KS = 8>
__device__ __forceinline__ void coarse_key_tile(f4 (&acc)[NT], const float* xs, int lda, int arow0,
                                                const float* __restrict__ centT, int ldc, int nlist, int d, int dk,
                                                int c0, int lane) {
  static_assert(64 % (8 * KS) == 0, "dk is padded to 64");
#pragma unroll
  for (int t = 0; t < NT; t++) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
  const int i16 = lane & 15, k4 = lane >> 4;
  const float* bcol[NT];
#pragma unroll
  for (int t = 0; t < NT; t++) bcol[t] = centT + min(c0 + t * 16 + i16, nlist - 1);  // clamped columns
  float b0[KS][NT], b1[KS][NT];
  auto load_b = [&](int k0, float (&b)[KS][NT]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < KS; j++) {
      const int64_t kr = min(k0 + 4 * j + k4, d - 1);
#pragma unroll
      for (int t = 0; t < NT; t++) b[j][t] = bcol[t][kr * ldc];
    }
  };
  auto mma = [&](int k0, const float (&b)[KS][NT]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < KS; j++) {
      const float av = xs[(k0 + 4 * j + k4) * lda + arow0 + i16];
#pragma unroll
      for (int t = 0; t < NT; t++) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b[j][t], acc[t], 0, 0, 0);
    }
  };
  constexpr int CH = 4 * KS;  // k per chunk
  // chunks up to the first multiple of CH at or past d (the staged A rows are zero up to
  // dk >= kend; an all-zero chunk would leave every accumulator unchanged): d = 96 takes
  // 3 chunks, not the 4 of its 64-padded staging
  const int kend = min(dk, (d + CH - 1) / CH * CH);
  load_b(0, b0);
  for (int k0 = 0; k0 < kend; k0 += 2 * CH) {
    load_b(k0 + CH, b1);  // past the end on the last pass: clamped, unused
    mma(k0, b0);
    if (k0 + CH >= kend) break;
    load_b(k0 + 2 * CH, b0);
    mma(k0 + CH, b1);
  }
}

// the quantizer key from <x, c>: L2 max(0, (|x|^2 + |c|^2) - 2 <x, c>), IP -<x, c>
__device__ __forceinline__ float coarse_key(float dot, float xn, float cn, int ip) {
  if (ip) return -dot;
  const float v = (xn + cn) - 2.0f * dot;
  return v < 0.f ? 0.f : v;
}

template <int HOIST>
__global__ __launch_bounds__(256) void k_coarse_gemm(const float* __restrict__ x, int64_t nq, int d,
                                                     const float* __restrict__ centT, int ldc,
                                                     const float* __restrict__ cn, int nlist,
                                                     float* __restrict__ keys, int ip, int ngemm, CoarseT3 t3) {
  extern __shared__ __attribute__((aligned(16))) float g_lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  CDIAG(0);
  if ((int)blockIdx.x >= ngemm) {
    // ---- T3 role: 16 queries x one sub-quantizer (256 entries, one per thread)
    const int tb = blockIdx.x - ngemm;
    const int total = t3.M * 256;
    const int dsub = d / t3.M;
    x = t3.x;
    nq = t3.nq;
    const int64_t q0 = (int64_t)(tb / t3.M) * GQ;
    const int m = tb % t3.M;
    const int e = m * 256 + tid;
    // the centroid is loaded before the sub-vectors are staged: one round trip, not two
    float4 c0 = {}, c1 = {};
    if (dsub == 8) {
      const float4* src = reinterpret_cast<const float4*>(t3.cb + (int64_t)e * 8);
      c0 = src[0];
      c1 = src[1];
    }
    float* xs = g_lds;  // [GQ][dsub]: the queries' sub-vectors m
    for (int i = tid; i < GQ * dsub; i += 256) {
      const int qq = i / dsub;
      xs[i] = q0 + qq < nq ? x[(q0 + qq) * d + m * dsub + (i - qq * dsub)] : 0.f;
    }
    __syncthreads();
    CDIAG(1);
    const int nqq = (int)min<int64_t>(GQ, nq - q0);
    if (dsub == 8) {
      const float w[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
      for (int qq = 0; qq < GQ; qq++) {
        const float4* xv = reinterpret_cast<const float4*>(xs + qq * 8);
        const float4 x0 = xv[0], x1 = xv[1];
        const float xq[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        const float v = tree<K_IP>([&](int t) { return xq[t]; }, [&](int t) { return w[t]; }, 8);
        if (qq < nqq) t3.out[(q0 + qq) * total + e] = v;
      }
    } else {
      const float* cwp = t3.cb + (int64_t)e * dsub;
      for (int qq = 0; qq < nqq; qq++) {
        const float* xq = xs + qq * dsub;
        t3.out[(q0 + qq) * total + e] = tree<K_IP>([&](int t) { return xq[t]; }, [&](int t) { return cwp[t]; }, dsub);
      }
    }
    CDIAG(5);
    return;
  }
  // ---- key tile: 16 queries x 128 centroids
  const int nct = (nlist + GC - 1) / GC;
  const int64_t q0 = (int64_t)(blockIdx.x / nct) * GQ;
  const int c0 = (blockIdx.x % nct) * GC + wave * 32;
  const int dk = (d + 63) & ~63;  // A rows, zero-padded to whole double chunks
  float* xs = g_lds;              // [dk][GQ]: the A operand, k-major
  float* xn = xs + dk * GQ;       // [GQ]
  f4 acc[NTL];
  const int i16 = lane & 15, k4 = lane >> 4;
  // B rows: HOIST = 0 (searches whose scan is k_scan_lean) in 32-deep chunks, two in
  // flight (coarse_key_tile), 74 + 16 registers per lane; HOIST = 1 (every other
  // search, d in (96, 128]) every B row of the wave up front, 148 + 16.  With batches in
  // flight this launch runs in the other stream's scan tail: beside the lean scan's
  // 200-register waves a SIMD fits two HOIST = 0 waves and one HOIST = 1 wave, and the
  // chunked form took the C2 two-in-flight step from 0.128 to 0.1145 ms (r06s); beside
  // k_scan_lists (k > 16: 236 registers) nothing fits, and the up-front loads' shorter
  // latency wins (r05: k = 100 4.74 -> 5.07 M queries/s).  DESIGN.md section 4.
  const bool paired = HOIST && d > 96 && d <= 128;
  if (paired) {
    // the two tiles take interleaved centroids, so a lane's two B values of a row are
    // adjacent: one 8-byte load.  Same ascending-k MFMA chain as coarse_key_tile (rows
    // past d clamped, their A entries 0; columns past nlist read the zero padding of
    // centT or are clamped, and never stored)
    static_assert(NTL == 2, "paired B loads: two tiles per wave");
    float b[32][NTL];
    const int cp2 = min(c0 + 2 * i16, ldc - 2);
#pragma unroll
    for (int j = 0; j < 32; j++) {
      const int64_t kr = min(4 * j + k4, d - 1);
      const float2 v = *reinterpret_cast<const float2*>(centT + kr * ldc + cp2);
      b[j][0] = v.x;
      b[j][1] = v.y;
    }
    coarse_stage_queries(xs, xn, x, q0, nq, d, dk, tid);
    CDIAG(1);
#pragma unroll
    for (int t = 0; t < NTL; t++) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 32; j++) {
      const float av = xs[(4 * j + k4) * GQ + i16];
#pragma unroll
      for (int t = 0; t < NTL; t++) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b[j][t], acc[t], 0, 0, 0);
    }
  } else {
    coarse_stage_queries(xs, xn, x, q0, nq, d, dk, tid);
    CDIAG(1);
    coarse_key_tile(acc, xs, GQ, 0, centT, ldc, nlist, d, dk, c0, lane);
  }
  CDIAG(2);
  __syncthreads();  // xn
#pragma unroll
  for (int t = 0; t < NTL; t++) {
    const int c = paired ? c0 + NTL * i16 + t : c0 + t * 16 + i16;
    if (c >= nlist) continue;
    const float cnv = ip ? 0.f : cn[c];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int i = k4 * 4 + r;
      if (q0 + i >= nq) continue;
      keys[(q0 + i) * nlist + c] = coarse_key(acc[t][r], xn[i], cnv, ip);
    }
  }
  CDIAG(5);
}

// Coarse key matrix for large d (C3: d = 768, nlist = 4096): workgroup = 64
// queries x 128 centroids, wave w = queries 16 w .. 16 w + 15 x all 128 centroids
// (8 tiles of v_mfma_f32_16x16x4_f32).  A (64 x KC) and B (KC x 128) k-chunks are
// staged in LDS, double-buffered, so each centroid column is read from L2 once per
// 64 queries (k_coarse_gemm: once per 16) and each query row once per 128
// centroids.  Every key still accumulates one ascending-k MFMA chain (the
// oracle's fmaf order, as k_coarse_gemm); |x|^2 comes from k_row_norms (same
// Faiss tree order as coarse_stage_queries).  Workgroups past the key tiles build
// T3 as in k_coarse_gemm.
constexpr int TQ = 64, TC = 128, TKC = 32;
constexpr int TAS = TKC + 2;   // A row stride (floats): 2 mod 32 -> conflict-free MFMA A reads
constexpr int TBS = TC + 16;   // B row stride: 16 mod 32 -> conflict-free B reads

__device__ __forceinline__ void t3_role(const float* __restrict__ x, int64_t nq, int d, const CoarseT3& t3, int tb,
                                        float* xs, int tid) {
  const int total = t3.M * 256;
  const int dsub = d / t3.M;
  const int64_t q0 = (int64_t)(tb / t3.M) * GQ;
  const int m = tb % t3.M;
  const int e = m * 256 + tid;
  for (int i = tid; i < GQ * dsub; i += 256) {
    const int qq = i / dsub;
    xs[i] = q0 + qq < nq ? x[(q0 + qq) * d + m * dsub + (i - qq * dsub)] : 0.f;
  }
  __syncthreads();
  const int nqq = (int)min<int64_t>(GQ, nq - q0);
  const float* cwp = t3.cb + (int64_t)e * dsub;
  for (int qq = 0; qq < nqq; qq++) {
    const float* xq = xs + qq * dsub;
    t3.out[(q0 + qq) * total + e] = tree<K_IP>([&](int t) { return xq[t]; }, [&](int t) { return cwp[t]; }, dsub);
  }
}

// The wave's 16 queries x 128 centroids of a 64 x 128 tile (queries q0.., centroids
// c0..), accumulated over d in ascending k: acc[t][r] = <x_{q0 + 16 wave + 4 k4 + r},
// c_{c0 + 16 t + i16}>.  As / Bs are the double-buffered staging tiles; every wave
// of the workgroup must call it (barriers), and they are free again on return.
__device__ __forceinline__ void tiled_key_acc(f4 (&acc)[TC / 16], const float* __restrict__ x, int64_t q0, int64_t nq,
                                              int d, const float* __restrict__ centT, int ldc, int c0,
                                              float (*As)[TQ * TAS], float (*Bs)[TKC * TBS], int tid) {
  const int lane = tid & 63, wave = tid >> 6;
  // staging: thread t loads A row (t >> 2), k offsets 8 (t & 3) .. + 7 and B row (t >> 3),
  // columns 16 (t & 7) .. + 15; rows past nq / d and columns past nlist read as 0 / clamped
  const int ar = tid >> 2, ak = (tid & 3) * 8;
  const int br = tid >> 3, bc = (tid & 7) * 16;
  const float* xrow = x + min<int64_t>(q0 + ar, nq - 1) * d;
  const bool arow_ok = q0 + ar < nq;
  // columns past the padded width: clamped per float4 (never written out)
  const int bc0 = min(c0 + bc, ldc - 4), bc1 = min(c0 + bc + 4, ldc - 4), bc2 = min(c0 + bc + 8, ldc - 4),
            bc3 = min(c0 + bc + 12, ldc - 4);
  float4 ra0, ra1, rb0, rb1, rb2, rb3;
#define TILE_LOAD(k0)                                                                                   \
  {                                                                                                     \
    const int kk_ = (k0) + ak;                                                                          \
    const float4 z_ = make_float4(0.f, 0.f, 0.f, 0.f);                                                  \
    ra0 = (arow_ok && kk_ < d) ? *reinterpret_cast<const float4*>(xrow + kk_) : z_;                     \
    ra1 = (arow_ok && kk_ + 4 < d) ? *reinterpret_cast<const float4*>(xrow + kk_ + 4) : z_;             \
    const float* bp_ = centT + (int64_t)min((k0) + br, d - 1) * ldc;                                    \
    rb0 = *reinterpret_cast<const float4*>(bp_ + bc0);                                                  \
    rb1 = *reinterpret_cast<const float4*>(bp_ + bc1);                                                  \
    rb2 = *reinterpret_cast<const float4*>(bp_ + bc2);                                                  \
    rb3 = *reinterpret_cast<const float4*>(bp_ + bc3);                                                  \
  }
#define TILE_STORE(b)                                                                                   \
  {                                                                                                     \
    float2* ap_ = reinterpret_cast<float2*>(&As[b][ar * TAS + ak]);                                     \
    ap_[0] = make_float2(ra0.x, ra0.y);                                                                 \
    ap_[1] = make_float2(ra0.z, ra0.w);                                                                 \
    ap_[2] = make_float2(ra1.x, ra1.y);                                                                 \
    ap_[3] = make_float2(ra1.z, ra1.w);                                                                 \
    float4* bq_ = reinterpret_cast<float4*>(&Bs[b][br * TBS + bc]);                                     \
    bq_[0] = rb0;                                                                                       \
    bq_[1] = rb1;                                                                                       \
    bq_[2] = rb2;                                                                                       \
    bq_[3] = rb3;                                                                                       \
  }
#pragma unroll
  for (int t = 0; t < TC / 16; t++) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
  const int i16 = lane & 15, k4 = lane >> 4;
  const int nk = (d + TKC - 1) / TKC;
  TILE_LOAD(0);
  TILE_STORE(0);
  __syncthreads();
  for (int kc = 0; kc < nk; kc++) {
    const int b = kc & 1;
    if (kc + 1 < nk) TILE_LOAD((kc + 1) * TKC);  // in flight during this chunk's MFMAs
    const float* A = &As[b][(wave * 16 + i16) * TAS];
    const float* B = &Bs[b][0];
#pragma unroll
    for (int j = 0; j < TKC / 4; j++) {
      const int kk = 4 * j + k4;
      const float av = A[kk];
#pragma unroll
      for (int t = 0; t < TC / 16; t++)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, B[kk * TBS + t * 16 + i16], acc[t], 0, 0, 0);
    }
    if (kc + 1 < nk) TILE_STORE(b ^ 1);
    __syncthreads();
  }
#undef TILE_LOAD
#undef TILE_STORE
}

__global__ __launch_bounds__(256) void k_coarse_gemm_tiled(const float* __restrict__ x, const float* __restrict__ xn,
                                                           int64_t nq, int d, const float* __restrict__ centT,
                                                           int ldc, const float* __restrict__ cn, int nlist,
                                                           float* __restrict__ keys, int ip, int ngemm, CoarseT3 t3) {
  __shared__ __attribute__((aligned(16))) float As[2][TQ * TAS];
  __shared__ __attribute__((aligned(16))) float Bs[2][TKC * TBS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if ((int)blockIdx.x >= ngemm) {
    t3_role(x, nq, d, t3, blockIdx.x - ngemm, &As[0][0], tid);
    return;
  }
  const int nct = (nlist + TC - 1) / TC;
  const int64_t q0 = (int64_t)(blockIdx.x / nct) * TQ;
  const int c0 = (blockIdx.x % nct) * TC;
  f4 acc[TC / 16];
  tiled_key_acc(acc, x, q0, nq, d, centT, ldc, c0, As, Bs, tid);
  const int i16 = lane & 15, k4 = lane >> 4;
  // the norms are loaded unconditionally (clamped) before any store: as loads under the
  // bounds branches they were issued one round trip at a time
  float cnv[TC / 16], xnv[4];
#pragma unroll
  for (int t = 0; t < TC / 16; t++) cnv[t] = ip ? 0.f : cn[min(c0 + t * 16 + i16, nlist - 1)];
#pragma unroll
  for (int r = 0; r < 4; r++) xnv[r] = ip ? 0.f : xn[min(q0 + wave * 16 + k4 * 4 + r, nq - 1)];
#pragma unroll
  for (int t = 0; t < TC / 16; t++) {
    const int c = c0 + t * 16 + i16;
    if (c >= nlist) continue;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int64_t q = q0 + wave * 16 + k4 * 4 + r;
      if (q >= nq) continue;
      keys[q * nlist + c] = coarse_key(acc[t][r], xnv[r], cnv[t], ip);
    }
  }
}

// Write a query's top-nprobe (run: packed (key, list), ascending across the
// wave) and, with cp.on, plan its probes for the list-major scan.
// -<x_q, c_{l(p)}> in Faiss tree order (tree<K_IP> over d) for the probes p < np of one
// query, probe p's list given by lane p's `l` (l < 0: not needed, any value returned):
// eight lanes per probe, lane j of a group holding the tree's accumulator j (as
// k_row_norms), so a 768-d product is 96 dependent steps per lane instead of 768 in
// one.  Must be called by the whole wave; the result is returned in lane p.
__device__ __forceinline__ float wave_ip_dis0(const float* __restrict__ xq, const float* __restrict__ cent, int64_t l,
                                             int d, int np, int lane) {
  const int j = lane & 7;
  const int d8 = d & ~7;
  float res = 0.f;
  for (int pass = 0; pass * 8 < np; pass++) {  // wave-uniform
    const int pp = pass * 8 + (lane >> 3);
    const int64_t lp = (int64_t)(((uint64_t)(uint32_t)__shfl((int)((uint64_t)l >> 32), pp & 63) << 32) |
                                 (uint32_t)__shfl((int)(uint32_t)(uint64_t)l, pp & 63));
    const bool ok = pp < np && lp >= 0;
    const float* cl = cent + (ok ? lp : 0) * d;
    float a = 0.f;
    if (ok) {
      int t = j;
      for (; t + 56 < d8; t += 64) {  // eight loads of each operand in flight, adds in element order
        float xv[8], cv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
          xv[u] = xq[t + 8 * u];
          cv[u] = cl[t + 8 * u];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) a = a + xv[u] * cv[u];
      }
      for (; t < d8; t += 8) a = a + xq[t] * cl[t];
    }
    float a4 = __shfl_down(a, 4, 8) + a;  // a8[j + 4] + a8[j]
    int r = d8;
    if (r + 4 <= d) {
      if (ok && j < 4) a4 = a4 + xq[r + j] * cl[r + j];
      r += 4;
    }
    if (ok && j < 4 && r + j < d) a4 = a4 + xq[r + j] * cl[r + j];
    const float h = a4 + __shfl_down(a4, 1, 8);
    const float v = h + __shfl_down(h, 2, 8);  // lane 8 g: probe pass * 8 + g
    const float mine = __shfl(v, (lane & 7) * 8);
    if ((lane >> 3) == pass) res = mine;
  }
  return -res;
}

// (IP a template parameter: the L2 instantiation carries no inner-product dis0 code --
// these one-shot kernels' time is largely instruction fetch)
template <int IP>
__device__ __forceinline__ void coarse_emit(uint64_t run, int64_t q, int lane, int nprobe, float* __restrict__ out_dis,
                                            int64_t* __restrict__ out_list, const float* __restrict__ x, int d,
                                            const CoarsePlan& cp) {
  constexpr int ip = IP;
  const bool empty = run == kKcNone;
  const float rd = kc_key(run);
  const int64_t ri = empty ? kSentinelId : (int64_t)(uint32_t)run;
  if (lane < nprobe) {
    out_dis[q * nprobe + lane] = empty ? (ip ? -FLT_MAX : FLT_MAX) : (ip ? -rd : rd);
    out_list[q * nprobe + lane] = empty ? -1 : ri;
  }
  if (cp.on) {  // list-major planning of this query's probes (k_plan_count's rules)
    const int64_t l = ri;  // kSentinelId when empty: outside [lo, hi)
    const bool use = lane < nprobe && l >= cp.lo && l < cp.hi && cp.list_off[l + 1] > cp.list_off[l];
    const uint64_t um = __ballot(use);
    const int fp = um ? (int)__builtin_ctzll(um) : 64;
    if (lane == 0) cp.pl.qmask[q * cp.pl.qmw] = um;  // the probes the scan covers (read by the merge)
    float d0 = rd;
    if (ip && um) d0 = wave_ip_dis0(x + q * d, cp.cent, use ? l : -1, d, nprobe, lane);  // (wave-uniform)
    if (use) plan_pair(cp.pl, cp.hi - cp.lo, l, cp.lo, lane == fp ? 0 : 1, (int)(q * nprobe + lane), d0);
  }
}

// Per query (one wave): the nprobe (<= 64) smallest keys of its row, by
// (key, list); per block of 1024 lists the candidates are cut by the
// nprobe-th smallest of the 64 lane minima (those minima are nprobe distinct
// keys, so every member of the block's top-nprobe is at or below it), sorted
// once and merged into the running list.  With `cp.on`, the epilogue plans
// the batch (first usable probe, per-list pair counts, bucket entries with the
// bucket entries with the scan's dis0).
// The nprobe (<= 64) smallest (key, list) words of one query's key row (global
// or LDS), ascending across the wave (packed, kKcNone = none); scratch: 64 words
// of LDS for this wave.
__device__ __forceinline__ uint64_t coarse_select_row(const float* row, int nlist, int nprobe, uint64_t* scratch,
                                                      int lane) {
  const uint64_t lt = (1ull << lane) - 1;
  uint64_t run = kKcNone;
  for (int base = 0; base < nlist; base += 1024) {
    float v[16];
    float m = kInf;
#pragma unroll
    for (int u = 0; u < 16; u++) {
      const int c = base + u * 64 + lane;
      v[u] = c < nlist ? row[c] : kInf;
      m = fminf(m, v[u]);
    }
    const float T = wave_kth_smallest(m, nprobe, lane);
    int total = 0;
#pragma unroll
    for (int u = 0; u < 16; u++) {
      const int c = base + u * 64 + lane;
      const bool pass = c < nlist && v[u] <= T;
      const uint64_t mk = __builtin_amdgcn_ballot_w64(pass);
      const int pos = total + __popcll(mk & lt);
      if (pass && pos < 64) scratch[pos] = pack_kc(v[u], c);
      total += __popcll(mk);
    }
    uint64_t p;
    if (total <= 64) {
      __builtin_amdgcn_wave_barrier();
      p = lane < total ? scratch[lane] : kKcNone;
      kc_sort64(p, lane);
      kc_merge64(run, p, lane);
    } else {  // many ties at the cut (rare): every 64-key slice of the block (a loop: compact code)
#pragma unroll 1
      for (int u = 0; u < 16; u++) {
        const int c = base + u * 64 + lane;
        p = c < nlist ? pack_kc(row[c], c) : kKcNone;
        kc_sort64(p, lane);
        kc_merge64(run, p, lane);
      }
    }
    __builtin_amdgcn_wave_barrier();  // scratch reuse
  }
  return run;
}

template <int IP>
__global__ __launch_bounds__(256) void k_coarse_select(const float* __restrict__ keys, int64_t nq, int nlist,
                                                       int nprobe, float* __restrict__ out_dis,
                                                       int64_t* __restrict__ out_list,
                                                       const float* __restrict__ x, int d, CoarsePlan cp) {
  __shared__ uint64_t scratch[4][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t q = (int64_t)blockIdx.x * 4 + wave;
  if (q >= nq) return;  // wave-uniform
  SDIAG(0);
  const uint64_t run = coarse_select_row(keys + q * nlist, nlist, nprobe, scratch[wave], lane);
  SDIAG(3);
  coarse_emit<IP>(run, q, lane, nprobe, out_dis, out_list, x, d, cp);
  SDIAG(5);
}

// ------------------------------------------------------ linear pre-transform
// y[i][j] = sum_t x[i][t] * A[j][t] (+ b[j]), the OPQ / LinearTransform apply
// (Faiss VectorTransform::apply, bench_gpu_1bn.py:485-489): a t-ordered fmaf
// chain from 0 (the oracle's or_linear_transform order), bias added last.
// AT = A transposed [d_in][d_out]: the threads of a row read it coalesced.
__global__ __launch_bounds__(256) void k_linear_transform(const float* __restrict__ x, int64_t n, int d_in,
                                                          const float* __restrict__ AT, const float* __restrict__ b,
                                                          int d_out, float* __restrict__ y) {
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= n * d_out) return;
  const int64_t i = gid / d_out;
  const int j = (int)(gid - i * d_out);
  const float* xi = x + i * d_in;
  float acc = 0.f;
  for (int t = 0; t < d_in; t++) acc = __builtin_fmaf(xi[t], AT[(int64_t)t * d_out + j], acc);
  y[gid] = b ? acc + b[j] : acc;
}

// -------------------------------------------------------------- PQ tables
// T3, one workgroup per query: thread t computes entries [16t, 16t+16) of the
// query's M x 256 table (m = t / 16); q is staged in LDS, codebook rows are
// contiguous.  DSUB = 0 is the generic (runtime dsub) variant.
template <int DSUB>
__global__ __launch_bounds__(256) void k_ip_table(const float* __restrict__ x, int64_t n, int d,
                                                  const float* __restrict__ cb, int M, int ksub,
                                                  float* __restrict__ out) {
  __shared__ float xs[2048];
  const int64_t q = blockIdx.x;
  const int tid = threadIdx.x;
  for (int e = tid; e < d; e += 256) xs[e] = x[q * d + e];
  __syncthreads();
  const int dsub = DSUB ? DSUB : d / M;
  const int total = M * ksub;
  if constexpr (DSUB > 0) {
    // 4 entries per round trip: all codebook loads first, then the trees
    constexpr int EB = 4;
    for (int e0 = tid; e0 < total; e0 += 256 * EB) {
      float cw[EB][DSUB];
#pragma unroll
      for (int b = 0; b < EB; b++) {
        const int e = min(e0 + b * 256, total - 1);
        const float* src = cb + (int64_t)e * DSUB;  // [M][ksub][dsub] == entry-major
#pragma unroll
        for (int t = 0; t < DSUB; t++) cw[b][t] = src[t];
      }
#pragma unroll
      for (int b = 0; b < EB; b++) {
        const int e = e0 + b * 256;
        if (e < total) {
          const float* xq = xs + (e / ksub) * DSUB;
          out[q * total + e] = tree<K_IP>([&](int t) { return xq[t]; }, [&](int t) { return cw[b][t]; }, DSUB);
        }
      }
    }
  } else {
    for (int e = tid; e < total; e += 256) {
      const int m = e / ksub;
      const float* xq = xs + m * dsub;
      const float* cwp = cb + (int64_t)e * dsub;
      out[q * total + e] = tree<K_IP>([&](int t) { return xq[t]; }, [&](int t) { return cwp[t]; }, dsub);
    }
  }
}

// T3 by (16 queries, sub-quantizer m) tiles: thread t holds codeword (m, t) in
// registers (read once per 16 queries instead of once per query: C3's codebook is
// 786 KB, which k_ip_table read from L2 for every query) and writes entry
// (q, m, t) for the 16 queries, coalesced over t.  Same tree order as k_ip_table.
template <int DSUB>
__global__ __launch_bounds__(256) void k_ip_tiles(const float* __restrict__ x, int64_t n, int d,
                                                  const float* __restrict__ cb, int M, float* __restrict__ out) {
  __shared__ float xs[GQ * DSUB];
  const int tid = threadIdx.x;
  const int64_t q0 = (int64_t)(blockIdx.x / M) * GQ;
  const int m = blockIdx.x % M;
  for (int i = tid; i < GQ * DSUB; i += 256) {
    const int qq = i / DSUB;
    xs[i] = q0 + qq < n ? x[(q0 + qq) * d + m * DSUB + (i - qq * DSUB)] : 0.f;
  }
  float cw[DSUB];
  const float* src = cb + ((int64_t)m * 256 + tid) * DSUB;
#pragma unroll
  for (int t = 0; t < DSUB; t++) cw[t] = src[t];
  __syncthreads();
  const int total = M * 256;
  const int nqq = (int)min<int64_t>(GQ, n - q0);
#pragma unroll 4
  for (int qq = 0; qq < nqq; qq++) {
    const float* xq = xs + qq * DSUB;
    out[(q0 + qq) * total + m * 256 + tid] =
        tree<K_IP>([&](int t) { return xq[t]; }, [&](int t) { return cw[t]; }, DSUB);
  }
}

__global__ __launch_bounds__(256) void k_precompute_T1(const float* __restrict__ cent, int nlist, int d,
                                                       const float* __restrict__ cb, int M, int ksub,
                                                       float* __restrict__ T1) {
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (int64_t)nlist * M * ksub) return;
  const int j = (int)(gid % ksub);
  const int64_t t = gid / ksub;
  const int m = (int)(t % M);
  const int64_t l = t / M;
  const int dsub = d / M;
  const float* cw = cb + ((int64_t)m * ksub + j) * dsub;
  const float* cl = cent + l * d + m * dsub;
  const float rn = tree<K_NORM>([&](int u) { return cw[u]; }, [&](int u) { return cw[u]; }, dsub);
  const float ip = tree<K_IP>([&](int u) { return cl[u]; }, [&](int u) { return cw[u]; }, dsub);
  T1[gid] = rn + 2.0f * ip;
}

// ---------------------------------------------------------------- encode
__global__ __launch_bounds__(256) void k_pq_encode(const float* __restrict__ x, int64_t n, int d,
                                                   const float* __restrict__ cent,
                                                   const int64_t* __restrict__ list_no,
                                                   const float* __restrict__ cb, int M, int ksub,
                                                   uint8_t* __restrict__ codes) {
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= n * M) return;
  const int m = (int)(gid % M);
  const int64_t i = gid / M;
  const int dsub = d / M;
  const float* xi = x + i * d + m * dsub;
  const float* ci = cent + list_no[i] * d + m * dsub;
  int best = 0;
  float bd = 0.f;
  for (int j = 0; j < ksub; j++) {
    const float* cw = cb + ((int64_t)m * ksub + j) * dsub;
    const float dd = tree<K_L2>([&](int u) { return xi[u] - ci[u]; }, [&](int u) { return cw[u]; }, dsub);
    if (j == 0 || dd < bd) {
      bd = dd;
      best = j;
    }
  }
  codes[gid] = (uint8_t)best;
}

// ===================================================== list-major planning
// One wave per query: tau reset, first usable probe, per-list pair counts and
// bucket entries (the fused coarse epilogue does the same for its batch).
// dedup (caller-supplied rows): a list repeated in a query's row is scanned
// once, at its first position (the later pairs are left out of the probe mask).
__global__ __launch_bounds__(256) void k_plan_count(const int64_t* __restrict__ lists, const float* __restrict__ Dq,
                                                    const float* __restrict__ x, const float* __restrict__ cent,
                                                    int64_t nq, int d, int nprobe,
                                                    const int64_t* __restrict__ list_off, int lo, int hi, int ip,
                                                    int dedup, int k, ListPlan pl) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nq) return;
  bool found = false;
  for (int p0 = 0; p0 < nprobe; p0 += 64) {
    const int p = p0 + lane;
    const int64_t l = p < nprobe ? lists[q * nprobe + p] : -1;
    // (L2) dis0 loaded with the probe, not after the range and duplicate checks
    const float dq = (!ip && Dq && p < nprobe) ? Dq[q * nprobe + p] : 0.f;
    bool use = p < nprobe && l >= lo && l < hi && list_off[l + 1] > list_off[l];
    if (dedup) {
      // an earlier probe with the same list: the earlier ones of this 64-probe
      // block by readlane (lanes below this one), those of earlier blocks from memory
      bool dup = false;
      for (int j = 0; j < 64 && p0 + j < nprobe; j++) {
        const int64_t lj = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)((uint64_t)l >> 32), j) << 32) |
                                     (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)l, j));
        dup = dup || (j < lane && lj == l);
      }
      for (int j = 0; j < p0 && use && !dup; j++) dup = lists[q * nprobe + j] == l;
      use = use && !dup;  // (its bit stays clear in qmask: the merge skips the pair)
    }
    const uint64_t um = __ballot(use);
    const int fp = (!found && um) ? (int)__builtin_ctzll(um) : 64;
    found = found || um != 0;
    if (lane == 0) pl.qmask[q * pl.qmw + (p0 >> 6)] = um;  // the pairs the scan covers (read by the merges)
    float d0 = 0.f;
    if (ip && um) d0 = wave_ip_dis0(x + q * d, cent, use ? l : -1, d, min(64, nprobe - p0), lane);  // (uniform)
    if (use) {
      if (!ip) d0 = dq;
      plan_pair(pl, hi - lo, l, lo, lane == fp ? 0 : 1, (int)(q * nprobe + p), d0);
    }
  }
}

// Work items from the per-list counts.  Items of kind 0 occupy [0, N0), kind 1
// [N0, N0 + N1), each in list order.  Small shard ranges (nloc <=
// kPlanSmall): every workgroup builds the whole per-list item prefix in LDS
// and writes the records of its 1024 items, one per thread (the grid covers
// the item-count bound).  Large ranges: every workgroup takes 1024 lists,
// derives the items before them by a reduction over the counts, and writes its
// lists' items.
constexpr int PLAN_T = 1024;
constexpr int kPlanSmall = 4096;

__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(v, off, 64);
    if (lane >= off) v += o;
  }
  return v;
}

// exclusive scan of (a, b) over the 1024 threads of the block; returns the block totals
__device__ __forceinline__ void block_scan2(int a, int b, int& ea, int& eb, int& ta, int& tb, int* ws /* [2][16] */) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ia = wave_incl_scan(a, lane), ib = wave_incl_scan(b, lane);
  __syncthreads();  // ws may still be read by a previous call
  if (lane == 63) {
    ws[wave] = ia;
    ws[16 + wave] = ib;
  }
  __syncthreads();
  int pa = 0, pb = 0;
  ta = 0;
  tb = 0;
  for (int w = 0; w < PLAN_T / 64; w++) {
    const int va = ws[w], vb = ws[16 + w];
    if (w < wave) {
      pa += va;
      pb += vb;
    }
    ta += va;
    tb += vb;
  }
  ea = pa + ia - a;
  eb = pb + ib - b;
}

__device__ __forceinline__ void write_item(const ListPlan& pl, const int64_t* __restrict__ list_off, int lo, int nloc,
                                           int G, int rec, int jj, int kind, int t) {
  const int c = min(pl.cnt[kind * nloc + jj], pl.cap);
  const int cnt = min(G, c - t * G);
  const int64_t l = lo + jj;
  const int64_t beg = list_off[l];
  int r[16];
  r[0] = (int)l;
  r[1] = cnt;
  r[2] = (int)(list_off[l + 1] - beg);
  r[3] = (int)(uint32_t)(uint64_t)beg;
  r[4] = (int)(uint32_t)((uint64_t)beg >> 32);
#pragma unroll
  for (int g = 0; g < 4; g++) {
    int2 v = make_int2(0, 0);
    if (g < cnt) v = pl.bucket[((int64_t)jj * 2 + kind) * pl.cap + t * G + g];
    r[5 + g] = v.x;
    r[9 + g] = v.y;
  }
  r[13] = kind;
  r[14] = 0;
  r[15] = 0;
  int4* rp = reinterpret_cast<int4*>(pl.recs + (int64_t)rec * 16);
  rp[0] = make_int4(r[0], r[1], r[2], r[3]);
  rp[1] = make_int4(r[4], r[5], r[6], r[7]);
  rp[2] = make_int4(r[8], r[9], r[10], r[11]);
  rp[3] = make_int4(r[12], r[13], r[14], r[15]);
}


__global__ __launch_bounds__(PLAN_T) void k_plan_items_small(ListPlan pl, const int64_t* __restrict__ list_off, int lo,
                                                             int nloc, int G) {
  __shared__ int ex[2][kPlanSmall + 1];
  __shared__ int ws[32];
  const int tid = threadIdx.x;
  // per-list exclusive prefix of the item counts, both kinds, in chunks of 1024 lists
  int ca = 0, cb = 0;
  const int32_t* ord = pl.order;
  for (int j0 = 0; j0 < nloc; j0 += PLAN_T) {
    const int j = j0 + tid;  // rank in the scheduling order
    const int jl = j < nloc ? (ord ? ord[j] : j) : 0;
    const int a = j < nloc ? (min(pl.cnt[jl], pl.cap) + G - 1) / G : 0;
    const int b = j < nloc ? (min(pl.cnt[nloc + jl], pl.cap) + G - 1) / G : 0;
    int ea, eb, ta, tb;
    block_scan2(a, b, ea, eb, ta, tb, ws);
    if (j < nloc) {
      ex[0][j] = ca + ea;
      ex[1][j] = cb + eb;
    }
    ca += ta;
    cb += tb;
  }
  if (tid == 0) {
    ex[0][nloc] = ca;
    ex[1][nloc] = cb;
  }
  const int T0 = ca, N = ca + cb;
  if (blockIdx.x == 0 && tid < 2) pl.hdr[tid] = tid == 0 ? N : T0;  // (hdr[2..] belong to the scan and merges)
  __syncthreads();
  const int e = blockIdx.x * PLAN_T + tid;
  if (e >= N) return;
  const int kind = e < T0 ? 0 : 1;
  const int ek = kind ? e - T0 : e;
  const int* exk = ex[kind];
  int lo_i = 0, hi_i = nloc;  // largest j with exk[j] <= ek
  while (hi_i - lo_i > 1) {
    const int mid = (lo_i + hi_i) >> 1;
    if (exk[mid] <= ek)
      lo_i = mid;
    else
      hi_i = mid;
  }
  write_item(pl, list_off, lo, nloc, G, e, ord ? ord[lo_i] : lo_i, kind, ek - exk[lo_i]);
}

__global__ __launch_bounds__(PLAN_T) void k_plan_items_big(ListPlan pl, const int64_t* __restrict__ list_off, int lo,
                                                           int nloc, int G) {
  __shared__ int ex0[PLAN_T + 1], ex1[PLAN_T + 1];
  __shared__ int ws[32];
  const int tid = threadIdx.x;
  const int my0 = blockIdx.x * PLAN_T;
  int t0 = 0, t1 = 0, p0 = 0, p1 = 0;
  for (int j = tid; j < nloc; j += PLAN_T) {
    const int a = (min(pl.cnt[j], pl.cap) + G - 1) / G, b = (min(pl.cnt[nloc + j], pl.cap) + G - 1) / G;
    t0 += a;
    t1 += b;
    if (j < my0) {
      p0 += a;
      p1 += b;
    }
  }
  int ea, eb, T0, T1, P0, P1;
  block_scan2(t0, t1, ea, eb, T0, T1, ws);
  block_scan2(p0, p1, ea, eb, P0, P1, ws);
  const int j = my0 + tid;
  const int a = j < nloc ? (min(pl.cnt[j], pl.cap) + G - 1) / G : 0;
  const int b = j < nloc ? (min(pl.cnt[nloc + j], pl.cap) + G - 1) / G : 0;
  int sa, sb;
  block_scan2(a, b, ea, eb, sa, sb, ws);
  ex0[tid] = ea;
  ex1[tid] = eb;
  if (tid == 0) {
    ex0[PLAN_T] = sa;
    ex1[PLAN_T] = sb;
  }
  if (blockIdx.x == 0 && tid < 2) pl.hdr[tid] = tid == 0 ? T0 + T1 : T0;
  __syncthreads();
  const int own0 = ex0[PLAN_T], own1 = ex1[PLAN_T];
  for (int e = tid; e < own0 + own1; e += PLAN_T) {
    const int kind = e < own0 ? 0 : 1;
    const int ek = kind ? e - own0 : e;
    const int* exk = kind ? ex1 : ex0;
    int lo_i = 0, hi_i = PLAN_T;  // largest jl with exk[jl] <= ek
    while (hi_i - lo_i > 1) {
      const int mid = (lo_i + hi_i) >> 1;
      if (exk[mid] <= ek)
        lo_i = mid;
      else
        hi_i = mid;
    }
    write_item(pl, list_off, lo, nloc, G, kind ? T0 + P1 + ek : P0 + ek, my0 + lo_i, kind, ek - exk[lo_i]);
  }
}

__device__ __forceinline__ uint32_t ukey_of(float v) {
  return (uint32_t)f2ord(v + 0.0f) ^ 0x80000000u;  // unsigned order == float order (-0 folded)
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// the kk-th smallest (1-based) of the wave's NV x 64 values (0xFFFFFFFF = absent);
// requires kk <= the number of present values
template <int NV>
__device__ __forceinline__ uint32_t wave_kth_u32(const uint32_t (&u)[NV], int kk) {
  uint32_t lo = 0, hi = 0xFFFFFFFEu;
  while (lo < hi) {
    const uint32_t mid = lo + ((hi - lo) >> 1);
    int cnt = 0;
#pragma unroll
    for (int t = 0; t < NV; t++) cnt += __popcll(__builtin_amdgcn_ballot_w64(u[t] <= mid));
    if (cnt >= kk) hi = mid; else lo = mid + 1;
  }
  return lo;
}

// ===================================================== list scan (phase B)
// The scan's per-wave running top-k on packed (key, position) words
// (pack_kc: unsigned 64-bit order == (key asc, position asc)): one 64-bit
// compare and two selects per network step instead of float + id compares.
template <int R>
struct PackedTopK {
  uint64_t p[R];  // sorted ascending across R rows x 64 lanes
  uint64_t tp;    // the k-th best word (admission threshold), wave-uniform
  int krow, klane;

  __device__ __forceinline__ void init(int k) {
#pragma unroll
    for (int r = 0; r < R; r++) p[r] = kKcNone;
    tp = kKcNone;
    krow = (k - 1) >> 6;
    klane = (k - 1) & 63;
  }
  __device__ __forceinline__ float td() const { return tp == kKcNone ? kInf : kc_key(tp); }
  __device__ __forceinline__ void refresh_tau() {
#pragma unroll
    for (int r = 0; r < R; r++)
      if (r == krow) tp = readlane_u64(p[r], klane);
  }
  // insert the candidate words c of the lanes set in `mask` (wave-uniform)
  __device__ __forceinline__ void insert(uint64_t mask, uint64_t c, int lane) {
    while (mask) {
      const int src = __builtin_ctzll(mask);
      mask &= mask - 1;
      const uint64_t v = readlane_u64(c, src);
      if (!(v < tp)) continue;  // overtaken by an earlier insert
      int pos = 0;
#pragma unroll
      for (int r = 0; r < R; r++) pos += __popcll(__builtin_amdgcn_ballot_w64(p[r] < v));
#pragma unroll
      for (int r = R - 1; r >= 0; r--) {
        if ((r + 1) * 64 <= pos) continue;  // row entirely before the slot
        const uint64_t carry = r > 0 ? readlane_u64(p[r - 1], 63) : v;
        const uint64_t u = shr1_u64(carry, p[r]);
        const int idx = r * 64 + lane;
        p[r] = idx > pos ? u : (idx == pos ? v : p[r]);
      }
      refresh_tau();
    }
  }
};
// merge up to 64 candidate words (one per lane, kKcNone = none) into a one-row top-k
template <int R>
__device__ __forceinline__ void kc_bulk_merge_rows(PackedTopK<R>& tk, uint64_t c, int lane) {
  kc_sort64(c, lane);
#pragma unroll
  for (int r = 0; r < R; r++) {
    const uint64_t rv = ((uint64_t)(uint32_t)rev64_i((int)(uint32_t)(c >> 32)) << 32) | (uint32_t)rev64_i((int)(uint32_t)c);
    const bool t = rv < tk.p[r];
    const uint64_t lo = t ? rv : tk.p[r], hi = t ? tk.p[r] : rv;
    tk.p[r] = lo;
    kc_steps<128, 32>(tk.p[r], lane);
    if (r + 1 < R) {
      c = hi;
      kc_steps<128, 32>(c, lane);
      // c is ascending: when its smallest word is empty, so is every carry and
      // the later rows keep their contents (a k = 1000 list holding a few hundred
      // entries merges into its first rows only)
      if (readlane_u64(c, 0) == kKcNone) break;
    }
  }
  tk.refresh_tau();
}
__device__ __forceinline__ void kc_bulk_merge(PackedTopK<1>& tk, uint64_t c, int lane) {
  kc_sort64(c, lane);
  kc_merge64(tk.p[0], c, lane);
  tk.refresh_tau();
}
// up to 16 candidate words in lanes 0..15 into a one-row top-k with k <= 16:
// 16-lane sort (DPP only), reverse-min against lanes 0..15, 16-lane merge
__device__ __forceinline__ void kc_row16_merge(PackedTopK<1>& tk, uint64_t c, int lane) {
  kc_steps<2, 1>(c, lane);
  kc_steps<4, 2>(c, lane);
  kc_steps<8, 4>(c, lane);
  kc_steps<128, 8>(c, lane);  // every row ascending
  const uint64_t rv = ((uint64_t)(uint32_t)rev16_i((int)(uint32_t)(c >> 32)) << 32) | (uint32_t)rev16_i((int)(uint32_t)c);
  uint64_t q = rv < tk.p[0] ? rv : tk.p[0];
  kc_steps<128, 8>(q, lane);
  tk.p[0] = lane >= 16 ? kKcNone : q;
  tk.refresh_tau();
}


// inclusive prefix sum over the wave on the VALU: 16-lane row scans by DPP
// row shifts (zero fill), then the row totals added by readlane
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_shr_z(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v, int lane) {
  uint32_t s = v + dpp_shr_z<0x111>(v) + dpp_shr_z<0x112>(v) + dpp_shr_z<0x113>(v);  // row_shr:1..3
  s += dpp_shr_z<0x114>(s);                                                          // row_shr:4
  s += dpp_shr_z<0x118>(s);                                                          // row_shr:8
  const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)s, 15);
  const uint32_t t1 = (uint32_t)__builtin_amdgcn_readlane((int)s, 31);
  const uint32_t t2 = (uint32_t)__builtin_amdgcn_readlane((int)s, 47);
  const int row = lane >> 4;
  return s + (row == 0 ? 0u : row == 1 ? t0 : row == 2 ? t0 + t1 : t0 + t1 + t2);
}


template <int G>
struct LutVec;
template <>
struct LutVec<1> {
  using T = float;
};
template <>
struct LutVec<2> {
  using T = float2;
};
template <>
struct LutVec<4> {
  using T = float4;
};

__device__ __forceinline__ float comp(float v, int) { return v; }
__device__ __forceinline__ float comp(float2 v, int g) { return g == 0 ? v.x : v.y; }
__device__ __forceinline__ float comp(float4 v, int g) { return g == 0 ? v.x : g == 1 ? v.y : g == 2 ? v.z : v.w; }
__device__ __forceinline__ void setc(float& o, int, float x) { o = x; }
__device__ __forceinline__ void setc(float2& o, int g, float x) {
  if (g == 0) o.x = x; else o.y = x;
}
__device__ __forceinline__ void setc(float4& o, int g, float x) {
  if (g == 0) o.x = x; else if (g == 1) o.y = x; else if (g == 2) o.z = x; else o.w = x;
}

template <int M>
struct CodeWords {
  uint32_t w[M / 4];
  __device__ __forceinline__ void load(const uint8_t* p) {
    if constexpr (M % 16 == 0) {
#pragma unroll
      for (int v = 0; v < M / 16; v++) {
        const uint4 t = reinterpret_cast<const uint4*>(p)[v];
        w[4 * v + 0] = t.x;
        w[4 * v + 1] = t.y;
        w[4 * v + 2] = t.z;
        w[4 * v + 3] = t.w;
      }
    } else if constexpr (M % 8 == 0) {
#pragma unroll
      for (int v = 0; v < M / 8; v++) {
        const uint2 t = reinterpret_cast<const uint2*>(p)[v];
        w[2 * v + 0] = t.x;
        w[2 * v + 1] = t.y;
      }
    } else {
#pragma unroll
      for (int v = 0; v < M / 4; v++) w[v] = reinterpret_cast<const uint32_t*>(p)[v];
    }
  }
  __device__ __forceinline__ uint32_t byte(int m) const { return (w[m >> 2] >> ((m & 3) * 8)) & 0xffu; }
};

template <int G>
struct Item {
  int l, cnt, n, kind;
  int64_t beg;
  int pair[G];
  float d0[G];
  int q[G];  // query of pair g (pair / nprobe; absent pairs: the first pair's query)
};

// Persistent workgroups take work items from one counter: kind-0 items (each
// query's first probe) first, so that a query's running k-th key tau_q is
// usually known before its other probes are scanned.  A work item is (list l,
// up to G pairs): the G LUTs are interleaved per entry ([m][j][g]) so one
// ds_read_b{32,64,128} returns the G lookups of a code and the bank conflicts
// of the random 8-bit gathers are paid once per G lookups.
// Per item: the item's codes (up to JB chunks of 256 codes) are loaded together
// with the LUT rows -- one memory round trip -- and the next item index is
// fetched at the same time; then the codes are gathered one chunk (64 codes
// per wave) at a time.  Candidates (key <= min(own k-th, tau_q)) go to a
// per-wave LDS queue that one compact loop drains into the wave's per-query
// top-k, ranked by (key, position in the list): device lists are
// label-sorted, so this equals (key, label) inside a list.  While a query has
// no bound yet the queue is drained after every chunk.  tau_q is shared
// across workgroups through global atomicMin (any k real candidates bound the
// final k-th; a stale read is only a looser bound).
constexpr int QCAP = 256;  // per-wave candidate queue entries


// x / d for 0 <= x <= 2^24 by a float reciprocal (|error| <= 2 there) and a
// correction from the remainder (an integer division is a ~40-instruction
// sequence on the GPU)
__device__ __forceinline__ int div_small(int x, int d, float inv_d) {
  const int q = (int)((float)x * inv_d);
  const int r = x - q * d;
  return q + (r >= d) + (r >= 2 * d) - (r < 0) - (r < -d);
}

// ---- fused planning: the list scan derives its work items itself
// (pl.fused: nloc <= kFusedPlanLists and fewer than 65536 items).  Every
// workgroup forms the exclusive prefix of the per-list item counts
// ceil(min(cnt, cap) / G) of both kinds in scheduling order (pl.order) in LDS;
// item e of kind 0 ([0, N0)) or kind 1 ([N0, N)) is then found by a two-step
// search over that prefix, and its record words are loaded from the counts,
// list offsets and bucket in one round trip.  Replaces k_plan_items (one
// launch) for the shard sizes where it fits in LDS.
constexpr int kFusedPlanLists = 1024;

// returns (N0, N1); ws: >= 8 ints of scratch (LDS)
__device__ __forceinline__ int2 fused_plan_prefix(const ListPlan& pl, int nloc, int G, uint16_t* ex0, uint16_t* ex1,
                                                  uint16_t* ord, int* ws) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // thread t: ranks 4t .. 4t + 3 (nloc <= 1024)
  int a[4], b[4], sa = 0, sb = 0;
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int j = 4 * tid + u;
    const int jl = j < nloc ? (pl.order ? pl.order[j] : j) : 0;
    a[u] = j < nloc ? (min(pl.cnt[jl], pl.cap) + G - 1) / G : 0;
    b[u] = j < nloc ? (min(pl.cnt[nloc + jl], pl.cap) + G - 1) / G : 0;
    if (j < nloc) ord[j] = (uint16_t)jl;
    sa += a[u];
    sb += b[u];
  }
  const int ia = wave_incl_scan(sa, lane), ib = wave_incl_scan(sb, lane);
  if (lane == 63 && wave < 4) {  // (larger workgroups: waves past the first 4 hold no ranks)
    ws[wave] = ia;
    ws[4 + wave] = ib;
  }
  __syncthreads();
  int pa = 0, pb = 0, ta = 0, tb = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    if (w < wave) {
      pa += ws[w];
      pb += ws[4 + w];
    }
    ta += ws[w];
    tb += ws[4 + w];
  }
  pa += ia - sa;
  pb += ib - sb;
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int j = 4 * tid + u;
    if (j < nloc) {
      ex0[j] = (uint16_t)pa;
      ex1[j] = (uint16_t)pb;
    }
    pa += a[u];
    pb += b[u];
  }
  if (tid == 0) {
    ex0[nloc] = (uint16_t)ta;
    ex1[nloc] = (uint16_t)tb;
  }
  __syncthreads();
  return make_int2(ta, tb);
}

// Item e's record, fetched ahead: lane w (< 16) issues ONE unconditional load of
// record word w -- no divergent branches, so no register receives loads under
// different exec masks -- whose value nothing consumes until unpack (the load stays
// in flight during the current item's scan).  Fused planning: word 1 = the list's
// pair count (count = min(G, min(c, cap) - t G)), words 2 / 3 = the low words of
// off[l + 1] / off[l] (n = w2 - w3), word 4 = off[l]'s high word, words 5..8 / 9..12
// = the bucket's pair ids / dis0 bits; the list, kind and t are wave-uniform and
// kept in scalars (the other lanes load word 1 again).  Non-fused: the 16 words of
// pl.recs (write_item's layout).
struct Rec {
  int raw;  // this lane's loaded word (in flight)
  int l, kind, t;
};
__device__ __forceinline__ Rec fused_record(const ScanArgs& a, const ListPlan& pl, int nloc, int e, int n0,
                                           const uint16_t* ex0, const uint16_t* ex1, const uint16_t* ord, int G,
                                           int lane) {
  const int kind = e < n0 ? 0 : 1;
  const int ek = kind ? e - n0 : e;
  const uint16_t* ex = kind ? ex1 : ex0;
  // largest j with ex[j] <= ek: first over every 16th rank, then within 16 ranks
  const int c16 = (nloc + 15) >> 4;
  const uint64_t m1 = __builtin_amdgcn_ballot_w64(lane < c16 && (int)ex[16 * lane] <= ek);
  const int j0 = 16 * (63 - __builtin_clzll(m1));
  const uint64_t m2 = __builtin_amdgcn_ballot_w64(lane < 16 && j0 + lane < nloc && (int)ex[j0 + lane] <= ek);
  const int j = j0 + 63 - __builtin_clzll(m2);
  const int jl = __builtin_amdgcn_readfirstlane((int)ord[j]);
  const int t = ek - __builtin_amdgcn_readfirstlane((int)ex[j]);
  const int64_t l = a.list_lo + jl;
  const int* off32 = reinterpret_cast<const int*>(a.list_off);
  const int* bk32 = reinterpret_cast<const int*>(pl.bucket);
  const int w = lane & 15;
  const int64_t slot = ((int64_t)jl * 2 + kind) * pl.cap + min(t * G + ((w - 5) & 3), pl.cap - 1);
  const int* src = w == 2 ? off32 + 2 * (l + 1)
                 : w == 3 ? off32 + 2 * l
                 : w == 4 ? off32 + 2 * l + 1
                 : (w >= 5 && w <= 12) ? bk32 + 2 * slot + (w <= 8 ? 0 : 1)
                 : pl.cnt + kind * nloc + jl;  // word 1 (and the unused lanes)
  Rec r;
  r.raw = *src;
  r.l = (int)l;
  r.kind = kind;
  r.t = t;
  return r;
}

// A wave's sorted partial list of one pair into slot `slot` = pair * 4 + wave, as
// tagged records (part_rec): k <= 64 pads the list to k entries ((FLT_MAX, -1));
// k > 64 writes the valid entries and their count only ((n, tag) in partN).
// fault (test hook, ivfpq_set_fault_injection): slots with slot % fault == 1 are
// not written at all, as if the stores were lost -- the merges must detect them.
template <int R>
__device__ __forceinline__ void write_partial(const ListPlan& pl, const PackedTopK<R>& tk, int64_t slot, int k,
                                              int64_t beg, int lane) {
  if (pl.fault > 0 && slot % pl.fault == 1) return;  // (uniform; 0 in every real search)
  const uint32_t tag = part_tag(pl.epoch, slot) | xcc_tag();
  uint4* o = pl.part + slot * pl.ks;
  int n = 0;
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int ix = r * 64 + lane;
    const bool empty = tk.p[r] == kKcNone;
    if (ix < k && (R == 1 || !empty))
      o[ix] = part_rec(empty ? FLT_MAX : kc_key(tk.p[r]), tag, empty ? -1 : beg + (int64_t)(uint32_t)tk.p[r]);
    if constexpr (R >= 2) n += __popcll(__builtin_amdgcn_ballot_w64(ix < k && !empty));
  }
  if constexpr (R >= 2)
    if (lane == 0) pl.partN[slot] = make_uint2((uint32_t)n, tag);
}

// ROWK (k <= 16, G = 4, R = 1): the 4 pairs' running top-k share one 64-bit
// word per lane, pair g in the 16 lanes of row g, so one 16-lane merge network
// (DPP row operations) serves all 4 pairs at once and one store writes their
// partial lists.
template <int M, int G, int R, int JB, bool ROWK = false>
__global__ __launch_bounds__(256, 2) void k_scan_lists(ScanArgs a, ListPlan pl) {
  static_assert(!ROWK || (G == 4 && R == 1), "row-packed top-k: 4 pairs, k <= 16");
  using V = typename LutVec<G>::T;
  constexpr int LUTN = M * 256;
  constexpr int NV = LUTN / 4 / 256;  // float4 per thread per table
  __shared__ __attribute__((aligned(16))) V lut[LUTN];
  constexpr int QG = QCAP / G;  // queue entries per wave and pair
  static_assert(QG >= 64, "a chunk's candidates must fit an empty queue");
  __shared__ float qd[4][QCAP];    // [wave][g][QG]
  __shared__ int32_t qi[4][QCAP];  // positions in the list
  __shared__ int s_next;
  __shared__ int32_t s_wb[G];  // the item's per-query bounds found by its waves (ordered ints)
  // fused planning (pl.fused): the item prefix of every list in scheduling order
  __shared__ uint16_t s_ex[2][kFusedPlanLists + 1];
  __shared__ uint16_t s_ord[kFusedPlanLists];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int k = a.k;
  const int ip = a.ip;
  const int nloc = a.list_hi - a.list_lo;
  const uint64_t lanemask_lt = (1ull << lane) - 1;
  const float inv_np = 1.0f / (float)a.nprobe;
  int n_items, n_items0 = 0;
  if (pl.fused) {
    const int2 t = fused_plan_prefix(pl, nloc, G, s_ex[0], s_ex[1], s_ord, reinterpret_cast<int*>(qi));
    n_items0 = t.x;
    n_items = t.x + t.y;
  } else {
    n_items = pl.hdr[0];
  }

  // An item's 64-B record: lanes 0..15 load its 16 words (vector loads, kept in
  // flight while the previous item is scanned), unpacked with readlane.  Fused
  // planning derives the words from the LDS prefix, the counts and the buckets.
  Item<G> it;
  auto fetch_rec = [&](int idx) __attribute__((always_inline)) -> Rec {
    if (!pl.fused) {
      Rec r;
      r.raw = pl.recs[(int64_t)idx * 16 + (lane & 15)];
      r.l = r.kind = r.t = 0;  // (words 0, 13 of the raw record)
      return r;
    }
    return fused_record(a, pl, nloc, idx, n_items0, s_ex[0], s_ex[1], s_ord, G, lane);
  };
  auto unpack = [&](const Rec& rc) __attribute__((always_inline)) {
    const int rv = rc.raw;
    if (pl.fused) {  // raw words (fused_record)
      it.l = rc.l;
      it.kind = rc.kind;
      it.cnt = min(G, min(__builtin_amdgcn_readlane(rv, 1), pl.cap) - rc.t * G);
      it.n = __builtin_amdgcn_readlane(rv, 2) - __builtin_amdgcn_readlane(rv, 3);
    } else {
      it.l = __builtin_amdgcn_readlane(rv, 0);
      it.kind = __builtin_amdgcn_readlane(rv, 13);
      it.cnt = __builtin_amdgcn_readlane(rv, 1);
      it.n = __builtin_amdgcn_readlane(rv, 2);
    }
    it.beg = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane(rv, 4) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane(rv, 3));
#pragma unroll
    for (int g = 0; g < G; g++) {
      it.pair[g] = __builtin_amdgcn_readlane(rv, 5 + g);
      it.d0[g] = __int_as_float(__builtin_amdgcn_readlane(rv, 9 + g));
    }
    // the pairs' queries (pair / nprobe; absent pairs: the first pair's), once per item
    // a pair id outside the batch would address another batch's tables and
    // partial lists: counted in pl.err, and the item scans nothing
    bool bad = false;
#pragma unroll
    for (int g = 0; g < G; g++)
      bad = bad || (g < it.cnt && (unsigned)it.pair[g] >= (unsigned)(a.nq * a.nprobe));
    if (bad) {
      if (lane == 0) atomicAdd(pl.err, 1);
      it.cnt = 0;
#pragma unroll
      for (int g = 0; g < G; g++) it.pair[g] = 0;
    }
#pragma unroll
    for (int g = 0; g < G; g++) it.q[g] = div_small((g < it.cnt ? it.pair[g] : it.pair[0]), a.nprobe, inv_np);
  };

  if (tid == 0) {
    const int t = atomicAdd(pl.hdr + 2, 1);
    s_next = t < n_items ? t : -1;
  }
  __syncthreads();
  int cur = s_next;
  if (cur >= 0) unpack(fetch_rec(cur));
  int it_no = 0;
  (void)it_no;
  // The next item's first loads -- its queries' running k-th keys (a stale
  // value is only a looser bound) and the first group of LUT rows -- are
  // issued at the end of the previous item's scan, before its partial writes,
  // so that they arrive while those and the barrier run.  Later LUT row groups
  // (M > 16) are software-pipelined in the build; the codes are loaded at the
  // item start, in flight during the LUT stores.
  constexpr int U = NV < 4 ? NV : 4;
  constexpr int NG = NV / U;
  static_assert(NV % U == 0, "LUT rows per thread");
  int tq[G];
  CodeWords<M> cw[JB];
  float4 b1[2][U], b3[2][U][G];
  auto t3row = [&](int g) __attribute__((always_inline)) {
    return reinterpret_cast<const float4*>(a.T3 + (int64_t)it.q[g] * LUTN);
  };
  // IP has no T1: read (and ignore) a T3 row instead, so that every load is unconditional
  auto t1row = [&]() __attribute__((always_inline)) {
    return ip ? t3row(0) : reinterpret_cast<const float4*>(a.T1 + (int64_t)it.l * LUTN);
  };
  auto fetch = [&](int u, int buf) __attribute__((always_inline)) {
    const float4* T1l = t1row();
#pragma unroll
    for (int e = 0; e < U; e++) {
      const int v = (u * U + e) * 256 + tid;
      b1[buf][e] = T1l[v];
#pragma unroll
      for (int g = 0; g < G; g++) {
        b3[buf][e][g] = t3row(g)[v];
      }
    }
  };
  auto issue = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < G; g++) tq[g] = tau_get(pl, it.q[g]);
    fetch(0, 0);
  };
  // (with R > 1 the larger top-k state leaves no registers for that: issued at the item start)
  constexpr bool kEarly = false;  // measured: no gain at C2 (register pressure)
  if (kEarly && cur >= 0) issue();
  while (cur >= 0) {
    __syncthreads();  // (A) every wave is done with the LUT of the previous item, and has read s_next
    DIAG(0, __builtin_amdgcn_s_memtime());
    // the next item, consumed after the LUT build (tnext is left undefined in the
    // other lanes: no merge copy that would wait for the atomic right here)
    int tnext;
    if (tid == 0) tnext = atomicAdd(pl.hdr + 2, 1);
    if constexpr (!kEarly) issue();
    const int n = it.n;
    const uint8_t* lc = a.codes + it.beg * M;
    // the item's first JB x 256 codes: in flight during the LUT stores
#pragma unroll
    for (int j = 0; j < JB; j++) {
      const int i = j * 256 + wave * 64 + lane;
      cw[j].load(lc + (int64_t)(i < n ? i : 0) * M);  // clamped: branch-free loads
    }
    // LUT = T1 - 2 T3 (L2) or -T3 (IP), G interleaved
#pragma unroll
    for (int u = 0; u < NG; u++) {
      if (u + 1 < NG) fetch(u + 1, (u + 1) & 1);
      // group u + 1's row loads stay issued ahead of group u's LUT stores: without this
      // fence the compiler sank every row load next to its use, one round trip per
      // element (16 in series per item at M = 64)
      __asm__ volatile("" ::: "memory");
#pragma unroll
      for (int e = 0; e < U; e++) {
        const int v = (u * U + e) * 256 + tid;
#pragma unroll
        for (int c = 0; c < 4; c++) {
          V o;
#pragma unroll
          for (int g = 0; g < G; g++) {
            const float x3 = comp(b3[u & 1][e][g], c);
            // T1 + (-2) T3 as one fma: -2 T3 is exact, so this rounds once like the
            // oracle's add of the product; entries of absent pairs are never admitted
            const float lv = ip ? -x3 : __builtin_fmaf(x3, -2.0f, comp(b1[u & 1][e], c));
            setc(o, g, lv);
          }
          lut[4 * v + c] = o;
        }
      }
    }
    if (tid == 0) s_next = tnext < n_items ? tnext : -1;
    if (tid < G) s_wb[tid] = f2ord(kInf);
    __syncthreads();  // (B) the LUT, s_next and s_wb are visible
    DIAG(1, __builtin_amdgcn_s_memtime());
    const int nxt = s_next;
    const Rec nrec = fetch_rec(nxt >= 0 ? nxt : cur);  // the next record, in flight during the scan
    int qix[G];  // the pairs' queries
    float bound[G];
    bool loose = false;  // some query of the item has no bound yet
#pragma unroll
    for (int g = 0; g < G; g++) {
      qix[g] = it.q[g];
      bound[g] = g < it.cnt ? ord2f(tq[g]) : -kInf;
      loose = loose || bound[g] == kInf;
    }

    PackedTopK<R> tk[ROWK ? 1 : G];
    uint64_t rk = kKcNone;  // ROWK: row g = pair g's sorted top-16
    uint64_t rtp[G];        // ROWK: pair g's k-th word (admission threshold)
#pragma unroll
    for (int g = 0; g < G; g++) rtp[g] = kKcNone;
    if constexpr (!ROWK)
#pragma unroll
      for (int g = 0; g < G; g++) tk[g].init(k);
    int qn[G];  // this wave's queue fills (wave-uniform)
    DIAG_ONLY(uint64_t d_gather = 0, d_push = 0, d_drain = 0, d_loose = 0, d_admit = 0, d_fdrain = 0;)
#pragma unroll
    for (int g = 0; g < G; g++) qn[g] = 0;

    // drain the queues into the per-query top-k lists and publish the bounds
    auto drain_rows = [&]() __attribute__((always_inline)) {
      // lane 16 g + e takes queue entry b0 + e of pair g; 16 entries per pair per pass
      int qmax = 0;
#pragma unroll
      for (int g = 0; g < G; g++) qmax = max(qmax, qn[g]);
      const int rg = lane >> 4, re = lane & 15;
      int qr = qn[0];  // this lane's pair's fill
#pragma unroll
      for (int g = 1; g < G; g++) qr = rg == g ? qn[g] : qr;
      uint64_t thr = rtp[0];
#pragma unroll
      for (int g = 1; g < G; g++) thr = rg == g ? rtp[g] : thr;
      for (int b0 = 0; b0 < qmax; b0 += 16) {
        const int e = b0 + re;
        uint64_t c = e < qr ? pack_kc(qd[wave][rg * QG + e], qi[wave][rg * QG + e]) : kKcNone;
        c = c < thr ? c : kKcNone;
        if (__builtin_amdgcn_ballot_w64(c != kKcNone) == 0) continue;
        kc_steps<2, 1>(c, lane);
        kc_steps<4, 2>(c, lane);
        kc_steps<8, 4>(c, lane);
        kc_steps<128, 8>(c, lane);  // every row ascending
        const uint64_t rv = ((uint64_t)(uint32_t)rev16_i((int)(uint32_t)(c >> 32)) << 32) |
                            (uint32_t)rev16_i((int)(uint32_t)c);
        uint64_t q = rv < rk ? rv : rk;
        kc_steps<128, 8>(q, lane);
        rk = q;
#pragma unroll
        for (int g = 0; g < G; g++) rtp[g] = readlane_u64(rk, 16 * g + k - 1);
        thr = rtp[0];
#pragma unroll
        for (int g = 1; g < G; g++) thr = rg == g ? rtp[g] : thr;
      }
#pragma unroll
      for (int g = 0; g < G; g++) bound[g] = fminf(bound[g], rtp[g] == kKcNone ? kInf : kc_key(rtp[g]));
    };
    auto drain = [&]() __attribute__((always_inline)) {
      DIAG_ONLY(d_drain++;)
      if constexpr (ROWK) drain_rows();
      else for (int b0 = 0; b0 < QG; b0 += 64) {
        bool any = false;
#pragma unroll
        for (int g = 0; g < G; g++) any = any || b0 < qn[g];
        if (!any) break;
        // every pair's queued words first (one LDS round trip for all of them)
        uint64_t cwg[G];
#pragma unroll
        for (int g = 0; g < G; g++) {
          const int e = b0 + lane;
          cwg[g] = e < qn[g] ? pack_kc(qd[wave][g * QG + e], qi[wave][g * QG + e]) : kKcNone;
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
          if (b0 >= qn[g]) continue;
          const uint64_t cw64 = cwg[g];
          const bool p = cw64 < tk[g].tp;
          const uint64_t mk = __ballot(p);
          if (!mk) continue;
          if constexpr (R == 1) {
            if (k <= 16 && qn[g] - b0 <= 16 && __popcll(mk) > 1)
              kc_row16_merge(tk[g], p ? cw64 : kKcNone, lane);
            else if (__popcll(mk) > 4)
              kc_bulk_merge(tk[g], p ? cw64 : kKcNone, lane);
            else
              tk[g].insert(mk, cw64, lane);
          } else {
            if (__popcll(mk) > 4)
              kc_bulk_merge_rows(tk[g], p ? cw64 : kKcNone, lane);
            else
              tk[g].insert(mk, cw64, lane);
          }
          bound[g] = fminf(bound[g], tk[g].td());
        }
      }
#pragma unroll
      for (int g = 0; g < G; g++) qn[g] = 0;
      loose = false;
#pragma unroll
      for (int g = 0; g < G; g++) {
        loose = loose || bound[g] == kInf;
        const uint64_t tp = ROWK ? rtp[g] : tk[ROWK ? 0 : g].tp;
        if (g < it.cnt && tp != kKcNone && lane == 0) {
          atomicMin(&s_wb[g], f2ord(kc_key(tp)));
          tau_lower(pl, qix[g], f2ord(kc_key(tp)));
        }
      }
    };

    // Chunks of 64 codes per wave (256 per workgroup), JB of them per super-batch:
    // all of a super-batch's keys are gathered first (held in registers), then
    // admitted chunk by chunk.  A straight sequence of guarded blocks
    // (compile-time register indices, no selection network) stops where the
    // queue needs draining; one drain site serves every stop.
    DIAG(11, __builtin_amdgcn_s_memtime());
    for (int sb = 0; sb < n; sb += 256 * JB) {
      if (sb > 0) {
#pragma unroll
        for (int j = 0; j < JB; j++) {
          const int i = sb + j * 256 + wave * 64 + lane;
          cw[j].load(lc + (int64_t)(i < n ? i : 0) * M);
        }
      }
      const int tn = min(JB, (n - sb + 255) >> 8);  // chunks with codes (wave-uniform)
      const bool last_sb = sb + 256 * JB >= n;
      DIAG_ONLY(const uint64_t tg0 = __builtin_amdgcn_s_memtime();)
      // G keys per code: dis0 + sum_m LUT[m][code_m], sequential in m (the
      // oracle's order); two chunks at a time, their 2 x M LDS gathers
      // interleaved m-outer for latency hiding
      float dis[JB][G];
      static_assert(JB % 2 == 0, "chunks are gathered in pairs");
#pragma unroll
      for (int jd = 0; jd < JB / 2; jd++) {
        if (2 * jd < tn) {  // wave-uniform
          // opaque copies of the words: keep the LUT addresses of all chunks from
          // being computed up front
          CodeWords<M> cc[2] = {cw[2 * jd], cw[2 * jd + 1]};
#pragma unroll
          for (int h = 0; h < 2; h++)
#pragma unroll
            for (int v = 0; v < M / 4; v++) asm volatile("" : "+v"(cc[h].w[v]));
#pragma unroll
          for (int h = 0; h < 2; h++)
#pragma unroll
            for (int g = 0; g < G; g++) dis[2 * jd + h][g] = it.d0[g];
#pragma unroll
          for (int m = 0; m < M; m++) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
              const V v = lut[m * 256 + cc[h].byte(m)];
#pragma unroll
              for (int g = 0; g < G; g++) dis[2 * jd + h][g] = dis[2 * jd + h][g] + comp(v, g);
            }
          }
        }
      }
      DIAG_ONLY(asm volatile("" ::"v"(dis[0][0]), "v"(dis[JB - 1][G - 1])); d_gather += __builtin_amdgcn_s_memtime() - tg0;)
      if constexpr (R == 1) {
        // A query without a bound gets one from this super-batch: the k-th
        // smallest of the 64 lane minima bounds the final k-th key (those minima
        // are k distinct codes), so only about k codes per wave are admitted
        // instead of every code until the wave's own top-k has filled.  The bound
        // is shared with the other waves (LDS) and workgroups (tau_q).
        if (loose) {
#pragma unroll
          for (int g = 0; g < G; g++) {
            if (bound[g] != kInf) continue;  // wave-uniform
            float mn = kInf;
#pragma unroll
            for (int j = 0; j < JB; j++)
              if (j < tn && sb + j * 256 + wave * 64 + lane < n) mn = fminf(mn, dis[j][g]);
            const float T = wave_kth_smallest(mn, k, lane);
            if (T < kInf && lane == 0) {
              atomicMin(&s_wb[g], f2ord(T));
              tau_lower(pl, qix[g], f2ord(T));
            }
          }
        }
      } else {
        // k > 64: once the super-batch holds k keys (distinct codes), their k-th
        // smallest bounds the final k-th key (JB x 64 per wave: k <= 384 at M = 16)
        if (loose && JB * 64 >= k) {
#pragma unroll
          for (int g = 0; g < G; g++) {
            if (bound[g] != kInf) continue;  // wave-uniform
            uint32_t u[JB];
            int nv = 0;
#pragma unroll
            for (int j = 0; j < JB; j++) {
              const bool v = j < tn && sb + j * 256 + wave * 64 + lane < n;
              u[j] = v ? ukey_of(dis[j][g]) : 0xFFFFFFFFu;
              nv += __popcll(__builtin_amdgcn_ballot_w64(v));
            }
            if (nv < k) continue;
            const int T = (int)(wave_kth_u32<JB>(u, k) ^ 0x80000000u);  // f2ord of the k-th key
            if (lane == 0) {
              atomicMin(&s_wb[g], T);
              tau_lower(pl, qix[g], T);
            }
          }
        }
      }
      loose = false;
#pragma unroll
      for (int g = 0; g < G; g++) {
        // (readfirstlane: one value for the wave, as tau_get -- the two 32-lane halves of
        // the LDS read can straddle another wave's atomicMin)
        if (g < it.cnt) bound[g] = fminf(bound[g], ord2f(__builtin_amdgcn_readfirstlane(s_wb[g])));
        loose = loose || bound[g] == kInf;
      }
      DIAG_ONLY(const uint64_t tb0 = __builtin_amdgcn_s_memtime(); d_loose += tb0 - tg0;)
      int t = 0;
      bool pend = false;  // a drain requested by the last chunk
      // One bit per (chunk, pair) and lane: code of chunk j passes pair g's bound.
      // Most super-batches of a query that already has a bound admit nothing (one
      // ballot decides that); when every queue has room for all of them, the
      // candidates take queue slots from per-wave LDS counters (one atomic per
      // candidate, no per-(chunk, pair) ballots); otherwise, and while a query
      // has no bound yet, the per-chunk admission below runs.
      uint32_t bits = 0;
#pragma unroll
      for (int j = 0; j < JB; j++) {
        if (j < tn) {  // wave-uniform
          const bool valid = sb + j * 256 + wave * 64 + lane < n;
#pragma unroll
          for (int g = 0; g < G; g++) bits |= (uint32_t)(valid && dis[j][g] <= bound[g]) << (j * G + g);
        }
      }
      if (__builtin_amdgcn_ballot_w64(bits != 0) == 0) {
        t = tn;  // nothing to admit in this super-batch
      } else if (!loose) {
        const int c = __popc(bits);  // this lane's candidates (<= JB x G < 32)
        int tot = 0;
#pragma unroll
        for (int b = 0; b < 5; b++) tot += __popcll(__builtin_amdgcn_ballot_w64((c >> b) & 1)) << b;
        int qmax = 0;
#pragma unroll
        for (int g = 0; g < G; g++) qmax = max(qmax, qn[g]);
        if (qmax + tot <= QG) {
          // queue slots from one prefix sum over the wave of the lanes' per-pair
          // counts, packed 32 / G bits per pair (each pair's total <= tot <= QG fits
          // its field, so fields never carry into each other): no LDS atomics
          constexpr int FB = 32 / G;
          uint32_t cp = 0;
#pragma unroll
          for (int g = 0; g < G; g++) {
            uint32_t cg = 0;
#pragma unroll
            for (int j = 0; j < JB; j++) cg += (bits >> (j * G + g)) & 1u;
            cp |= cg << (FB * g);
          }
          const uint32_t incl = wave_incl_scan_u32(cp, lane);
          const uint32_t totp = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
          const uint32_t at = incl - cp;
          constexpr uint32_t FM = FB >= 32 ? 0xFFFFFFFFu : (1u << FB) - 1;
          int off[G];
#pragma unroll
          for (int g = 0; g < G; g++) off[g] = g * QG + qn[g] + (int)((at >> (FB * g)) & FM);
#pragma unroll
          for (int j = 0; j < JB; j++) {
#pragma unroll
            for (int g = 0; g < G; g++) {
              if ((bits >> (j * G + g)) & 1u) {
                qd[wave][off[g]] = dis[j][g];
                qi[wave][off[g]] = sb + j * 256 + wave * 64 + lane;
                off[g]++;
              }
            }
          }
#pragma unroll
          for (int g = 0; g < G; g++) qn[g] += (int)((totp >> (FB * g)) & FM);
          DIAG_ONLY(d_push += tot;)
          t = tn;
        }
      }
      while (t < tn) {
        int stop = tn;       // first chunk not yet admitted
        bool want = false;   // drain requested
        bool go = true;
#pragma unroll
        for (int j = 0; j < JB; j++) {
          if (go && j >= t && j < tn) {  // wave-uniform
            const int i = sb + j * 256 + wave * 64 + lane;
            const bool valid = i < n;
            uint64_t mk[G];
            int tj = 0;
#pragma unroll
            for (int g = 0; g < G; g++) {
              mk[g] = __builtin_amdgcn_ballot_w64(valid && dis[j][g] <= bound[g]);
              tj += __popcll(mk[g]);
            }
            bool full = false;
#pragma unroll
            for (int g = 0; g < G; g++) full = full || qn[g] + __popcll(mk[g]) > QG;
            if (tj > 0) {
              if (full) {  // no room: drain first, then redo this chunk
                stop = j;
                want = true;
                go = false;
              } else {
#pragma unroll
                for (int g = 0; g < G; g++) {
                  if ((mk[g] >> lane) & 1) {
                    const int sl = g * QG + qn[g] + __popcll(mk[g] & lanemask_lt);
                    qd[wave][sl] = dis[j][g];
                    qi[wave][sl] = i;
                  }
                  qn[g] += __popcll(mk[g]);
                  DIAG_ONLY(d_push += __popcll(mk[g]);)
                }
                if (loose) {  // a query of the item has no bound yet: get one now
                  stop = j + 1;
                  want = true;
                  go = false;
                }
              }
            }
          }
        }
        if (stop >= tn) {  // a drain wanted here is left to the end of the super-batch
          pend = want;
          break;
        }
        drain();
        t = stop;
      }
      bool queued = false;
#pragma unroll
      for (int g = 0; g < G; g++) queued = queued || qn[g] > 0;
      DIAG_ONLY(const uint64_t tc0 = __builtin_amdgcn_s_memtime(); d_admit += tc0 - tb0;)
      if (pend || (last_sb && queued)) {
        drain();
      }
      DIAG_ONLY(asm volatile("" ::"v"(ROWK ? rk : tk[0].p[0])); d_fdrain += __builtin_amdgcn_s_memtime() - tc0;)
    }
    DIAG(2, __builtin_amdgcn_s_memtime());
    DIAG(4, n);
    DIAG(5, it.cnt | (it.kind << 8));
    DIAG(6, d_gather);
    DIAG(7, d_push | (d_drain << 32));
    DIAG(8, d_loose);
    DIAG(9, d_admit);
    DIAG(10, d_fdrain);

    // each wave writes its own sorted partial list per pair (merged by k_merge_probes)
    if constexpr (ROWK) {  // lane 16 g + e: entry e of pair g, one store for all pairs
      const int rg = lane >> 4, re = lane & 15;
      int pr = it.pair[0];
#pragma unroll
      for (int g = 1; g < G; g++) pr = rg == g ? it.pair[g] : pr;
      const int64_t slot = (int64_t)pr * 4 + wave;
      if (rg < it.cnt && re < k && !(pl.fault > 0 && slot % pl.fault == 1)) {  // (fault: test hook, write_partial)
        const bool empty = rk == kKcNone;
        pl.part[slot * pl.ks + re] =
            part_rec(empty ? FLT_MAX : kc_key(rk), part_tag(pl.epoch, slot) | xcc_tag(), empty ? -1 : it.beg + (int64_t)(uint32_t)rk);
      }
    } else {
#pragma unroll
      for (int g = 0; g < G; g++) {
        if (g >= it.cnt) continue;
        write_partial<R>(pl, tk[g], (int64_t)it.pair[g] * 4 + wave, k, it.beg, lane);
      }
    }
    if (nxt >= 0) {  // the next item's fields; with kEarly its first loads start here
      unpack(nrec);
      if constexpr (kEarly) issue();
    }
    DIAG(3, __builtin_amdgcn_s_memtime());
    it_no++;
    cur = nxt;
  }
}

#ifndef SCAN_LEAN
#define SCAN_LEAN 1
#endif
#ifndef SCAN_PREFETCH
#define SCAN_PREFETCH 0  // (r06 A/B at C2: 106.9 us with, 106.8 without at JB 4; JB 6 without: 103.7)
#endif
constexpr bool kScanLean = SCAN_LEAN != 0;  // (-DSCAN_LEAN=0: the queue-based k_scan_lists for A/B builds)
constexpr bool kScanPrefetch = SCAN_PREFETCH != 0;  // (-DSCAN_PREFETCH=0: tables loaded at the item start)
#ifndef SCAN_LEAN_JB
#define SCAN_LEAN_JB 6
#endif
constexpr int kLeanJB = SCAN_LEAN_JB;  // code chunks per super-batch of k_scan_lean

// ------------------------------------------------ lean list scan (k <= 16)
// k_scan_lean: the C2 configuration (G = 4 pairs per item, k <= 16, M <= 16,
// fused planning) without the candidate queue.  Same items, LUT build, gathers,
// bounds and partial lists as k_scan_lists<M, 4, 1, JB, true> -- so the same
// merge and bit-identical results -- but a candidate (a code whose key passes
// its pair's bound, about 3 per wave and item at C2) is inserted at once into
// its pair's 16-lane row of the row-packed top-k: one 64-bit compare, a ballot,
// a DPP row shift and two selects, instead of LDS queue slots from a prefix sum,
// a queue round trip and a 16-lane sort network per drain.  The bounds tighten
// at every insertion, and the item's bounds are published (LDS, tau_q) once per
// super-batch.  The next item's record is unpacked before the item's partial
// lists are stored and its bounds published, so its wait does not include them.
// pack_kc of a key given by its bits, in integer ops (scalar when b is):
// unsigned order of the high word == float order, -0 folded into +0
__device__ __forceinline__ uint64_t pack_kc_bits(uint32_t b, uint32_t pos) {
  b = b == 0x80000000u ? 0u : b;
  const uint32_t o = (int32_t)b >= 0 ? (b ^ 0x80000000u) : ~b;
  return ((uint64_t)o << 32) | pos;
}
__device__ __forceinline__ uint64_t row_shr1_u64(uint64_t v) {  // lane i <- lane i - 1 inside each row of 16
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)v, (int)(uint32_t)v, 0x111, 0xf, 0xf, false);
  const uint32_t hi =
      (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(v >> 32), (int)(uint32_t)(v >> 32), 0x111, 0xf, 0xf, false);
  return ((uint64_t)hi << 32) | lo;
}

template <int M, int JB>
__global__ __launch_bounds__(256, 2) void k_scan_lean(ScanArgs a, ListPlan pl) {
  constexpr int G = 4;
  constexpr int LUTN = M * 256;
  constexpr int NV = LUTN / 4 / 256;  // float4 per thread per table row
  static_assert(NV <= 4 && JB % 2 == 0, "lean scan: M <= 16");
  __shared__ __attribute__((aligned(16))) float4 lut[LUTN];  // [m][j][g]
  __shared__ int s_next;
  __shared__ int32_t s_wb[G];
  __shared__ int s_ws[8];
  __shared__ uint16_t s_ex[2][kFusedPlanLists + 1];
  __shared__ uint16_t s_ord[kFusedPlanLists];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // (uniform: positions and slots stay scalar)
  const int k = a.k;
  const int ip = a.ip;
  const int nloc = a.list_hi - a.list_lo;
  const float inv_np = 1.0f / (float)a.nprobe;
  const int rg = lane >> 4, re = lane & 15;  // row-packed top-k: lane 16 g + e = entry e of pair g
  const int2 nn = fused_plan_prefix(pl, nloc, G, s_ex[0], s_ex[1], s_ord, s_ws);
  const int n_items0 = nn.x, n_items = nn.x + nn.y;

  Item<G> it;
  auto unpack = [&](const Rec& rc) __attribute__((always_inline)) {
    const int rv = rc.raw;
    it.l = rc.l;
    it.kind = rc.kind;
    it.cnt = min(G, min(__builtin_amdgcn_readlane(rv, 1), pl.cap) - rc.t * G);
    it.n = __builtin_amdgcn_readlane(rv, 2) - __builtin_amdgcn_readlane(rv, 3);
    it.beg = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane(rv, 4) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane(rv, 3));
#pragma unroll
    for (int g = 0; g < G; g++) {
      it.pair[g] = __builtin_amdgcn_readlane(rv, 5 + g);
      it.d0[g] = __int_as_float(__builtin_amdgcn_readlane(rv, 9 + g));
    }
    bool bad = false;  // a pair id outside the batch: counted in pl.err, the item scans nothing
#pragma unroll
    for (int g = 0; g < G; g++) bad = bad || (g < it.cnt && (unsigned)it.pair[g] >= (unsigned)(a.nq * a.nprobe));
    if (bad) {
      if (lane == 0) atomicAdd(pl.err, 1);
      it.cnt = 0;
#pragma unroll
      for (int g = 0; g < G; g++) it.pair[g] = 0;
    }
#pragma unroll
    for (int g = 0; g < G; g++) it.q[g] = div_small((g < it.cnt ? it.pair[g] : it.pair[0]), a.nprobe, inv_np);
  };
  auto fetch_rec = [&](int idx) __attribute__((always_inline)) {
    return fused_record(a, pl, nloc, idx, n_items0, s_ex[0], s_ex[1], s_ord, G, lane);
  };

  if (tid == 0) {
    const int t = atomicAdd(pl.hdr + 2, 1);
    s_next = t < n_items ? t : -1;
  }
  __syncthreads();
  int cur = s_next;
  if (cur >= 0) unpack(fetch_rec(cur));
  CodeWords<M> cw[JB];
  // An item's table rows: T1[l] (IP: a T3 row, ignored) and its G pairs' T3 rows,
  // one round trip, and its queries' bounds tau_q.  With kScanPrefetch they are
  // loaded for the NEXT item right after the current item's last gathers (its
  // record has arrived by then), so that the 80 KB per item from L2 / the Infinity
  // Cache arrive during the admission, the partial writes and the barrier instead
  // of stalling the next LUT build (the build waited ~5 000 cycles for them, r04
  // stamps: about the per-CU Infinity-Cache rate).
  uint64_t tw[G];  // the queries' tau words, decoded after barrier B
  float4 b1[NV], b3[NV][G];
  // (with kScanPrefetch the T3 rows, 64 of the 80 KB, come ahead; the T1 row is
  // loaded at the item start: all 80 KB ahead left too few VGPRs at JB 6)
  auto prefetch_t3 = [&](const int (&q)[G]) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < G; g++) tw[g] = tau_load(pl, q[g]);
#pragma unroll
    for (int e = 0; e < NV; e++) {
      const int v = e * 256 + tid;
#pragma unroll
      for (int g = 0; g < G; g++) b3[e][g] = reinterpret_cast<const float4*>(a.T3 + (int64_t)q[g] * LUTN)[v];
    }
  };
  auto load_t1 = [&](int l, int q0) __attribute__((always_inline)) {
    const float4* T1l = reinterpret_cast<const float4*>(ip ? a.T3 + (int64_t)q0 * LUTN : a.T1 + (int64_t)l * LUTN);
#pragma unroll
    for (int e = 0; e < NV; e++) b1[e] = T1l[e * 256 + tid];
  };
  if (kScanPrefetch && cur >= 0) prefetch_t3(it.q);
  int it_no = 0;  // (DIAG stamps)
  (void)it_no;
  while (cur >= 0) {
    __syncthreads();  // (A) every wave is done with the previous LUT and has read s_next
    DIAG(0, __builtin_amdgcn_s_memtime());
    int tnext;
    if (tid == 0) tnext = atomicAdd(pl.hdr + 2, 1);
    if (!kScanPrefetch) prefetch_t3(it.q);
    load_t1(it.l, it.q[0]);
    const int n = it.n;
    const uint8_t* lc = a.codes + it.beg * M;
#pragma unroll
    for (int j = 0; j < JB; j++) {  // the item's first JB x 256 codes, in flight during the LUT stores
      const int i = j * 256 + wave * 64 + lane;
      cw[j].load(lc + (int64_t)(i < n ? i : 0) * M);
    }
#pragma unroll
    for (int e = 0; e < NV; e++) {
      const int v = e * 256 + tid;
#pragma unroll
      for (int c = 0; c < 4; c++) {
        float4 o;
#pragma unroll
        for (int g = 0; g < G; g++) {
          const float x3 = comp(b3[e][g], c);
          setc(o, g, ip ? -x3 : __builtin_fmaf(x3, -2.0f, comp(b1[e], c)));  // (oracle: one rounding)
        }
        lut[4 * v + c] = o;
      }
    }
    if (tid == 0) s_next = tnext < n_items ? tnext : -1;
    if (tid < G) s_wb[tid] = f2ord(kInf);
    __syncthreads();  // (B) the LUT, s_next and s_wb are visible
    DIAG(1, __builtin_amdgcn_s_memtime());
    const int nxt = s_next;
    const Rec nrec = fetch_rec(nxt >= 0 ? nxt : cur);  // in flight during the scan
    // this item's fields the scan still needs after the next record is unpacked into `it`
    const int cnt = it.cnt;
    int pr = it.pair[0];  // the partial-list slot of this lane's row (pair rg, this wave)
#pragma unroll
    for (int g = 1; g < G; g++) pr = rg == g ? it.pair[g] : pr;
    const int64_t slot = (int64_t)pr * 4 + wave;
    const bool st = rg < cnt && re < k && !(pl.fault > 0 && slot % pl.fault == 1);  // (fault: test hook)
    const int64_t beg = it.beg;
    int qix[G];
    float bound[G];
    bool loose = false;
    uint64_t rtp[G];  // pair g's k-th word (kKcNone until k entries)
#pragma unroll
    for (int g = 0; g < G; g++) {
      qix[g] = it.q[g];
      bound[g] = g < cnt ? ord2f(tau_decode(pl, tw[g])) : -kInf;
      loose = loose || bound[g] == kInf;
      rtp[g] = kKcNone;
    }
    uint64_t rk = kKcNone;  // row g: pair g's sorted top-16 (key, position) words
    uint32_t pub = 0;       // pairs whose k-th word fell since their bound was last published
    DIAG_ONLY(uint64_t d_gather = 0, d_bounds = 0, d_admit = 0, n_ins = 0;)

    // insert candidate (key, position) into pair g's row
    // Insert candidate word v into pair g's row.  The row keeps its 16 smallest
    // words; a word that lands past the k-th is harmless (it is never published),
    // so pair g's k-th word and bound are refreshed once per super-batch (refresh),
    // not per insertion: one ballot, a DPP row shift and selects, no readlane chain.
    uint32_t ins = 0;  // pairs with an insertion since the last refresh
    auto insert = [&](int g, uint64_t v) __attribute__((always_inline)) {
      if (!(v < rtp[g])) return;  // (rtp[g]: pair g's k-th word at the last refresh)
      const uint64_t lt = __builtin_amdgcn_ballot_w64(rk < v);
      const int p = __popcll((lt >> (16 * g)) & 0xFFFFull);
      const uint64_t sh = row_shr1_u64(rk);
      rk = rg == g ? (re > p ? sh : (re == p ? v : rk)) : rk;
      ins |= 1u << g;
      DIAG_ONLY(n_ins++;)
    };
    auto refresh = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int g = 0; g < G; g++) {
        if ((ins >> g) & 1u) {
          rtp[g] = readlane_u64(rk, 16 * g + k - 1);
          if (rtp[g] != kKcNone) bound[g] = fminf(bound[g], kc_key(rtp[g]));
        }
      }
      pub |= ins;
      ins = 0;
    };
    auto publish = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int g = 0; g < G; g++) {
        if (((pub >> g) & 1u) && rtp[g] != kKcNone && lane == 0) {
          atomicMin(&s_wb[g], f2ord(kc_key(rtp[g])));
          tau_lower(pl, qix[g], f2ord(kc_key(rtp[g])));
        }
      }
      pub = 0;
    };

    DIAG(11, __builtin_amdgcn_s_memtime());
    for (int sb = 0; sb < n; sb += 256 * JB) {
      DIAG_ONLY(const uint64_t tg0 = __builtin_amdgcn_s_memtime();)
      // this wave's chunks with codes (wave-uniform): chunk j holds codes sb + 256 j + 64 wave + lane
      const int tn = max(0, min(JB, (n - sb - 64 * wave + 255) >> 8));
      const bool last_sb = sb + 256 * JB >= n;
      // G keys per code: dis0 + sum_m LUT[m][code_m], sequential in m (the oracle's order);
      // two chunks at a time (their 2 M gathers interleaved), a lone last chunk alone
      float dis[JB][G];
#pragma unroll
      for (int jd = 0; jd < JB / 2; jd++) {
        if (2 * jd + 1 < tn) {
          CodeWords<M> cc[2] = {cw[2 * jd], cw[2 * jd + 1]};
#pragma unroll
          for (int h = 0; h < 2; h++)
#pragma unroll
            for (int v = 0; v < M / 4; v++) asm volatile("" : "+v"(cc[h].w[v]));
#pragma unroll
          for (int h = 0; h < 2; h++)
#pragma unroll
            for (int g = 0; g < G; g++) dis[2 * jd + h][g] = it.d0[g];
#pragma unroll
          for (int m = 0; m < M; m++) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
              const float4 v = lut[m * 256 + cc[h].byte(m)];
#pragma unroll
              for (int g = 0; g < G; g++) dis[2 * jd + h][g] = dis[2 * jd + h][g] + comp(v, g);
            }
          }
        } else if (2 * jd < tn) {
          CodeWords<M> cc = cw[2 * jd];
#pragma unroll
          for (int v = 0; v < M / 4; v++) asm volatile("" : "+v"(cc.w[v]));
#pragma unroll
          for (int g = 0; g < G; g++) dis[2 * jd][g] = it.d0[g];
#pragma unroll
          for (int m = 0; m < M; m++) {
            const float4 v = lut[m * 256 + cc.byte(m)];
#pragma unroll
            for (int g = 0; g < G; g++) dis[2 * jd][g] = dis[2 * jd][g] + comp(v, g);
          }
        }
      }
      DIAG_ONLY(asm volatile("" ::"v"(dis[0][0]), "v"(dis[JB - 1][G - 1])); const uint64_t tg1 = __builtin_amdgcn_s_memtime(); d_gather += tg1 - tg0;)
      if (!last_sb) {  // the next super-batch's codes, in flight during this one's admission
#pragma unroll
        for (int j = 0; j < JB; j++) {
          const int i = sb + 256 * JB + j * 256 + wave * 64 + lane;
          cw[j].load(lc + (int64_t)(i < n ? i : 0) * M);
        }
      }
      if (kScanPrefetch && last_sb && nxt >= 0) {
        // the next item: its record unpacked here (its load is the oldest in flight, so
        // this waits for nothing younger), then its table rows and bounds loaded, in
        // flight during this item's admission, partial writes and barrier (see prefetch)
        unpack(nrec);
        prefetch_t3(it.q);
      }
      if (loose) {
        // a pair without a bound gets one from this super-batch: the k-th smallest
        // of the 64 lane minima bounds the final k-th key (k distinct codes)
#pragma unroll
        for (int g = 0; g < G; g++) {
          if (bound[g] != kInf) continue;  // wave-uniform
          float mn = kInf;
#pragma unroll
          for (int j = 0; j < JB; j++)
            if (j < tn && sb + j * 256 + wave * 64 + lane < n) mn = fminf(mn, dis[j][g]);
          const float T = wave_kth_smallest(mn, k, lane);
          if (T < kInf && lane == 0) {
            atomicMin(&s_wb[g], f2ord(T));
            tau_lower(pl, qix[g], f2ord(T));
          }
        }
      }
      loose = false;
#pragma unroll
      for (int g = 0; g < G; g++) {
        // (readfirstlane: one value for the wave, DESIGN.md §4 "Uniform bounds")
        if (g < cnt) bound[g] = fminf(bound[g], ord2f(__builtin_amdgcn_readfirstlane(s_wb[g])));
        loose = loose || bound[g] == kInf;
      }
      DIAG_ONLY(const uint64_t tb1 = __builtin_amdgcn_s_memtime(); d_bounds += tb1 - tg1;)
      // admission: one ballot per chunk for all pairs, then per pair only where a
      // chunk has candidates; each candidate inserted at once
#pragma unroll
      for (int j = 0; j < JB; j++) {
        if (j < tn) {  // wave-uniform
          const int i0 = sb + j * 256 + wave * 64;
          const bool valid = i0 + lane < n;
          bool c = false;
#pragma unroll
          for (int g = 0; g < G; g++) c = c || dis[j][g] <= bound[g];
          if (__builtin_amdgcn_ballot_w64(valid && c) == 0) continue;
#pragma unroll
          for (int g = 0; g < G; g++) {
            uint64_t mk = __builtin_amdgcn_ballot_w64(valid && dis[j][g] <= bound[g]);
            while (mk) {
              const int src = (int)__builtin_ctzll(mk);
              mk &= mk - 1;
              const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(dis[j][g]), src);
              insert(g, pack_kc_bits(b, (uint32_t)(i0 + src)));
            }
          }
        }
      }
      refresh();
      DIAG_ONLY(d_admit += __builtin_amdgcn_s_memtime() - tb1;)
      if (!last_sb) publish();  // (the last super-batch's bounds: after the next record is unpacked)
    }
    DIAG(2, __builtin_amdgcn_s_memtime());
    DIAG(4, n);
    DIAG(5, it.cnt | (it.kind << 8));
    DIAG(6, d_gather);
    DIAG(7, n_ins);
    DIAG(8, d_bounds);
    DIAG(9, d_admit);
    DIAG(10, 0);
    // the next item's fields (without the prefetch: its record load is older than the
    // stores and atomics below, so this waits for it alone), then this item's bounds
    // and partial lists
    if (!kScanPrefetch && nxt >= 0) unpack(nrec);
    publish();
    if (st) {
      const bool empty = rk == kKcNone;
      pl.part[slot * pl.ks + re] =
          part_rec(empty ? FLT_MAX : kc_key(rk), part_tag(pl.epoch, slot) | xcc_tag(), empty ? -1 : beg + (int64_t)(uint32_t)rk);
    }
    DIAG(3, __builtin_amdgcn_s_memtime());
    DIAG_ONLY(it_no++;)
    cur = nxt;
  }
}

// ------------------------------------------- large-nlist coarse (no key matrix)
// Segmented coarse quantizer: workgroup = 16 queries x one segment of `seg`
// centroids, walked in key tiles of 128 (coarse_key_tile: the MFMA keys of
// k_coarse_gemm).  Each tile's keys go through LDS; wave w keeps the nprobe best
// (key, list) words of queries 4w .. 4w + 3 in a packed one-row top-k, into
// which a tile's candidates under its nprobe-th are inserted one by one when
// few, bulk-merged when many.  Output: cand [nq][nseg][nprobe] packed words
// (kKcNone = none).  The [nq][nlist] key matrix is never written (C4: 1024 x
// 65536 keys would be 256 MB per chunk).
constexpr int kSegQ = 128;  // candidate queue per query (k_coarse_segtop)
__global__ __launch_bounds__(256) void k_coarse_segtop(const float* __restrict__ x, int64_t nq, int d,
                                                       const float* __restrict__ centT, int ldc,
                                                       const float* __restrict__ cn, int nlist, int ip, int seg,
                                                       int nseg, int nprobe, uint64_t* __restrict__ cand) {
  extern __shared__ __attribute__((aligned(16))) float g_lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int64_t q0 = (int64_t)(blockIdx.x / nseg) * GQ;
  const int sg = blockIdx.x % nseg;
  const int cb = sg * seg, ce = min(nlist, cb + seg);
  const int dk = (d + 63) & ~63;
  float* xs = g_lds;             // [dk][GQ]
  float* xn = xs + dk * GQ;      // [GQ] + 128 scratch
  float* kt = xn + GQ + GQ * 8;  // [GQ][GC] key tile
  // per query a queue of candidate words under its running nprobe-th, merged 64 at a
  // time (kSegQ per query): a tile's survivors are appended, not merged one tile at a time
  uint64_t* cq = reinterpret_cast<uint64_t*>(kt + GQ * GC);
  coarse_stage_queries(xs, xn, x, q0, nq, d, dk, tid);
  const int i16 = lane & 15, k4 = lane >> 4;
  const uint64_t lt = (1ull << lane) - 1;
  PackedTopK<1> tk[4];  // queries 4 wave .. 4 wave + 3
  int qn[4];            // queue fills (wave-uniform)
#pragma unroll
  for (int u = 0; u < 4; u++) {
    tk[u].init(nprobe);
    qn[u] = 0;
  }
  auto drain = [&](int u) __attribute__((always_inline)) {
    uint64_t* qv = cq + (wave * 4 + u) * kSegQ;
    for (int b = 0; b < qn[u]; b += 64) {
      uint64_t c = b + lane < qn[u] ? qv[b + lane] : kKcNone;
      c = c < tk[u].tp ? c : kKcNone;
      if (__builtin_amdgcn_ballot_w64(c != kKcNone)) kc_bulk_merge(tk[u], c, lane);
    }
    qn[u] = 0;
  };
  for (int t0 = cb; t0 < ce; t0 += GC) {
    f4 acc[NTL];
    coarse_key_tile(acc, xs, GQ, 0, centT, ldc, nlist, d, dk, t0 + wave * 32, lane);
    __syncthreads();  // xn (first tile); the previous tile's keys have been read
#pragma unroll
    for (int t = 0; t < NTL; t++) {
      const int c = t0 + wave * 32 + t * 16 + i16;
      const float cnv = ip ? 0.f : cn[min(c, nlist - 1)];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int i = k4 * 4 + r;
        kt[i * GC + wave * 32 + t * 16 + i16] = coarse_key(acc[t][r], xn[i], cnv, ip);
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int i = wave * 4 + u;
#pragma unroll
      for (int h = 0; h < GC / 64; h++) {
        const int c = t0 + h * 64 + lane;
        const uint64_t p = c < ce ? pack_kc(kt[i * GC + h * 64 + lane], c) : kKcNone;
        const bool pass = p < tk[u].tp;
        const uint64_t mk = __builtin_amdgcn_ballot_w64(pass);
        if (!mk) continue;  // wave-uniform
        const int cnt = (int)__popcll(mk);
        if (qn[u] + cnt > kSegQ) drain(u);
        if (pass) cq[i * kSegQ + qn[u] + (int)__popcll(mk & lt)] = p;
        qn[u] += cnt;
      }
    }
  }
#pragma unroll
  for (int u = 0; u < 4; u++) {
    drain(u);
    const int64_t q = q0 + wave * 4 + u;
    if (q < nq && lane < nprobe) cand[(q * nseg + sg) * nprobe + lane] = tk[u].p[0];
  }
}

// Per query (one wave): merge its nseg x nprobe segment candidates into the
// final top-nprobe by (key, list), then emit and plan as k_coarse_select does.
template <int IP>
__global__ __launch_bounds__(256) void k_coarse_select_cand(const uint64_t* __restrict__ cand, int64_t nq, int nseg,
                                                            int nprobe, float* __restrict__ out_dis,
                                                            int64_t* __restrict__ out_list,
                                                            const float* __restrict__ x, int d, CoarsePlan cp) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nq) return;  // wave-uniform
  const int total = nseg * nprobe;
  const uint64_t* row = cand + q * total;
  PackedTopK<1> tk;
  tk.init(nprobe);
  for (int b0 = 0; b0 < total; b0 += 256) {
    uint64_t p[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int e = b0 + u * 64 + lane;
      p[u] = e < total ? row[e] : kKcNone;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const bool pass = p[u] < tk.tp;
      const uint64_t mk = __builtin_amdgcn_ballot_w64(pass);
      if (!mk) continue;  // wave-uniform
      if (__popcll(mk) > 4)
        kc_bulk_merge(tk, pass ? p[u] : kKcNone, lane);
      else
        tk.insert(mk, p[u], lane);
    }
  }
  coarse_emit<IP>(tk.p[0], q, lane, nprobe, out_dis, out_list, x, d, cp);
}

// ---- stale partial lists: accounting, event log, repair
// hdr[kHdrStale] counts (query, merge launch) pairs that read an entry whose tag
// was not this batch's, hdr[kHdrRepair] the probes k_merge_probes rescanned, and
// hdr[kHdrLog] the events offered to the log (the first kEvLog are kept:
// ListPlan::evlog, 8 words each -- site | reader XCD << 8, query, list j | rank
// << 16, expected tag, found tag, found key bits, epoch, and the system-scope
// re-read result: the reads until the tag was fresh (full merge), or 0xFFFFFFFF
// when it never was within kSpin reads).
__device__ __forceinline__ int log_slot(const ListPlan& pl) {
  // (the counter stops growing once the log is full, so it can never wrap negative)
  if (__hip_atomic_load(pl.hdr + kHdrLog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= kEvLog) return -1;
  const int e = atomicAdd(pl.hdr + kHdrLog, 1);
  return (e >= 0 && e < kEvLog) ? e : -1;
}
__device__ __forceinline__ void log_stale(const ListPlan& pl, int e, int site, int64_t q, int j, int i, uint32_t expect,
                                          uint32_t found, uint32_t keyb, uint32_t spin) {
  uint32_t* r = pl.evlog + 8 * e;
  r[0] = (uint32_t)site | (xcc_tag() >> 20);
  r[1] = (uint32_t)q;
  r[2] = (uint32_t)j | ((uint32_t)i << 16);
  r[3] = expect;
  r[4] = found;
  r[5] = keyb;
  r[6] = pl.epoch;
  r[7] = spin;
}
// re-read a stale record's (key, tag) word at system scope until its tag is
// fresh: the number of reads it took, or 0xFFFFFFFF (never, within kSpin)
constexpr int kSpin = 2000;
__device__ __forceinline__ uint32_t spin_fresh(const uint4* rec, uint32_t expect) {
  for (int t = 0; t < kSpin; t++) {
    const uint64_t v = __hip_atomic_load(reinterpret_cast<const uint64_t*>(rec), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM);
    if (tag_ok((uint32_t)(v >> 32), expect)) return (uint32_t)t + 1;
    __builtin_amdgcn_s_sleep(8);
  }
  return 0xFFFFFFFFu;
}

// Rescan probe p of query q from the index itself -- the list's codes, the
// query's T3 row and the list's T1 row, with the scan's arithmetic (LUT entry
// fma(T3, -2, T1) or -T3, dis0 + sum over m in order), so every key is the
// scan's to the bit -- and merge every code of the list into tk by (key, label),
// skipping entries tk already holds (a partial list can be stale from some rank
// on, after its fresh prefix was merged).  One wave; rare (the stale-list path).
template <int R>
__device__ __forceinline__ void repair_probe(const ScanArgs& a, const ListPlan& pl, int64_t q, int p, WaveTopK<R>& tk,
                                          int lane) {
  const int64_t pair = q * a.nprobe + p;
  const int64_t l = a.probe_list[pair];
  const int64_t beg = a.list_off[l], n = a.list_off[l + 1] - beg;
  const float d0 = pl.pd0[pair];
  const int M = a.M;
  const float* T3q = a.T3 + q * (int64_t)M * 256;
  const float* T1l = a.ip ? T3q : a.T1 + l * (int64_t)M * 256;
  for (int64_t i0 = 0; i0 < n; i0 += 64) {
    const int64_t i = i0 + lane;
    const bool valid = i < n;
    const int64_t pos = beg + (valid ? i : 0);
    const uint32_t* cw = reinterpret_cast<const uint32_t*>(a.codes + pos * M);
    float key = d0;
    for (int m4 = 0; m4 < M / 4; m4++) {
      const uint32_t w = cw[m4];
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const int e = (m4 * 4 + b) * 256 + (int)((w >> (8 * b)) & 255u);
        const float x3 = T3q[e];
        const float lv = a.ip ? -x3 : __builtin_fmaf(x3, -2.0f, T1l[e]);
        key = key + lv;
      }
    }
    const int64_t id = valid ? a.ids[pos] : kSentinelId;
    uint64_t mask = __builtin_amdgcn_ballot_w64(valid && lexless(key, id, tk.td, tk.ti));
    while (mask) {
      const int src = __builtin_ctzll(mask);
      mask &= mask - 1;
      const float vd = readlane_f(key, src);
      const int64_t vi = id_readlane(id, src);
      bool dup = false;
#pragma unroll
      for (int r = 0; r < R; r++) dup = dup || __builtin_amdgcn_ballot_w64(tk.d[r] == vd && tk.id[r] == vi) != 0;
      if (!dup) tk.insert(1ull << src, key, id, lane);
    }
  }
}

// Per query (one wave): merge the per-wave partial lists of every scanned
// probe ([probe][4 waves][k] tagged records, sorted by (key, position)).  All
// entries are fetched in batches of 64 lanes x B loads (one round trip per
// batch); labels are looked up only for entries that can still enter the top-k.
// An entry whose tag is not this batch's is never used: its probe is rescanned
// (repair_probe) after the other lists are merged.
template <int R>
__global__ __launch_bounds__(256) void k_merge_probes(ScanArgs a, ListPlan pl) {
  constexpr int B = 4;
  __shared__ uint64_t s_bad[4][kMaxK / 64];  // per wave: the probes with a stale entry (full merge)
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  if (blockIdx.x == 0) {  // the scan consumed the counts and its work counter: zero them for the next batch
    const int nloc = a.list_hi - a.list_lo;
    for (int i = threadIdx.x; i < 2 * nloc; i += 256) pl.cnt[i] = 0;
    if (threadIdx.x == 0) pl.hdr[2] = 0;
  }
  const int64_t q = (int64_t)blockIdx.x * 4 + wave;
  if (q >= a.nq) return;
  const int k = a.k;
  const int np = a.nprobe;
  const float pad = a.ip ? -FLT_MAX : FLT_MAX;
  const float sgn = a.ip ? -1.f : 1.f;  // key -> reported value
  const int64_t ks = pl.ks;
  // this query's stale read already counted (hdr[kHdrStale] counts a query once per
  // search: the fast path or an earlier k > 64 merge stage that fell back here)
  bool counted = false;
  if (R == 1 && np * 4 <= 64) {
    // fast path: lane j owns partial list j = (probe j/4, wave j%4), sorted by
    // (key, label).  T = the k-th smallest list head bounds the k-th key (k
    // distinct entries are at or below it), so only the list prefixes <= T are
    // candidates: they are compacted into one slot per lane, their labels
    // looked up, and one 64-lane sort yields the top-k.
    __shared__ float sd[4][64];
    __shared__ int64_t sp[4][64];
    constexpr int U = 16;
    float d[U];
    const int p = min(lane >> 2, np - 1);
    // the planner's mask of the probes the scan covered (empty or foreign lists are not)
    const bool scanned = (lane >> 2) < np && ((pl.qmask[q] >> p) & 1);
    const int64_t slot = (q * np + p) * 4 + (lane & 3);
    const uint32_t expect = part_tag(pl.epoch, slot);
    // clamped loads, only for scanned probes: slots of unscanned probes (empty or
    // foreign lists, lanes past nprobe) were never written this batch (their
    // contents are stale and must not be used), and a list-range shard scans few of
    // a query's probes -- at N = 8 about 2 of 16, so loading every slot read 8x the
    // partial lists the scan wrote
    // (unconditional loads: an unscanned lane reads the first scanned lane's slot --
    // the same lines, no extra traffic -- and ignores what it reads)
    int64_t pos[U];
    bool fresh[U];
    const uint64_t sm = __builtin_amdgcn_ballot_w64(scanned);
    const int64_t rslot = scanned || !sm ? slot : (int64_t)__builtin_amdgcn_readlane((int)slot, (int)__builtin_ctzll(sm));
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint4 r = pl.part[rslot * ks + min(u, k - 1)];
      d[u] = rec_key(r);
      pos[u] = rec_pos(r);
      fresh[u] = tag_ok(r.y, expect);
    }
    int bad_u = -1;
#pragma unroll
    for (int u = U - 1; u >= 0; u--) bad_u = (scanned && u < k && !fresh[u]) ? u : bad_u;
    if (__builtin_amdgcn_ballot_w64(bad_u >= 0)) {  // stale entries: the full merge below re-reads and repairs
      counted = true;  // (the full merge does not count this query again)
      if (lane == (int)__builtin_ctzll(__builtin_amdgcn_ballot_w64(bad_u >= 0))) atomicAdd(pl.hdr + kHdrStale, 1);
      if (bad_u >= 0) {
        const int ev = log_slot(pl);
        if (ev >= 0) {  // (and whether an immediate system-scope re-read is already fresh)
          const uint4 r = pl.part[slot * ks + bad_u];
          log_stale(pl, ev, 1, q, lane, bad_u, expect, r.y, r.x,
                    spin_fresh(pl.part + slot * ks + bad_u, expect) == 1 ? 1u : 0u);
        }
      }
    } else {
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; u++) ok[u] = scanned && u < k && pos_ok(a, pl, pos[u]);
      // a bound on the k-th key from m sorted lists: with j = ceil(k / m) - 1, the
      // i = ceil(k / (j + 1)) smallest of the lists' entries j are each preceded in
      // their list by j entries, so i (j + 1) >= k entries are at or below the i-th
      // smallest of them (m >= k: the k-th smallest list head).  A list-range shard
      // scans few probes of a query (N = 8: about 2 of 16, m = 8 < k), so the
      // head-only bound left nearly every query to the full merge below.
      const int m = __popcll(__builtin_amdgcn_ballot_w64(ok[0]));
      if (m == 0) {  // nothing scanned for this query (every probe empty or outside the range)
        if (lane < k) {
          a.outD[q * k + lane] = pad;
          a.outI[q * k + lane] = -1;
        }
        return;
      }
      const int jb = (k + m - 1) / m - 1;  // < k <= U (wave-uniform)
      float vj = kInf;
#pragma unroll
      for (int u = 0; u < U; u++) vj = (u == jb && ok[u]) ? d[u] : vj;
      const float T = wave_kth_smallest(vj, (k + jb) / (jb + 1), lane);
      const uint64_t lt = (1ull << lane) - 1;
      int total = 0;
#pragma unroll
      for (int u = 0; u < U; u++) {
        const bool pass = ok[u] && d[u] <= T;
        const uint64_t mk = __builtin_amdgcn_ballot_w64(pass);
        const int at = total + __popcll(mk & lt);
        if (pass && at < 64) {
          sd[wave][at] = d[u];
          sp[wave][at] = pos[u];
        }
        total += __popcll(mk);
      }
      // a list whose 16 loaded entries all pass may hold more candidates
      const bool cut = k > U && __builtin_amdgcn_ballot_w64(ok[U - 1] && d[U - 1] <= T) != 0;
      if (T < kInf && total <= 64 && !cut) {
        __builtin_amdgcn_wave_barrier();
        float cd = lane < total ? sd[wave][lane] : kInf;
        int64_t ci = lane < total ? a.ids[sp[wave][lane]] : kSentinelId;
        bitonic_sort64<2>(cd, ci, lane);
        if (lane < k) {
          const bool empty = ci == kSentinelId;
          a.outD[q * k + lane] = empty ? pad : sgn * cd;
          a.outI[q * k + lane] = empty ? -1 : ci;
        }
        return;
      }
    }
  }
  if constexpr (R >= 2) {
    // k > 64, nprobe <= 64: k_merge_radix / k_merge_big ran first and merged every
    // query whose candidates fit their buffers and whose lists were all fresh;
    // the rest (ties, stale entries) take the full merge below
    if (np <= 64) {
      const int done = pl.qdone[q];  // 1: merged; 2: a stale read (counted), merge here
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) pl.qdone[q] = 0;  // zero for the next batch
      if (done == 1) return;
      counted = done == 2;
    }
  }
  // Full merge.  For k > 64 the entries are visited rank-major across the
  // L = 4 nprobe sorted lists (every list's entry i, then every list's entry
  // i + 1, ...), so the running k-th key falls fast and few labels are looked
  // up; once a batch of at least L consecutive entries (one per list) admits
  // nothing, no later entry of any list can (each list is ascending and the
  // k-th key only falls).  Stale entries mark their probe in s_bad.
  if (lane < kMaxK / 64) s_bad[wave][lane] = 0;
  __builtin_amdgcn_wave_barrier();
  WaveTopK<R> tk;
  tk.init(k);
  const int L = 4 * np;
  const int total = L * k;
  const int qmw = pl.qmw;
  bool stale = false;
  for (int e0 = 0; e0 < total; e0 += 64 * B) {
    float d[B];
    int64_t pos[B];
#pragma unroll
    for (int b = 0; b < B; b++) {
      const int e = e0 + b * 64 + lane;
      d[b] = kInf;
      pos[b] = -1;
      if (e < total) {
        // R == 1 (k <= 64, a fast-path miss): list-major order; R >= 2: rank-major
        const int i = R == 1 ? e % k : e / L;
        const int j = R == 1 ? e / k : e - (e / L) * L;  // rank i of list j = (probe j / 4, wave j % 4)
        const int p = j >> 2;
        const bool scanned = (pl.qmask[q * qmw + (p >> 6)] >> (p & 63)) & 1;
        const int64_t slot = q * (int64_t)L + j;
        const uint32_t expect = part_tag(pl.epoch, slot);
        bool bad = false;
        if (scanned) {
          // k > 64 writes only each list's valid prefix ((count, tag) in partN)
          int nv = k;
          if (R >= 2) {
            const uint2 nt = pl.partN[slot];
            if (tag_ok(nt.y, expect)) nv = (int)nt.x;
            else bad = true;
            const int ev = (bad && i == 0) ? log_slot(pl) : -1;
            if (ev >= 0)
              log_stale(pl, ev, 2, q, j, 0xFFFF, expect, nt.y, nt.x,
                        spin_fresh(reinterpret_cast<const uint4*>(pl.partN + slot), expect));
          }
          if (!bad && i < nv) {
            const uint4* rp = pl.part + slot * ks + i;
            const uint4 r = *rp;
            if (tag_ok(r.y, expect)) {
              d[b] = rec_key(r);
              pos[b] = rec_pos(r);
            } else {
              bad = true;
              const int ev = log_slot(pl);
              if (ev >= 0) log_stale(pl, ev, 2, q, j, i, expect, r.y, r.x, spin_fresh(rp, expect));
            }
          }
        }
        if (bad) {
          atomicOr(reinterpret_cast<unsigned long long*>(&s_bad[wave][p >> 6]), 1ull << (p & 63));
          stale = true;
        }
      }
    }
    bool any = false;
#pragma unroll
    for (int b = 0; b < B; b++) any = any || (pos[b] >= 0 && d[b] <= tk.td);
    if (R >= 2 && L <= 64 * B && __builtin_amdgcn_ballot_w64(any) == 0) break;  // wave-uniform
#pragma unroll
    for (int b = 0; b < B; b++) {
      const bool maybe = pos_ok(a, pl, pos[b]) && d[b] <= tk.td;
      int64_t id = kSentinelId;
      if (maybe) id = a.ids[pos[b]];
      const bool pass = maybe && lexless(d[b], id, tk.td, tk.ti);
      const uint64_t mask = __ballot(pass);
      if (!mask) continue;
      if (__popcll(mask) > 6) {
        if constexpr (R == 1)
          bulk_merge_row(tk, pass ? d[b] : kInf, pass ? id : kSentinelId, lane);
        else
          bulk_merge_rows(tk, pass ? d[b] : kInf, pass ? id : kSentinelId, lane);
        continue;
      }
      tk.insert(mask, d[b], id, lane);
    }
  }
  if (__builtin_amdgcn_ballot_w64(stale)) {  // (wave-uniform) rescan every probe with a stale entry
    __builtin_amdgcn_wave_barrier();
    if (lane == 0 && !counted) atomicAdd(pl.hdr + kHdrStale, 1);
    for (int w = 0; w < (np + 63) / 64; w++) {
      uint64_t m = s_bad[wave][w];
      while (m) {
        const int p = w * 64 + (int)__builtin_ctzll(m);
        m &= m - 1;
        repair_probe<R>(a, pl, q, p, tk, lane);
        if (lane == 0) atomicAdd(pl.hdr + kHdrRepair, 1);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int idx = r * 64 + lane;
    if (idx < k) {
      const bool empty = tk.id[r] == kSentinelId;
      a.outD[q * k + idx] = empty ? pad : sgn * tk.d[r];
      a.outI[q * k + idx] = empty ? -1 : tk.id[r];
    }
  }
}

// ------------------------------------------------- probe merge, k > 64
// One wave per query (nprobe <= 64).  The L = 4 nprobe per-wave partial lists
// of the query's scanned probes are sorted by (key, position) and hold
// partN[j] valid entries each (k > 64: only those are written).
//  1. Candidate prefixes: every list entirely (C = sum of lengths).
//  2. While C > CAP: sample each list's prefix at stride r = ceil(C / NS)
//     (positions r-1, 2r-1, ...); if the lists hold m_j samples <= v, at least
//     r * sum m_j entries are <= v, so the ceil(k / r)-th smallest sample T
//     bounds the final k-th key.  Each list's prefix <= T is found by binary
//     search; C shrinks to at most k + r + L r per round (r = 1: exact).
//  3. The prefixes are compacted into LDS; the exact k-th key (bisection on
//     the order-preserving integers) cuts them to the k best and their ties.
//  4. Labels for those only; one bitonic sort by (key, label) in LDS.
// Queries whose ties overflow CAP are left to k_merge_probes' full merge
// (flag in pl.qdone).  Replaces the per-query selection of faiss-gpu's
// pass2SelectLists (classify_stages.py:127-136; 78 % of the time at K = 1000,
// MICRO_GPU_profiling/out_img/profile_experiment_5_topK.png).
constexpr int kBigCap = 2048;

__global__ __launch_bounds__(64) void k_merge_big(ScanArgs a, ListPlan pl) {
  constexpr int SV = 20;  // sample slots per lane
  __shared__ float cd[kBigCap];
  __shared__ int64_t cl[kBigCap];  // code positions, then labels
  __shared__ int lens[257];        // per-list candidate prefix lengths, then exclusive offsets
  __shared__ int sp[257];          // exclusive prefix of the per-list sample counts
  const int lane = threadIdx.x;
  const int64_t q = blockIdx.x;
  const int k = a.k, np = a.nprobe, L = 4 * np;
  const uint64_t qm = pl.qmask[q];
  const int64_t qb = q * (int64_t)L;  // list j: entries at (qb + j) * k + i
  const float pad = a.ip ? -FLT_MAX : FLT_MAX;
  const float sgn = a.ip ? -1.f : 1.f;
  // every record and count read is tag-checked: a stale one sends the query to
  // k_merge_probes' full merge (which rescans its probe) instead of being used
  bool stale = false;
  // (the tag test is a bitwise or, not a short-circuit: no branch per load, so
  // independent loads stay in flight together)
  auto key_at = [&](int j, int i) __attribute__((always_inline)) {
    const uint2 v = *reinterpret_cast<const uint2*>(pl.part + (qb + j) * pl.ks + i);
    stale = stale | !tag_ok(v.y, part_tag(pl.epoch, qb + j));
    return __uint_as_float(v.x);
  };

  int C = 0;
#pragma unroll
  for (int t = 0; t < 4; t++) {
    const int j = t * 64 + lane;
    int n = 0;
    if (j < L && ((qm >> (j >> 2)) & 1)) {
      const uint2 nt = pl.partN[qb + j];
      n = (int)nt.x;
      if (!tag_ok(nt.y, part_tag(pl.epoch, qb + j))) {
        stale = true;
        n = 0;
      } else if (n < 0 || n > k) {  // a partial list holds at most k entries
        atomicAdd(pl.err, 1);
        n = 0;
      }
    }
    lens[j] = n;
    C += n;
  }
  if (__builtin_amdgcn_ballot_w64(stale)) {  // (uniform) counted here; k_merge_probes repairs (qdone 2)
    if (lane == 0) {
      atomicAdd(pl.hdr + kHdrStale, 1);
      pl.qdone[q] = 2;
    }
    return;
  }
  C = wave_sum_i(C);
  __builtin_amdgcn_wave_barrier();
  uint32_t Tu = 0xFFFFFFFFu;  // every entry is a candidate
  bool exact = false;         // Tu is the exact k-th key (a round sampled every entry)
  const int Cmax = max(2 * k, k + 64);
  for (int round = 0; C > Cmax && round < 8; round++) {
    const int r = (C + 64 * SV - 1) / (64 * SV);
    exact = r == 1;
    // exclusive prefix of per-list sample counts (lists in j order: 4 scans of 64)
    int carry = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const int j = t * 64 + lane;
      const int c = lens[j] / r;
      const int incl = wave_incl_scan(c, lane);
      sp[j] = carry + incl - c;
      carry += __builtin_amdgcn_readlane(incl, 63);
    }
    if (lane == 0) sp[256] = carry;
    __builtin_amdgcn_wave_barrier();
    const int S = carry, K2 = (k + r - 1) / r;
    if (S < K2) break;  // too few samples to bound (cannot happen for C > kBigCap, L <= 256)
    // sample positions first (LDS searches), then all SV loads at once (positions of
    // absent samples clamped to entry 0 of list 0 and their keys dropped)
    int sj[SV], si[SV];
#pragma unroll
    for (int t = 0; t < SV; t++) {
      const int e = t * 64 + lane;
      int lo = 0, hi = 256;  // largest j with sp[j] <= e
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (sp[mid] <= e) lo = mid; else hi = mid;
      }
      sj[t] = e < S ? lo : 0;
      si[t] = e < S ? (e - sp[lo] + 1) * r - 1 : 0;
    }
    uint32_t u[SV];
#pragma unroll
    for (int t = 0; t < SV; t++) {
      const uint2 v = *reinterpret_cast<const uint2*>(pl.part + (qb + sj[t]) * pl.ks + si[t]);
      const bool ok = t * 64 + lane < S;  // (an absent sample's record is not tag-checked)
      stale = stale | (ok & !tag_ok(v.y, part_tag(pl.epoch, qb + sj[t])));
      u[t] = ok ? ukey_of(__uint_as_float(v.x)) : 0xFFFFFFFFu;
    }
    Tu = wave_kth_u32<SV>(u, K2);
    // each list's prefix <= Tu: an 8-ary search over its current prefix (7
    // independent pivot loads per step, so ~3 dependent round trips for 1000
    // entries instead of 10), then the last <= 8 entries at once
    C = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const int j = t * 64 + lane;
      int lo = 0, hi = lens[j];  // entries [0, lo) <= Tu, [hi, n) > Tu
      while (hi - lo > 8) {
        uint32_t pk[7];
        int pv[7];
#pragma unroll
        for (int i = 0; i < 7; i++) {
          pv[i] = lo + (int)(((int64_t)(hi - lo) * (i + 1)) >> 3);
          pk[i] = ukey_of(key_at(j, pv[i]));
        }
        int nlo = lo, nhi = hi;
#pragma unroll
        for (int i = 0; i < 7; i++) nlo = pk[i] <= Tu ? pv[i] + 1 : nlo;
#pragma unroll
        for (int i = 6; i >= 0; i--) nhi = pk[i] > Tu ? pv[i] : nhi;
        lo = nlo;
        hi = nhi;
      }
      // the last <= 8 entries: 8 unconditional loads (clamped into the list's slots;
      // an absent entry's record is neither used nor tag-checked)
      // (lanes j >= L hold no list: their clamped loads read list L - 1's slot 0, inside
      // this query's lists, never past the last query's)
      const int jj = min(j, L - 1);
      uint32_t tail[8];
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const int ii = max(min(lo + i, hi - 1), 0);
        const uint2 v = *reinterpret_cast<const uint2*>(pl.part + (qb + jj) * pl.ks + ii);
        const bool ok = lo + i < hi;
        stale = stale | (ok & !tag_ok(v.y, part_tag(pl.epoch, qb + j)));
        tail[i] = ok ? ukey_of(__uint_as_float(v.x)) : 0xFFFFFFFFu;
      }
      int cnt = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) cnt += (lo + i < hi && tail[i] <= Tu) ? 1 : 0;
      lo += cnt;
      lens[j] = lo;
      C += lo;
    }
    C = wave_sum_i(C);
    __builtin_amdgcn_wave_barrier();
  }
  if (C > kBigCap) return;  // ties overflow: the full merge of k_merge_probes takes this query
  // compact the prefixes (offsets in j order)
  {
    int carry = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const int j = t * 64 + lane;
      const int c = lens[j];
      const int incl = wave_incl_scan(c, lane);
      sp[j] = carry + incl - c;
      carry += __builtin_amdgcn_readlane(incl, 63);
    }
    __builtin_amdgcn_wave_barrier();
    // lane-parallel over the flat candidate index: one coalesced pass per 64
    for (int e0 = 0; e0 < C; e0 += 64) {
      const int e = e0 + lane;
      if (e < C) {
        int lo = 0, hi = 256;
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (sp[mid] <= e) lo = mid; else hi = mid;
        }
        const uint4 r = pl.part[(qb + lo) * pl.ks + (e - sp[lo])];
        stale = stale | !tag_ok(r.y, part_tag(pl.epoch, qb + lo));
        cd[e] = rec_key(r);
        cl[e] = rec_pos(r);
      }
    }
  }
  if (__builtin_amdgcn_ballot_w64(stale)) {  // (uniform) counted here; k_merge_probes repairs (qdone 2)
    if (lane == 0) {
      atomicAdd(pl.hdr + kHdrStale, 1);
      pl.qdone[q] = 2;
    }
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // the exact k-th key: keep the k best and their ties (in place, order kept)
  if (C > k && !exact) {
    const int nt = (C + 63) >> 6;  // wave-uniform: rows of the buffer in use
    uint32_t u2[kBigCap / 64];
#pragma unroll
    for (int t = 0; t < kBigCap / 64; t++) {
      const int e = t * 64 + lane;
      u2[t] = (t < nt && e < C) ? ukey_of(cd[e]) : 0xFFFFFFFFu;
    }
    uint32_t lo = 0, hi = 0xFFFFFFFEu;
    while (lo < hi) {
      const uint32_t mid = lo + ((hi - lo) >> 1);
      int cnt = 0;
#pragma unroll
      for (int t = 0; t < kBigCap / 64; t++)
        if (t < nt) cnt += __popcll(__builtin_amdgcn_ballot_w64(u2[t] <= mid));
      if (cnt >= k) hi = mid; else lo = mid + 1;
    }
    const uint32_t T2 = lo;
    int n2 = 0;
#pragma unroll
    for (int t = 0; t < kBigCap / 64; t++) {
      const int e = t * 64 + lane;
      const bool keep = t < nt && e < C && u2[t] <= T2;
      const uint64_t mk = __builtin_amdgcn_ballot_w64(keep);
      if (mk) {  // wave-uniform
        const float dv = cd[e < C ? e : 0];
        const int64_t pv = cl[e < C ? e : 0];
        __builtin_amdgcn_wave_barrier();
        if (keep) {
          const int at = n2 + __popcll(mk & ((1ull << lane) - 1));
          cd[at] = dv;
          cl[at] = pv;
        }
        n2 += __popcll(mk);
      }
    }
    C = n2;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // labels, and padding up to the sort size P (a power of two)
  int P = 64;
  while (P < C) P <<= 1;
  for (int e = lane; e < P; e += 64) {
    if (e < C) {
      const int64_t pos = cl[e];
      cl[e] = pos_ok(a, pl, pos) ? a.ids[pos] : kSentinelId;
    } else {
      cd[e] = kInf;
      cl[e] = kSentinelId;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // bitonic sort of P entries by (key, label), ascending
  for (int sz = 2; sz <= P; sz <<= 1) {
    for (int st = sz >> 1; st > 0; st >>= 1) {
      for (int p0 = 0; p0 < P / 2; p0 += 64) {
        const int pi = p0 + lane;  // compare pair index
        const int i = ((pi / st) * 2 * st) + (pi % st);
        const int j = i + st;
        const bool up = (i & sz) == 0;
        const float di = cd[i], dj = cd[j];
        const int64_t li = cl[i], lj = cl[j];
        const bool sw = lexless(dj, lj, di, li) == up;  // pairs of a stage are disjoint
        if (sw) {
          cd[i] = dj;
          cl[i] = lj;
          cd[j] = di;
          cl[j] = li;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  for (int e = lane; e < k; e += 64) {
    const bool empty = e >= C;
    a.outD[q * k + e] = empty ? pad : sgn * cd[e];
    a.outI[q * k + e] = empty ? -1 : cl[e];
  }
  if (lane == 0) pl.qdone[q] = 1;
}

// ------------------------------------------- probe merge, k > 64, small L k
// One 256-thread workgroup per query when its L = 4 nprobe partial lists hold
// at most kRadixU x 256 entries (C2 at k = 100: 6400).  Every key is loaded with
// one coalesced pass (the lists are contiguous: entry (j, i) at (qb + j) k + i)
// into registers; the exact k-th smallest key T comes from a 4-pass MSB-first
// radix select (8-bit digits, LDS histogram, equal digits of a wave counted by
// one ballot); the entries <= T (the k best and every tie at T) are compacted,
// labelled and sorted by (key, label).  No dependent global round trips beyond
// the key load, the positions and the labels (k_merge_big: about a dozen).
// Queries whose ties overflow kRadixCap are left to k_merge_probes' full merge.
constexpr int kRadixU = 32;
constexpr int kRadixCap = 512;

__global__ __launch_bounds__(256) void k_merge_radix(ScanArgs a, ListPlan pl) {
  __shared__ int s_len[256];
  __shared__ int s_hist[256];
  __shared__ int s_wsum[4];
  __shared__ int s_sel[3];
  __shared__ int s_n;
  __shared__ float cd[kRadixCap];
  __shared__ int64_t cl[kRadixCap];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t q = blockIdx.x;
  const int k = a.k, np = a.nprobe, L = 4 * np;
  const uint64_t qm = pl.qmask[q];
  const int64_t qb = q * (int64_t)L;
  const float pad = a.ip ? -FLT_MAX : FLT_MAX;
  const float sgn = a.ip ? -1.f : 1.f;
  const uint64_t lt = (1ull << lane) - 1;
  // every count and record read is tag-checked: a stale one sends the query to
  // k_merge_probes' full merge (which rescans its probe) instead of being used
  bool stale = false;
  {
    int n = 0;
    if (tid < L && ((qm >> (tid >> 2)) & 1)) {
      const uint2 nt = pl.partN[qb + tid];
      n = (int)nt.x;
      if (!tag_ok(nt.y, part_tag(pl.epoch, qb + tid))) {
        stale = true;
        n = 0;
      } else if (n < 0 || n > k) {  // a partial list holds at most k entries
        atomicAdd(pl.err, 1);
        n = 0;
      }
    }
    s_len[tid] = n;
    const int ws = wave_sum_i(n);
    if (lane == 0) s_wsum[wave] = ws;
  }
  __syncthreads();
  const int C = s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
  const int ks = pl.ks;
  const int E = L * ks;
  const float inv_k = 1.0f / (float)ks;
  const uint4* pr = pl.part + qb * ks;
  uint32_t key[kRadixU];
#pragma unroll
  for (int u = 0; u < kRadixU; u++) {
    const int e = u * 256 + tid;
    key[u] = 0xFFFFFFFFu;  // absent (no finite key maps here)
    if (e < E) {
      const int j = div_small(e, ks, inv_k);
      if (e - j * ks < s_len[j]) {
        const uint2 v = *reinterpret_cast<const uint2*>(pr + e);  // (key, tag)
        stale = stale | !tag_ok(v.y, part_tag(pl.epoch, qb + j));
        key[u] = ukey_of(__uint_as_float(v.x));
      }
    }
  }
  if (__syncthreads_or(stale)) {  // counted here; k_merge_probes repairs (qdone 2)
    if (tid == 0) {
      atomicAdd(pl.hdr + kHdrStale, 1);
      pl.qdone[q] = 2;
    }
    return;
  }
  // the k-th smallest present key (all of them when there are at most k)
  uint32_t T = 0xFFFFFFFEu;
  if (C > k) {
    uint32_t prefix = 0;
    int r = k;  // rank of the k-th key among the keys matching the prefix
#pragma unroll 1
    for (int pass = 0; pass < 4; pass++) {
      const int shift = 24 - 8 * pass;
      s_hist[tid] = 0;
      __syncthreads();
#pragma unroll
      for (int u = 0; u < kRadixU; u++) {
        const uint32_t kv = key[u];
        const bool m = u * 256 < E && kv != 0xFFFFFFFFu && (pass == 0 || (kv >> (shift + 8)) == (prefix >> (shift + 8)));
        const int bin = (int)((kv >> shift) & 255u);
        uint64_t act = __builtin_amdgcn_ballot_w64(m);
        // lanes sharing the first active lane's digit: one LDS add for all of them
        // (keys of one query mostly share their high digits); the rest add singly
        if (act) {
          const int l0 = (int)__builtin_ctzll(act);
          const int b0 = __builtin_amdgcn_readlane(bin, l0);
          const uint64_t same = __builtin_amdgcn_ballot_w64(m && bin == b0);
          if (lane == l0) atomicAdd(&s_hist[b0], (int)__popcll(same));
          if (m && bin != b0) atomicAdd(&s_hist[bin], 1);
        }
      }
      __syncthreads();
      const int h = s_hist[tid];
      const int iw = wave_incl_scan(h, lane);
      if (lane == 63) s_wsum[wave] = iw;
      __syncthreads();
      int incl = iw;
      for (int w = 0; w < wave; w++) incl += s_wsum[w];
      if (incl >= r && incl - h < r) {
        s_sel[0] = tid;
        s_sel[1] = r - (incl - h);
        s_sel[2] = h;
      }
      __syncthreads();
      prefix |= (uint32_t)s_sel[0] << shift;
      r = s_sel[1];
      // after 16 bits (when the candidates fit one wave's register sort) or 24 bits (when
      // they fit the candidate buffer): take every key of the selected bucket with the
      // k - r keys below it; the sort below cuts them to the k best
      const int nb = (k - r) + s_sel[2];
      if ((pass == 1 && nb <= 128 && k <= 128) || (pass == 2 && nb <= kRadixCap)) {  // block-uniform
        prefix |= (1u << shift) - 1u;
        break;
      }
      __syncthreads();  // s_wsum / s_sel are rewritten by the next pass
    }
    T = prefix;
  }
  // compact the entries <= T (records re-read whole: positions, and the tags checked again)
  if (tid == 0) s_n = 0;
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kRadixU; u++) {
    const bool c = key[u] <= T;  // (absent keys: 0xFFFFFFFF > T)
    const uint64_t mk = __builtin_amdgcn_ballot_w64(c);
    if (!mk) continue;  // wave-uniform
    int base = 0;
    if (lane == (int)__builtin_ctzll(mk)) base = atomicAdd(&s_n, (int)__popcll(mk));
    base = __builtin_amdgcn_readlane(base, (int)__builtin_ctzll(mk));
    const int at = base + (int)__popcll(mk & lt);
    if (c && at < kRadixCap) {
      const int e = u * 256 + tid;
      const uint4 r = pr[e];
      stale = stale | !tag_ok(r.y, part_tag(pl.epoch, qb + div_small(e, ks, inv_k)));
      cd[at] = rec_key(r);
      cl[at] = rec_pos(r);
    }
  }
  if (__syncthreads_or(stale)) {  // counted here; k_merge_probes repairs (qdone 2)
    if (tid == 0) {
      atomicAdd(pl.hdr + kHdrStale, 1);
      pl.qdone[q] = 2;
    }
    return;
  }
  const int n = s_n;
  if (n > kRadixCap) return;  // ties overflow: the full merge of k_merge_probes takes this query
  int P = 64;
  while (P < n) P <<= 1;
  for (int e = tid; e < P; e += 256) {
    if (e < n) {
      const int64_t pos = cl[e];
      cl[e] = pos_ok(a, pl, pos) ? a.ids[pos] : kSentinelId;
    } else {
      cd[e] = kInf;
      cl[e] = kSentinelId;
    }
  }
  __syncthreads();
  if (n <= 128 && k <= 128) {  // one wave sorts the candidates in registers (two 64-lane rows), no barriers
    if (wave == 0) {
      float d0 = lane < n ? cd[lane] : kInf, d1 = lane + 64 < n ? cd[lane + 64] : kInf;
      int64_t i0 = lane < n ? cl[lane] : kSentinelId, i1 = lane + 64 < n ? cl[lane + 64] : kSentinelId;
      bitonic_sort64<2>(d0, i0, lane);
      bitonic_sort64<2>(d1, i1, lane);
      const float rd = rev64_f(d1);
      const int64_t ri = id_rev64(i1);
      const bool t = lexless(rd, ri, d0, i0);
      float lo = t ? rd : d0, hi = t ? d0 : rd;
      int64_t li = t ? ri : i0, hi_i = t ? i0 : ri;
      bitonic_steps<128, 32>(lo, li, lane);  // the 64 smallest, ascending
      bitonic_steps<128, 32>(hi, hi_i, lane);
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int e = h * 64 + lane;
        if (e < k) {
          const bool empty = e >= n;
          const float dv = h ? hi : lo;
          const int64_t iv = h ? hi_i : li;
          a.outD[q * k + e] = empty ? pad : sgn * dv;
          a.outI[q * k + e] = empty ? -1 : iv;
        }
      }
      if (lane == 0) pl.qdone[q] = 1;
    }
    return;
  }
  // bitonic sort of P entries by (key, label), ascending
  for (int sz = 2; sz <= P; sz <<= 1) {
    for (int st = sz >> 1; st > 0; st >>= 1) {
      for (int p0 = 0; p0 < P / 2; p0 += 256) {
        const int pi2 = p0 + tid;
        if (pi2 < P / 2) {
          const int i = ((pi2 / st) * 2 * st) + (pi2 % st);
          const int j = i + st;
          const bool up = (i & sz) == 0;
          const float di = cd[i], dj = cd[j];
          const int64_t li = cl[i], lj = cl[j];
          if (lexless(dj, lj, di, li) == up) {
            cd[i] = dj;
            cl[i] = lj;
            cd[j] = di;
            cl[j] = li;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int e = tid; e < k; e += 256) {
    const bool empty = e >= n;
    a.outD[q * k + e] = empty ? pad : sgn * cd[e];
    a.outI[q * k + e] = empty ? -1 : cl[e];
  }
  if (tid == 0) pl.qdone[q] = 1;
}

// ------------------------------------------------------------ shard merge
__global__ __launch_bounds__(256) void k_merge_topk(int S, int64_t n, int k, const float* __restrict__ Din,
                                                    const int64_t* __restrict__ Iin, float* __restrict__ Dout,
                                                    int64_t* __restrict__ Iout, int ip) {
  // the query's S x k entries staged in LDS when they fit (N = 8, k = 10: 80), so the
  // (S - 1) binary searches of every entry are LDS reads, not dependent global loads
  constexpr int kStage = 2048;
  __shared__ float s_d[kStage];
  __shared__ int64_t s_i[kStage];
  const int64_t q = blockIdx.x;
  const float sgn = ip ? -1.f : 1.f;
  const bool staged = S * k <= kStage;
  auto gkey_d = [&](int s, int j) { return sgn * Din[((int64_t)s * n + q) * k + j]; };
  auto gkey_i = [&](int s, int j) {
    const int64_t v = Iin[((int64_t)s * n + q) * k + j];
    return v < 0 ? kSentinelId : v;
  };
  if (staged) {
    for (int e = threadIdx.x; e < S * k; e += 256) {
      const int s = e / k;
      s_d[e] = gkey_d(s, e - s * k);
      s_i[e] = gkey_i(s, e - s * k);
    }
    __syncthreads();
  }
  auto key_d = [&](int s, int j) { return staged ? s_d[s * k + j] : gkey_d(s, j); };
  auto key_i = [&](int s, int j) { return staged ? s_i[s * k + j] : gkey_i(s, j); };
  for (int e = threadIdx.x; e < S * k; e += 256) {
    const int s = e / k;
    const int idx = e - s * k;
    const float vd = key_d(s, idx);
    const int64_t vi = key_i(s, idx);
    int rank = idx;
    for (int s2 = 0; s2 < S; s2++) {
      if (s2 == s) continue;
      int lo = 0, hi = k;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const float ed = key_d(s2, mid);
        const int64_t ei = key_i(s2, mid);
        const bool before = (s2 < s) ? !lexless(vd, vi, ed, ei) : lexless(ed, ei, vd, vi);
        if (before)
          lo = mid + 1;
        else
          hi = mid;
      }
      rank += lo;
    }
    if (rank < k) {
      const bool empty = vi == kSentinelId;
      Dout[q * k + rank] = empty ? (ip ? -FLT_MAX : FLT_MAX) : sgn * vd;
      Iout[q * k + rank] = empty ? -1 : vi;
    }
  }
}

inline unsigned nblocks(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

inline int rows_for(int k) { return k <= 64 ? 1 : k <= 128 ? 2 : k <= 256 ? 4 : k <= 512 ? 8 : 16; }


}  // namespace

void launch_row_norms(const float* x, int64_t n, int d, float* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_row_norms, dim3(nblocks(n, 8)), dim3(64), 0, s, x, n, d, out);
}

void launch_l2_dist(const float* x, const float* xn, int64_t nx, const float* c, const float* cn, int nc, int d,
                    float* out, hipStream_t s, bool ip) {
  if (nx <= 0 || nc <= 0) return;
  dim3 grid(nblocks(nc, DT_B), nblocks(nx, DT_B));
  hipLaunchKernelGGL(k_l2_dist, grid, dim3(256), 0, s, x, xn, nx, c, cn, nc, d, out, ip ? 1 : 0);
}

void launch_select_rows(const float* dist, int64_t nrows, int ncols, int n, float* ov, int64_t* oc,
                        hipStream_t s, bool neg) {
  if (nrows <= 0) return;
  const dim3 grid(nblocks(nrows, 4));
  const int ng = neg ? 1 : 0;
  switch (rows_for(n)) {
    case 1: hipLaunchKernelGGL(k_select_rows<1>, grid, dim3(256), 0, s, dist, nrows, ncols, n, ov, oc, ng); break;
    case 2: hipLaunchKernelGGL(k_select_rows<2>, grid, dim3(256), 0, s, dist, nrows, ncols, n, ov, oc, ng); break;
    case 4: hipLaunchKernelGGL(k_select_rows<4>, grid, dim3(256), 0, s, dist, nrows, ncols, n, ov, oc, ng); break;
    case 8: hipLaunchKernelGGL(k_select_rows<8>, grid, dim3(256), 0, s, dist, nrows, ncols, n, ov, oc, ng); break;
    default: hipLaunchKernelGGL(k_select_rows<16>, grid, dim3(256), 0, s, dist, nrows, ncols, n, ov, oc, ng); break;
  }
}

bool coarse_tiled_ok(int d, int64_t nq) { return d % 4 == 0 && d >= 256 && nq >= 64; }

void launch_coarse_keys(const float* x, int64_t nq, int d, const float* centT, const float* cn, int nlist,
                        float* keys, hipStream_t s, bool ip, float* T3out, const float* cb, int M, float* xn_buf,
                        const float* xt, int64_t nt, bool hoist) {
  if (nq <= 0) return;
#ifdef COARSE_NO_HOIST  // A/B switch (r06)
  hoist = false;
#endif
  if (!xt) {  // T3 of the key tiles' own queries
    xt = x;
    nt = nq;
  }
  if (xn_buf && coarse_tiled_ok(d, nq)) {  // large d: 64-query x 128-centroid tiles, k-chunks staged in LDS
    if (!ip) launch_row_norms(x, nq, d, xn_buf, s);
    const int ngemm = (int)(nblocks(nq, TQ) * nblocks(nlist, TC));
    // T3 in its own launch: as extra workgroups of this kernel each would hold the
    // GEMM's 54 KB of static LDS, two per CU (C3: 4 096 T3 workgroups, ~0.13 ms)
    if (T3out) launch_ip_table(xt, nt, d, cb, M, 256, T3out, s);
    hipLaunchKernelGGL(k_coarse_gemm_tiled, dim3((unsigned)ngemm), dim3(256), 0, s, x, xn_buf, nq, d, centT,
                       (nlist + 3) & ~3, cn, nlist, keys, ip ? 1 : 0, ngemm, CoarseT3{});
    return;
  }
  const unsigned nqb = nblocks(nq, GQ);
  const int ngemm = (int)(nqb * nblocks(nlist, GC));
  CoarseT3 t3;
  if (T3out && M > 0 && d % M == 0 && nt > 0) {
    t3.out = T3out;
    t3.cb = cb;
    t3.M = M;
    t3.nblk = (int)(nblocks(nt, GQ) * (unsigned)M);
    t3.x = xt;
    t3.nq = nt;
  }
  const size_t smem = sizeof(float) * std::max<size_t>((size_t)GQ * ((d + 63) & ~63) + GQ * 9, (size_t)GQ * d);
  if (smem > 64 * 1024) {  // dynamic LDS above 64 KiB is opted into per device
    static uint64_t attr_done = 0;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 64 && !(attr_done & (1ull << dev))) {
      (void)hipFuncSetAttribute((const void*)k_coarse_gemm<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)k_coarse_gemm<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr_done |= 1ull << dev;
    }
  }
  if (hoist)
    hipLaunchKernelGGL(k_coarse_gemm<1>, dim3((unsigned)(ngemm + t3.nblk)), dim3(256), smem, s, x, nq, d, centT,
                       (nlist + 3) & ~3, cn, nlist, keys, ip ? 1 : 0, ngemm, t3);
  else
    hipLaunchKernelGGL(k_coarse_gemm<0>, dim3((unsigned)(ngemm + t3.nblk)), dim3(256), smem, s, x, nq, d, centT,
                       (nlist + 3) & ~3, cn, nlist, keys, ip ? 1 : 0, ngemm, t3);
}

int coarse_segments(int64_t nq, int nlist, int d) {
  const int64_t qt = (nq + GQ - 1) / GQ;
  const int tiles = (nlist + GC - 1) / GC;
  const int64_t min_wg = 1024;  // four k_coarse_segtop workgroups per CU
  const int want = (int)std::max<int64_t>(1, std::min<int64_t>(tiles, (min_wg + qt - 1) / qt));
  const int seg = (tiles + want - 1) / want * GC;
  return (nlist + seg - 1) / seg;
}

void launch_coarse_segmented(const float* x, int64_t nq, int d, const float* centT, const float* cn, int nlist,
                             int nprobe, uint64_t* cand, float* out_dis, int64_t* out_list, hipStream_t s, bool ip,
                             const ListPlan* plan, const int64_t* list_off, int lo, int hi, const float* cent) {
  if (nq <= 0) return;
  const int nseg = coarse_segments(nq, nlist, d);
  const int tiles = (nlist + GC - 1) / GC;
  const int seg = (tiles + nseg - 1) / nseg * GC;
  const int dk = (d + 63) & ~63;
  const size_t smem = sizeof(float) * ((size_t)dk * GQ + GQ + GQ * 8 + GQ * GC) + sizeof(uint64_t) * GQ * kSegQ;
  if (smem > 64 * 1024) {  // dynamic LDS above 64 KiB is opted into per device
    static uint64_t attr_done = 0;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 64 && !(attr_done & (1ull << dev))) {
      (void)hipFuncSetAttribute((const void*)k_coarse_segtop, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr_done |= 1ull << dev;
    }
  }
  const unsigned grid = (unsigned)(nblocks(nq, GQ) * (unsigned)nseg);
  hipLaunchKernelGGL(k_coarse_segtop, dim3(grid), dim3(256), smem, s, x, nq, d, centT, (nlist + 3) & ~3, cn, nlist,
                     ip ? 1 : 0, seg, nseg, nprobe, cand);
  CoarsePlan cp;
  if (plan) {
    cp.pl = *plan;
    cp.on = 1;
    cp.list_off = list_off;
    cp.lo = lo;
    cp.hi = hi;
    cp.cent = cent;
  }
if (ip)
      hipLaunchKernelGGL(k_coarse_select_cand<1>, dim3(nblocks(nq, 4)), dim3(256), 0, s, cand, nq, nseg, nprobe, out_dis,
                     out_list, x, d, cp);
  else
      hipLaunchKernelGGL(k_coarse_select_cand<0>, dim3(nblocks(nq, 4)), dim3(256), 0, s, cand, nq, nseg, nprobe, out_dis,
                     out_list, x, d, cp);
}

void launch_coarse_select(const float* keys, int64_t nq, int nlist, int nprobe, float* out_dis, int64_t* out_list,
                          hipStream_t s, bool ip, const ListPlan* plan, const int64_t* list_off, int lo, int hi,
                          const float* x, const float* cent, int d) {
  if (nq <= 0) return;
  CoarsePlan cp;
  if (plan) {
    cp.pl = *plan;
    cp.on = 1;
    cp.list_off = list_off;
    cp.lo = lo;
    cp.hi = hi;
    cp.cent = cent;
  }
  if (ip)
    hipLaunchKernelGGL(k_coarse_select<1>, dim3(nblocks(nq, 4)), dim3(256), 0, s, keys, nq, nlist, nprobe, out_dis,
                       out_list, x, d, cp);
  else
    hipLaunchKernelGGL(k_coarse_select<0>, dim3(nblocks(nq, 4)), dim3(256), 0, s, keys, nq, nlist, nprobe, out_dis,
                       out_list, x, d, cp);
}

void launch_linear_transform(const float* x, int64_t n, int d_in, const float* AT, const float* b, int d_out, float* y,
                             hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_linear_transform, dim3(nblocks(n * d_out, 256)), dim3(256), 0, s, x, n, d_in, AT, b, d_out, y);
}

void launch_ip_table(const float* x, int64_t n, int d, const float* cb, int M, int ksub, float* out,
                     hipStream_t s) {
  if (n <= 0) return;
  const int dsub = d / M;
  const dim3 grid((unsigned)n);
  if (d > 2048 || (M * ksub) % 16 != 0) return;  // guarded by the host (d <= 2048, ksub = 256)
  if (ksub == 256 && n >= GQ) {  // (16 queries, m) tiles: the codebook read once per 16 queries
    const dim3 tg((unsigned)(nblocks(n, GQ) * (unsigned)M));
    switch (dsub) {
      case 2: hipLaunchKernelGGL(k_ip_tiles<2>, tg, dim3(256), 0, s, x, n, d, cb, M, out); return;
      case 4: hipLaunchKernelGGL(k_ip_tiles<4>, tg, dim3(256), 0, s, x, n, d, cb, M, out); return;
      case 8: hipLaunchKernelGGL(k_ip_tiles<8>, tg, dim3(256), 0, s, x, n, d, cb, M, out); return;
      case 12: hipLaunchKernelGGL(k_ip_tiles<12>, tg, dim3(256), 0, s, x, n, d, cb, M, out); return;
      case 16: hipLaunchKernelGGL(k_ip_tiles<16>, tg, dim3(256), 0, s, x, n, d, cb, M, out); return;
      default: break;
    }
  }
  switch (dsub) {
    case 2: hipLaunchKernelGGL(k_ip_table<2>, grid, dim3(256), 0, s, x, n, d, cb, M, ksub, out); break;
    case 4: hipLaunchKernelGGL(k_ip_table<4>, grid, dim3(256), 0, s, x, n, d, cb, M, ksub, out); break;
    case 8: hipLaunchKernelGGL(k_ip_table<8>, grid, dim3(256), 0, s, x, n, d, cb, M, ksub, out); break;
    case 12: hipLaunchKernelGGL(k_ip_table<12>, grid, dim3(256), 0, s, x, n, d, cb, M, ksub, out); break;
    case 16: hipLaunchKernelGGL(k_ip_table<16>, grid, dim3(256), 0, s, x, n, d, cb, M, ksub, out); break;
    default: hipLaunchKernelGGL(k_ip_table<0>, grid, dim3(256), 0, s, x, n, d, cb, M, ksub, out); break;
  }
}

void launch_precompute_T1(const float* cent, int nlist, int d, const float* cb, int M, int ksub, float* T1,
                          hipStream_t s) {
  hipLaunchKernelGGL(k_precompute_T1, dim3(nblocks((int64_t)nlist * M * ksub, 256)), dim3(256), 0, s, cent, nlist,
                     d, cb, M, ksub, T1);
}

void launch_pq_encode(const float* x, int64_t n, int d, const float* cent, const int64_t* list_no,
                      const float* cb, int M, int ksub, uint8_t* codes, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pq_encode, dim3(nblocks(n * M, 256)), dim3(256), 0, s, x, n, d, cent, list_no, cb, M, ksub,
                     codes);
}

void launch_plan_count(const int64_t* lists, const float* Dq, const float* x, const float* cent, int64_t nq, int d,
                       int nprobe, const int64_t* list_off, int lo, int hi, bool ip, bool dedup, int k,
                       const ListPlan& pl, hipStream_t s) {
  if (nq <= 0) return;
  hipLaunchKernelGGL(k_plan_count, dim3(nblocks(nq, 4)), dim3(256), 0, s, lists, Dq, x, cent, nq, d, nprobe,
                     list_off, lo, hi, ip ? 1 : 0, dedup ? 1 : 0, k, pl);
}

bool scan_fused_plan(int nloc, int max_items, int M) {
  return nloc <= kFusedPlanLists && max_items < 65536 && M > 0;
}

void launch_plan_items(const ListPlan& pl, const int64_t* list_off, int lo, int hi, int G, hipStream_t s) {
  if (pl.fused) return;  // the list scan plans its own items
  const int nloc = hi - lo;
  if (nloc <= kPlanSmall)
    hipLaunchKernelGGL(k_plan_items_small, dim3(std::max(1u, nblocks(pl.max_items, PLAN_T))), dim3(PLAN_T), 0, s, pl,
                       list_off, lo, nloc, G);
  else
    hipLaunchKernelGGL(k_plan_items_big, dim3(std::max(1u, nblocks(nloc, PLAN_T))), dim3(PLAN_T), 0, s, pl, list_off,
                       lo, nloc, G);
}

bool scan_supported_M(int M) { return M == 8 || M == 16 || M == 32 || M == 48 || M == 64; }
// Pairs per work item: G LUTs of M x 256 floats interleaved in LDS (<= 64 KB),
// G x R <= 8 (the per-wave top-k state).  For k > 64 at M <= 16, G = 2 and three
// workgroups per CU beat G = 4 with two (k = 100 at C2: 174 vs 225 us, r02 A/B;
// r03 on the 200k-centre data: 4.08 vs 3.38 M queries/s).
constexpr int scan_group(int M, int R) {
  return (M * 1024 * 4 <= 65536 && 4 * R <= 8 && !(R >= 2 && M <= 16)) ? 4
         : (M * 1024 * 2 <= 65536 && 2 * R <= 8)                      ? 2
                                                                      : 1;
}
int list_scan_group(int M, int k) {
  const int R = rows_for(k);
  switch (R) {
    case 1: return scan_group(M, 1);
    case 2: return scan_group(M, 2);
    case 4: return scan_group(M, 4);
    case 8: return scan_group(M, 8);
    default: return scan_group(M, 16);
  }
}

int list_scan_max_items(int64_t npairs, int nloc, int G) {
  // sum over (list, kind) buckets of ceil(c / G) <= npairs / G + (non-empty buckets)
  const int64_t v = (npairs + G - 1) / G + std::min<int64_t>(2 * (int64_t)nloc, npairs) + 8;
  return (int)v;
}

int scan_lists_grid(int M, int k, int free_cus) {
  static int cus = 0;
  if (!cus) {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    cus = n;
  }
  // workgroups per CU the LDS allows (LUTs, candidate queues, fused-plan prefix), at most 3
  const int lds = M * 256 * 4 * list_scan_group(M, k) + 4 * QCAP * 8 + 6 * kFusedPlanLists + 96;
  const int per_cu = std::max(1, std::min(3, 160 * 1024 / lds));
#ifdef SCAN_GRID_QUARTERS  // (A/B builds: workgroups per CU in quarters, e.g. 7 = 1.75 per CU)
  if (per_cu == 2) return std::max(8, (SCAN_GRID_QUARTERS * cus / 4 + 7) / 8 * 8);
#endif
  // free_cus: the persistent scan is sized for that many CUs fewer, so kernels of other
  // streams (the next batch's coarse step and merge, RCCL's collectives in the shard
  // flow) find room while a scan runs instead of waiting for its tail.  Performance
  // only; IVFPQ_SCAN_FREE_CUS overrides it (A/B runs)
  static int env_free = -2;
  if (env_free == -2) {
    const char* e = getenv("IVFPQ_SCAN_FREE_CUS");
    env_free = e ? std::max(0, atoi(e)) : -1;
  }
  if (env_free >= 0) free_cus = env_free;
  free_cus = std::max(0, std::min(free_cus, cus / 2));
  return std::max(8, (per_cu * (cus - free_cus) + 7) / 8 * 8);
}

int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    cus = n;
  }
  return cus;
}

template <int M, int R>
static void launch_lists_MR(const ScanArgs& a, const ListPlan& pl, hipStream_t s, hipEvent_t* ev) {
  constexpr int G = scan_group(M, R);
  // code chunks held in registers per item (32 VGPRs), even; r02 A/B at C2 M = 16:
  // 6 -> 111.8 us, 8 -> 114.3, 4 -> 113.9
  // (M > 32: 4 chunks, r04 A/B vs 2: C3 scan 643 -> 624 us, C4 214 -> 210 us)
  constexpr int JB = M <= 16 ? 6 : 4;
  if (ev) (void)hipEventRecord(ev[0], s);
  if constexpr (G == 4 && R == 1) {
    if (a.k <= 16 && pl.fused && kScanLean && M <= 16) {  // (row-packed top-k, insertion instead of a queue)
      hipLaunchKernelGGL((k_scan_lean<M, kLeanJB>), dim3((unsigned)pl.grid), dim3(256), 0, s, a, pl);
    } else if (a.k <= 16) {  // r03 A/B at C2: 115.1 vs 125.7 us
      hipLaunchKernelGGL((k_scan_lists<M, G, R, JB, true>), dim3((unsigned)pl.grid), dim3(256), 0, s, a, pl);
    } else {
      hipLaunchKernelGGL((k_scan_lists<M, G, R, JB>), dim3((unsigned)pl.grid), dim3(256), 0, s, a, pl);
    }
  } else {
    hipLaunchKernelGGL((k_scan_lists<M, G, R, JB>), dim3((unsigned)pl.grid), dim3(256), 0, s, a, pl);
  }
  if (ev) (void)hipEventRecord(ev[1], s);
  if (R >= 2 && a.nprobe <= 64) {
    if (4 * a.nprobe * pl.ks <= kRadixU * 256)  // every key of a query in one workgroup's registers
      hipLaunchKernelGGL(k_merge_radix, dim3((unsigned)a.nq), dim3(256), 0, s, a, pl);
    else
      hipLaunchKernelGGL(k_merge_big, dim3((unsigned)a.nq), dim3(64), 0, s, a, pl);
  }
  hipLaunchKernelGGL(k_merge_probes<R>, dim3(nblocks(a.nq, 4)), dim3(256), 0, s, a, pl);
#ifdef DIAG_TWICE  // (diagnostic builds: the same merge again, warm; idempotent for k <= 64)
  if (R == 1) hipLaunchKernelGGL(k_merge_probes<R>, dim3(nblocks(a.nq, 4)), dim3(256), 0, s, a, pl);
#endif
}

template <int M>
static void launch_lists_M(const ScanArgs& a, const ListPlan& pl, hipStream_t s, hipEvent_t* ev) {
  switch (rows_for(a.k)) {
    case 1: launch_lists_MR<M, 1>(a, pl, s, ev); break;
    case 2: launch_lists_MR<M, 2>(a, pl, s, ev); break;
    case 4: launch_lists_MR<M, 4>(a, pl, s, ev); break;
    case 8: launch_lists_MR<M, 8>(a, pl, s, ev); break;
    default: launch_lists_MR<M, 16>(a, pl, s, ev); break;
  }
}

void launch_scan_lists(const ScanArgs& a, const ListPlan& pl, hipStream_t s, hipEvent_t* ev_lists) {
  if (a.nq <= 0) return;
  switch (a.M) {
    case 8: launch_lists_M<8>(a, pl, s, ev_lists); break;
    case 16: launch_lists_M<16>(a, pl, s, ev_lists); break;
    case 32: launch_lists_M<32>(a, pl, s, ev_lists); break;
    case 48: launch_lists_M<48>(a, pl, s, ev_lists); break;
    case 64: launch_lists_M<64>(a, pl, s, ev_lists); break;
    default: break;
  }
}

void launch_merge_topk(int S, int64_t n, int k, const float* Din, const int64_t* Iin, float* Dout, int64_t* Iout,
                       hipStream_t s, bool ip) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_merge_topk, dim3((unsigned)n), dim3(256), 0, s, S, n, k, Din, Iin, Dout, Iout, ip ? 1 : 0);
}

}  // namespace chivf

#if defined(DIAG_STAMPS) || defined(DIAG_CSTAMPS)
extern "C" int ivfpq_diag_stamps(void* out, size_t bytes) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(chivf::g_diag), bytes) != hipSuccess) return -1;
  static uint64_t zeros[chivf::kDiagWG * chivf::kDiagItems * chivf::kDiagSlots];
  return hipMemcpyToSymbol(HIP_SYMBOL(chivf::g_diag), zeros, sizeof(zeros)) == hipSuccess ? 0 : -1;
}
#endif
