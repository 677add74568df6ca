// Launchers for the gfx950 IVF-PQ kernels (ivfpq_kernels.hip).
// All launchers are asynchronous on `stream` and allocate nothing.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace chivf {

constexpr int kMaxK = 1024;       // largest k / nprobe served by the fused wave top-k
constexpr int64_t kSentinelId = INT64_MAX;

// out[i] = |x_i|^2 in Faiss AVX order (fvec_norm_L2sqr)
void launch_row_norms(const float* x, int64_t n, int d, float* out, hipStream_t s);

// out[i][j] = max(0, (xn[i] + cn[j]) - 2 * <x_i, c_j>), <.,.> = k-ordered fmaf chain
void launch_l2_dist(const float* x, const float* xn, int64_t nx, const float* c, const float* cn, int nc, int d,
                    float* out, hipStream_t s);

// per row: the n smallest (value, column) pairs, ascending lexicographic.
void launch_select_rows(const float* dist, int64_t nrows, int ncols, int n, float* out_val, int64_t* out_col,
                        hipStream_t s);

// T3[q][m][j] = <x_q[m], C_mj>  (Faiss AVX order)
void launch_ip_table(const float* x, int64_t n, int d, const float* codebook, int M, int ksub, float* out,
                     hipStream_t s);

// T1[l][m][j] = |C_mj|^2 + 2 <c_l[m], C_mj>
void launch_precompute_T1(const float* cent, int nlist, int d, const float* codebook, int M, int ksub, float* T1,
                          hipStream_t s);

// codes[i][m] = first argmin_j |(x_i - c_{list_i})[m] - C_mj|^2
void launch_pq_encode(const float* x, int64_t n, int d, const float* cent, const int64_t* list_no,
                      const float* codebook, int M, int ksub, uint8_t* codes, hipStream_t s);

// Fused LUT-in-LDS + PQ-code scan + per-query top-k.
struct ScanArgs {
  const float* T1;          // [nlist][M][ksub]
  const float* T3;          // [nq][M][ksub]
  const uint8_t* codes;     // [n_codes][M], lists concatenated
  const int64_t* ids;       // [n_codes]
  const int64_t* list_off;  // [nlist + 1]
  const int64_t* probe_list;  // [nq][nprobe]
  const float* probe_dis0;    // [nq][nprobe] or null (zeros)
  int64_t nq;
  int nprobe;
  int k;
  int M;
  int list_lo, list_hi;  // only lists in [list_lo, list_hi) are scanned (shard range)
  float* outD;           // [nq][k]
  int64_t* outI;         // [nq][k]
};
void launch_scan_topk(const ScanArgs& a, hipStream_t s);
bool scan_supported_M(int M);

// merge S sorted partial top-k lists [S][n][k] into [n][k]
void launch_merge_topk(int S, int64_t n, int k, const float* Din, const int64_t* Iin, float* Dout, int64_t* Iout,
                       hipStream_t s);

}  // namespace chivf
