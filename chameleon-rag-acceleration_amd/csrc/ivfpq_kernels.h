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

// Fused coarse quantizer for nlist <= kCoarseFusedMax: per query the distances
// to all centroids (centT = centroids transposed [d][nlist], cn = |c|^2) and
// the nprobe smallest (dis, list) pairs.  Same arithmetic as launch_l2_dist +
// launch_select_rows.
constexpr int kCoarseFusedMax = 8192;
void set_coarse_debug(int v);  // timing ablations of the fused coarse kernel (wrong results)
struct ListPlan;
// plan (nullable): also count the list-major buckets for `plan` (shard range [lo, hi)) in the epilogue;
// sets plan->counted when it does (nprobe <= 64)
void launch_coarse_fused(const float* x, int64_t nq, int d, const float* centT, const float* cn, int nlist,
                         int nprobe, float* out_dis, int64_t* out_list, hipStream_t s, ListPlan* plan = nullptr,
                         const int64_t* list_off = nullptr, int lo = 0, int hi = 0, float* T3out = nullptr,
                         const float* codebook = nullptr, int M = 0);  // T3out: also build T3 (sets plan->t3done)

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
  // threshold-seed mode of the query-major kernel: scan only probe first_probe[q]
  // (skip the query if it is >= nprobe) and write the result to the partial slot
  // partD/partI + (q * nprobe + first_probe[q]) * k.
  const int32_t* first_probe = nullptr;
  float* partD = nullptr;
  int64_t* partI = nullptr;
  int32_t* tauq = nullptr;  // seed mode also publishes each query's k-th distance here
  int debug = 0;            // timing ablations only (wrong results): 1 = no phase-B top-k, 2 = no LUT reads
  uint64_t* stamps = nullptr;  // diagnostic in-kernel s_memtime stamps (phase B), null in production
  // List-major path: the seed launch builds T3 itself (no k_ip_table launch) from
  // the queries and the codebook and stores it to T3out for the list scan.
  const float* xq = nullptr;  // [nq][d]
  const float* cb = nullptr;  // [M][ksub][dsub]
  int d = 0;
  float* T3out = nullptr;     // [nq][M][ksub]; null: T3 is read from T3
  // Seed launch only: scatter pair ids into the list-scan work items (k_bucket_scatter's job)
  const int32_t* scat_slot = nullptr;
  const int32_t* scat_ioff = nullptr;
  int32_t* scat_recs = nullptr;
  int scat_G = 1;
};
constexpr int kStampItems = 32;  // items stamped per phase-B workgroup
constexpr int kStampSlots = 6;   // per item: start, LUT ready, scan done, merge done, n, cnt
void launch_scan_topk(const ScanArgs& a, hipStream_t s);
bool scan_supported_M(int M);

// ---- Two-phase scan ------------------------------------------
// Phase A (query-major k_scan_topk in seed mode): each query's first usable
// probe, giving a per-query bound tau_q = its k-th distance.  Phase B
// (list-major): work item = (inverted list, up to G queries probing it), every
// other probe, admission dis <= tau_q.  A per-query merge combines the partials.
struct ListPlan {
  int32_t* first_probe;  // [nq]
  int32_t* slot;         // [nq * nprobe]
  int32_t* cnt;          // [nloc]  zero between batches (k_bucket_plan re-zeroes after reading)
  int32_t* ioff;         // [nloc]  first work item of each list
  int32_t* recs;         // [cap][16] work item: list, count, size, offset(2), pairs(4), coarse dist(4)
  int32_t* n_items;      // [1]
  float* partD;          // [nq][nprobe][4 waves][k]  per-wave sorted partial top-k
  int64_t* partI;        // same shape: global code positions (-1 = none)
  int32_t* tauq;         // [nq] running k-th distance bound per query (fp32 bits, atomicMin)
  int cap;               // upper bound on the number of work items
  int grid;              // persistent phase-B workgroups (multiple of 8)
  int seed = 1;          // run the threshold-seed pass (0: every probe in phase B)
  int counted = 0;       // first_probe / tauq / slot / cnt already produced by the coarse epilogue
  int t3done = 0;        // T3 already built by the coarse kernel
};
int list_scan_group(int M, int k);  // queries per work item (G) used for (M, k)
// phase-B item-count upper bound for a batch (host side, to size ListPlan)
int list_scan_cap(int64_t nq, int nprobe, int nloc, int G);
// ev_lists (nullable): two events recorded around the phase-B list-scan kernel alone
void launch_scan_lists(const ScanArgs& a, const ListPlan& plan, hipStream_t s, hipEvent_t* ev_lists = nullptr);
int scan_lists_grid();  // persistent grid size for the device (2 workgroups per CU)

// merge S sorted partial top-k lists [S][n][k] into [n][k]
void launch_merge_topk(int S, int64_t n, int k, const float* Din, const int64_t* Iin, float* Dout, int64_t* Iout,
                       hipStream_t s);

}  // namespace chivf
