// Launchers for the gfx950 IVF-PQ kernels (ivfpq_kernels.hip).
// All launchers are asynchronous on `stream` and allocate nothing.
//
// Metric handling: the kernels rank by a KEY that is ascending-better for both
// metrics.  L2: key = distance.  Inner product: key = -similarity, formed by
// negating every LUT entry and dis0 (negation is exact and rounding is
// symmetric, so (-a) + (-b) == -(a + b) bit for bit); results are negated back
// on output.  Ties are broken by label in both cases, i.e. (key, label)
// lexicographic = (distance asc, label) for L2 and (similarity desc, label)
// for IP.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace chivf {

constexpr int kMaxK = 1024;       // largest k / nprobe served by the fused wave top-k
constexpr int64_t kSentinelId = INT64_MAX;

// out[i] = |x_i|^2 in Faiss AVX order (fvec_norm_L2sqr)
void launch_row_norms(const float* x, int64_t n, int d, float* out, hipStream_t s);

// key[i][j] = L2: max(0, (xn[i] + cn[j]) - 2 * <x_i, c_j>);  IP: -<x_i, c_j>
// <.,.> = k-ordered fmaf chain (xn/cn unused for IP)
void launch_l2_dist(const float* x, const float* xn, int64_t nx, const float* c, const float* cn, int nc, int d,
                    float* out, hipStream_t s, bool ip = false);

// per row: the n smallest (key, column) pairs, ascending lexicographic.
// neg: write -key (IP similarities) and pad with -FLT_MAX instead of FLT_MAX.
void launch_select_rows(const float* dist, int64_t nrows, int ncols, int n, float* out_val, int64_t* out_col,
                        hipStream_t s, bool neg = false);

struct ListPlan;

// Coarse quantizer keys on the matrix cores: keys[q][c] (launch_l2_dist's
// arithmetic; centT = centroids transposed [d][(nlist + 3) & ~3], cn = |c|^2).
// With T3out, the same launch builds T3 [nt][M][256] (Faiss tree order) of the
// queries xt (nullable: the key tiles' own x, nq) -- the list-range shard step keys
// its own slice and tabulates the whole global batch in one launch.
// hoist: the key tiles load every centroid row up front (more registers, shorter
// latency: for searches whose scan is not k_scan_lean).
// xn_buf (nullable, [nq] floats of scratch): with d % 4 == 0, d >= 256 and nq >= 64
// (coarse_tiled_ok) the keys come from 64-query x 128-centroid tiles with k-chunks
// staged in LDS (|x|^2 from launch_row_norms into xn_buf), same arithmetic.
bool coarse_tiled_ok(int d, int64_t nq);
void launch_coarse_keys(const float* x, int64_t nq, int d, const float* centT, const float* cn, int nlist,
                        float* keys, hipStream_t s, bool ip, float* T3out = nullptr, const float* cb = nullptr,
                        int M = 0, float* xn_buf = nullptr, const float* xt = nullptr, int64_t nt = 0,
                        bool hoist = false);
// Per query the nprobe (<= 64) smallest (key, list) pairs of a key matrix;
// out_dis receives the quantizer's distances (L2) or similarities (IP).  With
// `plan`, the epilogue also plans the batch (first usable probe, tau reset,
// per-list pair counts, bucket entries with the scan's dis0: L2 the coarse
// distance, IP -<x, c_l> in Faiss tree order over d).
void launch_coarse_select(const float* keys, int64_t nq, int nlist, int nprobe, float* out_dis, int64_t* out_list,
                          hipStream_t s, bool ip, const ListPlan* plan = nullptr, const int64_t* list_off = nullptr,
                          int lo = 0, int hi = 0, const float* x = nullptr, const float* cent = nullptr, int d = 0);

// Large-nlist coarse quantizer without the key matrix: per (16 queries,
// centroid segment) the nprobe (<= 64) best (key, list) words on the matrix
// cores (cand [nq][coarse_segments(nq, nlist)][nprobe]), then per query their
// merge, output and (with plan) the batch planning of launch_coarse_select.
int coarse_segments(int64_t nq, int nlist, int d);
void launch_coarse_segmented(const float* x, int64_t nq, int d, const float* centT, const float* cn, int nlist,
                             int nprobe, uint64_t* cand, float* out_dis, int64_t* out_list, hipStream_t s, bool ip,
                             const ListPlan* plan = nullptr, const int64_t* list_off = nullptr, int lo = 0, int hi = 0,
                             const float* cent = nullptr);

// y[i][j] = sum_t x[i][t] * AT[t][j] (t-ordered fmaf chain) + b[j] (b nullable): OPQ / LinearTransform apply
void launch_linear_transform(const float* x, int64_t n, int d_in, const float* AT, const float* b, int d_out, float* y,
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

// ---- list-major search ------------------------------------------
// A batch's (query, probe) pairs whose list is in the shard range [lo, hi) and
// non-empty are bucketed by list: kind 0 = the query's first usable probe,
// kind 1 = every other probe (cap slots per list and kind; a list holds at most
// one pair per query).  Work items are (list, up to G pairs of one kind); all
// kind-0 items are scheduled before kind-1 items, so each query's running
// k-th key (tau) is usually known when its other probes are scanned.
// Stride of one per-wave partial list in `part`: k records of 16 B.
inline int part_stride(int k) { return k; }

// ListPlan::hdr words owned by the merges (hdr[0..1]: item counts, hdr[2]: the list
// scan's work counter, hdr[15]: the index-check error word)
constexpr int kHdrLog = 12;     // stale-entry events offered to the event log
constexpr int kHdrStale = 13;   // (query, merge launch) pairs that read a stale entry
constexpr int kHdrRepair = 14;  // probes rescanned by k_merge_probes
constexpr int kEvLog = 64;      // events kept in ListPlan::evlog (8 words each)

struct ListPlan {
  int32_t* cnt;      // [2][nloc] pair counts per kind; zero between batches (k_scan_lists re-zeroes)
  int2* bucket;      // [nloc][2 kinds][cap] (pair id q*nprobe+p, dis0 key bits)
  int cap;           // bucket slots per list (>= queries in the batch)
  int32_t* recs;     // [max_items][16] work items: list, count, size, beg(2), pairs[4], dis0[4]
  int32_t* hdr;      // [16]: n_items, n_items of kind 0, the list scan's work counter, 0...
  int max_items;
  // [nq][nprobe][4 waves][k] per-wave sorted partial top-k, one 16-B record per entry:
  // {key bits, tag, global code position lo, hi} (position -1 = none; k <= 64 pads
  // every list to k).  tag = part_tag(epoch, slot) | writer XCD << 28 (ivfpq_kernels.hip)
  uint4* part;
  uint2* partN;      // [nq][nprobe][4] (valid entries, tag) of each partial list (k > 64 writes only those)
  float* pd0;        // [nq][nprobe] the dis0 each planned pair was scanned with (a merge's rescan)
  int32_t* qdone;    // [nq] k > 64: 1 = merged by k_merge_big (k_merge_probes resets it to 0)
  // [nq] running k-th key per query, tagged with the batch: (~epoch) << 32 |
  // order-preserving key bits, lowered by 64-bit atomicMin.  A newer batch's
  // words compare below every older batch's, so no reset store is needed and a
  // word left by an earlier batch reads as "no bound" (tau_get); the buffer is
  // initialised to all-ones.  Read with agent-scope atomic loads.
  uint64_t* tauq;
  uint32_t epoch;    // this batch's tag (>= 1, strictly increasing per workspace)
  int32_t* err;      // [1] index-check violations counted by the merge kernels (0 = none; never reset; = hdr + 15)
  uint64_t* qmask;   // [nq][qmw] probes the scan covers: bit p of word p / 64 = pair (q, p) is scanned
  int qmw = 1;       // 64-bit mask words per query (ceil(nprobe / 64))
  uint32_t* evlog;   // [kEvLog][8] the first stale-entry events (k_merge_probes log_stale)
  int fault = 0;     // test hook (ivfpq_set_fault_injection): > 0 = slots with slot % fault == 1 are not written
  int grid;          // persistent list-scan workgroups (multiple of 8)
  const int32_t* order = nullptr;  // [nloc] item order of the lists within a kind (nullable = list order)
  int fused = 0;     // 1: the list scan derives its items from cnt/bucket (no k_plan_items launch, recs unused)
  int ks = 0;        // partial-list stride in entries (part_stride(k))
};

struct ScanArgs {
  const float* T1;          // [nlist][M][ksub]
  const float* T3;          // [nq][M][ksub]
  const uint8_t* codes;     // [n_codes][M], lists concatenated, each list sorted by label
  const int64_t* ids;       // [n_codes]
  const int64_t* list_off;  // [nlist + 1]
  int64_t n_codes;          // entries in codes / ids (bound of every code position the merges dereference)
  const int64_t* probe_list;  // [nq][nprobe] (-1 = skipped probe)
  int64_t nq;
  int nprobe;
  int k;
  int M;
  int ip;                // 1: inner product (LUT = -T3, output similarity = -key)
  int list_lo, list_hi;  // only lists in [list_lo, list_hi) are scanned (shard range)
  float* outD;           // [nq][k]
  int64_t* outI;         // [nq][k]
};

// Planning for batches whose probes come from elsewhere (search_preassigned,
// the large-nlist coarse path, nprobe > 64): same work as the fused coarse
// epilogue.  dis0: L2 -> Dq (NULL = zeros); IP -> -<x_q, c_l> (Faiss tree
// order over d, computed from x and cent; Dq is not used, as in Faiss).
// dedup (caller-supplied rows): a list id repeated within a query's row is
// scanned once (its later pairs get empty partials; Faiss would scan it twice
// and could return a label twice).
void launch_plan_count(const int64_t* lists, const float* Dq, const float* x, const float* cent, int64_t nq, int d,
                       int nprobe, const int64_t* list_off, int lo, int hi, bool ip, bool dedup, int k,
                       const ListPlan& pl, hipStream_t s);
// item records from the per-list counts (G = list_scan_group(M, k)); nothing to do when pl.fused
void launch_plan_items(const ListPlan& pl, const int64_t* list_off, int lo, int hi, int G, hipStream_t s);
// whether the list scan can plan its own items (nloc lists, at most max_items items, code size M)
bool scan_fused_plan(int nloc, int max_items, int M);

int list_scan_group(int M, int k);  // pairs per work item (G) used for (M, k)
int list_scan_max_items(int64_t npairs, int nloc, int G);
int scan_lists_grid(int M, int k, int free_cus = 0);  // persistent grid (2-3 workgroups per CU by LDS) on all but free_cus CUs
bool scan_supported_M(int M);
// list scan + probe merge; ev_lists (nullable): two events recorded around the list-scan kernel alone
void launch_scan_lists(const ScanArgs& a, const ListPlan& plan, hipStream_t s, hipEvent_t* ev_lists = nullptr);

// merge S sorted partial results [S][n][k] into [n][k]; ip: entries are similarities (descending)
void launch_merge_topk(int S, int64_t n, int k, const float* Din, const int64_t* Iin, float* Dout, int64_t* Iout,
                       hipStream_t s, bool ip = false);

}  // namespace chivf
