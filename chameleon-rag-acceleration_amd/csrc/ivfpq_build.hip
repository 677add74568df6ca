// Device-side inverted-list image build (ivfpq_add_device, and the host add
// path routed through it): the new entries' (list, label, code) arrays are
// merged with the current list-contiguous image into a new image, entirely on
// the GPU.  Faiss appends to per-list vectors on the host
// (InvertedLists::add_entries, Chameleon/Faiss_experiments/bench_gpu_1bn.py:
// 598-658 adds 1e9 vectors in 1e6-vector slices); here a 1e9 / 8 shard
// (125 M codes) is rebuilt in HBM without a host round trip.
//
// Order: stable by (list, label) -- two LSD radix sorts (label, then list),
// rocprim's radix sort being stable -- which is the device image's within-list
// label order.  Entries whose list lies outside the handle's
// range [lo, hi) are dropped (a list-range shard keeps its own lists only).
#include <stdint.h>

#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include "ivfpq_build.h"

namespace chivf {

namespace {

inline unsigned nblk(int64_t n, int t) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }

// list number of every entry of the current image (from its offsets); one workgroup per list
__global__ __launch_bounds__(256) void k_expand_lists(const int64_t* __restrict__ off, int lo, int hi,
                                                      uint32_t* __restrict__ lno) {
  const int l = lo + blockIdx.x;
  if (l >= hi) return;
  for (int64_t i = off[l] + threadIdx.x; i < off[l + 1]; i += 256) lno[i] = (uint32_t)l;
}

// new entries: list numbers (int64, from the coarse assignment) -> sort keys;
// outside [lo, hi) -> nlist (sorted after every kept entry)
__global__ __launch_bounds__(256) void k_new_keys(const int64_t* __restrict__ lists, int64_t n, int lo, int hi,
                                                  int nlist, uint32_t* __restrict__ lno) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t l = lists[i];
  lno[i] = (l >= lo && l < hi) ? (uint32_t)l : (uint32_t)nlist;
}

__global__ __launch_bounds__(256) void k_iota_u32(uint32_t* __restrict__ v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) v[i] = (uint32_t)i;
}

__global__ __launch_bounds__(256) void k_iota_i64(int64_t* __restrict__ v, int64_t n, int64_t start) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) v[i] = start + i;
}

// the labels of all entries (old image then new), in source order
__global__ __launch_bounds__(256) void k_concat_ids(const int64_t* __restrict__ a, int64_t na,
                                                    const int64_t* __restrict__ b, int64_t nb,
                                                    int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < na) out[i] = a[i];
  else if (i < na + nb) out[i] = b[i - na];
}

__global__ __launch_bounds__(256) void k_gather_keys(const uint32_t* __restrict__ lno, const uint32_t* __restrict__ perm,
                                                     int64_t n, uint32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = lno[perm[i]];
}

// off[l] = first sorted position whose list is >= l, for l in [0, nlist]
__global__ __launch_bounds__(256) void k_list_offsets(const uint32_t* __restrict__ sorted, int64_t n, int nlist,
                                                      int64_t* __restrict__ off) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i > n) return;
  const int64_t prev = i == 0 ? -1 : (int64_t)sorted[i - 1];
  const int64_t cur = i == n ? (int64_t)nlist + 1 : (int64_t)sorted[i];
  for (int64_t l = prev + 1; l <= cur && l <= nlist; l++) off[l] = i;
}

// entry i of the new image <- source perm[i] (old image below n_old, new entries above)
__global__ __launch_bounds__(256) void k_gather_entries(const uint32_t* __restrict__ perm, int64_t n, int M,
                                                        const uint8_t* __restrict__ old_codes, int64_t n_old,
                                                        const uint8_t* __restrict__ new_codes,
                                                        const int64_t* __restrict__ ids_all,
                                                        uint8_t* __restrict__ codes, int64_t* __restrict__ ids) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t src = perm[i];
  const uint8_t* s = src < n_old ? old_codes + src * M : new_codes + (src - n_old) * M;
  uint8_t* d = codes + i * M;
  if ((M & 15) == 0) {
    for (int v = 0; v < M / 16; v++) reinterpret_cast<uint4*>(d)[v] = reinterpret_cast<const uint4*>(s)[v];
  } else if ((M & 7) == 0) {
    for (int v = 0; v < M / 8; v++) reinterpret_cast<uint2*>(d)[v] = reinterpret_cast<const uint2*>(s)[v];
  } else {
    for (int v = 0; v < M; v++) d[v] = s[v];
  }
  ids[i] = ids_all[src];
}

int key_bits(int nlist) {
  int b = 1;
  while ((1ll << b) <= (int64_t)nlist) b++;
  return b;
}

}  // namespace

size_t image_merge_scratch_bytes(int64_t n_all, int nlist) {
  // lno (2 x u32), perm (2 x u32), ids_all (i64), sort temp (the larger of the two sorts)
  size_t t1 = 0, t2 = 0;
  (void)rocprim::radix_sort_pairs(nullptr, t1, (const int64_t*)nullptr, (int64_t*)nullptr, (const uint32_t*)nullptr,
                                  (uint32_t*)nullptr, (size_t)n_all, 0, 64);
  (void)rocprim::radix_sort_pairs(nullptr, t2, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)n_all, 0, key_bits(nlist));
  const size_t a = 256;
  auto up = [&](size_t b) { return (b + a - 1) / a * a; };
  return up(4 * n_all) * 4 + up(8 * n_all) * 2 + up(std::max(t1, t2));
}

hipError_t image_merge_sort(const ImageMergeArgs& g, void* scratch, size_t scratch_bytes, hipStream_t s) {
  const int64_t n = g.n_old + g.n_new;
  const size_t al = 256;
  auto up = [&](size_t b) { return (b + al - 1) / al * al; };
  char* p = static_cast<char*>(scratch);
  uint32_t* lno = reinterpret_cast<uint32_t*>(p);
  p += up(4 * n);
  uint32_t* lno2 = reinterpret_cast<uint32_t*>(p);
  p += up(4 * n);
  uint32_t* perm = reinterpret_cast<uint32_t*>(p);
  p += up(4 * n);
  uint32_t* perm2 = reinterpret_cast<uint32_t*>(p);
  p += up(4 * n);
  int64_t* ids_all = reinterpret_cast<int64_t*>(p);
  p += up(8 * n);
  int64_t* ids_sorted = reinterpret_cast<int64_t*>(p);
  p += up(8 * n);
  void* tmp = p;
  size_t tmp_bytes = scratch_bytes - (size_t)(p - static_cast<char*>(scratch));
  if (n <= 0) return hipSuccess;
  // keys: every entry's list (old image: expanded from its offsets; new: assignment)
  if (g.n_old > 0)
    hipLaunchKernelGGL(k_expand_lists, dim3((unsigned)std::max(1, g.hi - g.lo)), dim3(256), 0, s, g.old_off, g.lo,
                       g.hi, lno);
  if (g.n_new > 0)
    hipLaunchKernelGGL(k_new_keys, dim3(nblk(g.n_new, 256)), dim3(256), 0, s, g.new_lists, g.n_new, g.lo, g.hi,
                       g.nlist, lno + g.n_old);
  hipLaunchKernelGGL(k_concat_ids, dim3(nblk(n, 256)), dim3(256), 0, s, g.old_ids, g.n_old, g.new_ids, g.n_new,
                     ids_all);
  hipLaunchKernelGGL(k_iota_u32, dim3(nblk(n, 256)), dim3(256), 0, s, perm, n);
  // 1) by label, 2) by list (stable): (list, label) order
  hipError_t e = rocprim::radix_sort_pairs(tmp, tmp_bytes, ids_all, ids_sorted, perm, perm2, (size_t)n, 0, 64, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_gather_keys, dim3(nblk(n, 256)), dim3(256), 0, s, lno, perm2, n, lno2);
  e = rocprim::radix_sort_pairs(tmp, tmp_bytes, lno2, lno, perm2, perm, (size_t)n, 0, key_bits(g.nlist), s);
  if (e != hipSuccess) return e;
  // lno: sorted lists; perm: source of every sorted position
  hipLaunchKernelGGL(k_list_offsets, dim3(nblk(n + 1, 256)), dim3(256), 0, s, lno, n, g.nlist, g.off_out);
  return hipGetLastError();
}

hipError_t image_merge_gather(const ImageMergeArgs& g, int64_t n_out, void* scratch, hipStream_t s) {
  const int64_t n = g.n_old + g.n_new;
  const size_t al = 256;
  auto up = [&](size_t b) { return (b + al - 1) / al * al; };
  char* p = static_cast<char*>(scratch);
  const uint32_t* perm = reinterpret_cast<const uint32_t*>(p + 2 * up(4 * n));
  const int64_t* ids_all = reinterpret_cast<const int64_t*>(p + 4 * up(4 * n));
  if (n_out > 0)
    hipLaunchKernelGGL(k_gather_entries, dim3(nblk(n_out, 256)), dim3(256), 0, s, perm, n_out, g.M, g.old_codes,
                       g.n_old, g.new_codes, ids_all, g.codes_out, g.ids_out);
  return hipGetLastError();
}

// ---- per-list merge of a sorted new image into the current one ---------------
namespace {

// out_off[l] = old_off[l] + new_off[l]  (both are list prefixes; l in [0, nlist])
__global__ __launch_bounds__(256) void k_sum_offsets(const int64_t* __restrict__ a, const int64_t* __restrict__ b,
                                                     int n, int64_t* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i <= n) out[i] = a[i] + b[i];
}

// first index in v[0, n) with v[i] >= x (lower) or > x (upper)
__device__ __forceinline__ int64_t bsearch_i64(const int64_t* __restrict__ v, int64_t n, int64_t x, bool upper) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (upper ? v[mid] <= x : v[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ void copy_code(uint8_t* __restrict__ d, const uint8_t* __restrict__ s, int M) {
  if ((M & 15) == 0) {
    for (int v = 0; v < M / 16; v++) reinterpret_cast<uint4*>(d)[v] = reinterpret_cast<const uint4*>(s)[v];
  } else if ((M & 7) == 0) {
    for (int v = 0; v < M / 8; v++) reinterpret_cast<uint2*>(d)[v] = reinterpret_cast<const uint2*>(s)[v];
  } else {
    for (int v = 0; v < M; v++) d[v] = s[v];
  }
}

// One workgroup per (list, 64 Ki-entry tile): list l's old entries O (label-sorted)
// and new entries N (label-sorted) interleaved by label into the output list, old
// before new on equal labels (the stable (list, label) order of a full re-sort of
// old + new).  Old entry r lands at r + |{n in N : n < label_r}|, new entry t at
// t + |{o in O : o <= label_t}|; when every new label is above the old ones (ids
// assigned sequentially) both counts are trivial and the list is an append.
constexpr int kTile = 65536;
__global__ __launch_bounds__(256) void k_merge_lists(int lo, int hi, const int64_t* __restrict__ old_off,
                                                     const uint8_t* __restrict__ old_codes,
                                                     const int64_t* __restrict__ old_ids,
                                                     const int64_t* __restrict__ new_off,
                                                     const uint8_t* __restrict__ new_codes,
                                                     const int64_t* __restrict__ new_ids,
                                                     const int64_t* __restrict__ out_off, int M,
                                                     uint8_t* __restrict__ out_codes, int64_t* __restrict__ out_ids) {
  // lists beyond gridDim.y (at most 65535 rows) are taken in strides of it
  for (int l = lo + blockIdx.y; l < hi; l += gridDim.y) {
    const int64_t ob = old_off[l], no = old_off[l + 1] - ob;
    const int64_t nb = new_off[l], nn = new_off[l + 1] - nb;
    const int64_t t0 = (int64_t)blockIdx.x * kTile;
    if (t0 >= no + nn) continue;
    const int64_t dst = out_off[l];
    const int64_t* O = old_ids + ob;
    const int64_t* N = new_ids + nb;
    const bool append = nn == 0 || no == 0 || O[no - 1] < N[0];
    const int64_t t1 = min(t0 + kTile, no + nn);
    for (int64_t e = t0 + threadIdx.x; e < t1; e += 256) {
      if (e < no) {  // old entry r = e
        const int64_t lab = O[e];
        const int64_t at = dst + e + (append ? 0 : bsearch_i64(N, nn, lab, false));
        copy_code(out_codes + at * M, old_codes + (ob + e) * M, M);
        out_ids[at] = lab;
      } else {  // new entry t = e - no
        const int64_t t = e - no;
        const int64_t lab = N[t];
        const int64_t at = dst + t + (append ? no : bsearch_i64(O, no, lab, true));
        copy_code(out_codes + at * M, new_codes + (nb + t) * M, M);
        out_ids[at] = lab;
      }
    }
  }
}

// entries of `lists` inside [lo, hi) (the ones a list-range shard keeps), added to *count
__global__ __launch_bounds__(256) void k_count_kept(const int64_t* __restrict__ lists, int64_t n, int lo, int hi,
                                                    unsigned long long* __restrict__ count) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool keep = i < n && lists[i] >= lo && lists[i] < hi;
  const unsigned long long m = __ballot(keep);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(count, (unsigned long long)__popcll(m));
}

}  // namespace

hipError_t image_merge_lists(const ListMergeArgs& g, hipStream_t s) {
  hipLaunchKernelGGL(k_sum_offsets, dim3(nblk(g.nlist + 1, 256)), dim3(256), 0, s, g.old_off, g.new_off, g.nlist,
                     g.out_off);
  if (g.hi > g.lo && g.max_list > 0) {
    const dim3 grid((unsigned)((g.max_list + kTile - 1) / kTile), (unsigned)std::min(g.hi - g.lo, 65535));
    hipLaunchKernelGGL(k_merge_lists, grid, dim3(256), 0, s, g.lo, g.hi, g.old_off, g.old_codes, g.old_ids, g.new_off,
                       g.new_codes, g.new_ids, g.out_off, g.M, g.out_codes, g.out_ids);
  }
  return hipGetLastError();
}

hipError_t count_kept(const int64_t* lists, int64_t n, int lo, int hi, unsigned long long* count, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_count_kept, dim3(nblk(n, 256)), dim3(256), 0, s, lists, n, lo, hi, count);
  return hipGetLastError();
}

void launch_iota_i64(int64_t* v, int64_t n, int64_t start, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_iota_i64, dim3(nblk(n, 256)), dim3(256), 0, s, v, n, start);
}

}  // namespace chivf
