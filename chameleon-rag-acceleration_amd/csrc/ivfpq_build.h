// Device-side inverted-list image build (ivfpq_build.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace chivf {

// Merge of the current image (n_old entries, list-contiguous, offsets old_off
// [nlist + 1]) with n_new new entries (list numbers from the assignment, labels,
// codes) into a new image, stable by (list, label); new entries whose list is
// outside [lo, hi) are dropped.  All pointers are device pointers.
struct ImageMergeArgs {
  int nlist = 0, lo = 0, hi = 0, M = 0;
  int64_t n_old = 0;
  const int64_t* old_off = nullptr;
  const int64_t* old_ids = nullptr;
  const uint8_t* old_codes = nullptr;
  int64_t n_new = 0;
  const int64_t* new_lists = nullptr;
  const int64_t* new_ids = nullptr;
  const uint8_t* new_codes = nullptr;
  int64_t* off_out = nullptr;  // [nlist + 1]; off_out[nlist] = kept entries
  uint8_t* codes_out = nullptr;
  int64_t* ids_out = nullptr;
};

size_t image_merge_scratch_bytes(int64_t n_all, int nlist);
// phase 1: sort and the new offsets (read off_out[nlist] to size the outputs)
hipError_t image_merge_sort(const ImageMergeArgs& g, void* scratch, size_t scratch_bytes, hipStream_t s);
// phase 2: the first n_out sorted entries' codes and labels into codes_out / ids_out
hipError_t image_merge_gather(const ImageMergeArgs& g, int64_t n_out, void* scratch, hipStream_t s);
void launch_iota_i64(int64_t* v, int64_t n, int64_t start, hipStream_t s);

// Per-list merge of a new image (new_off / new_codes / new_ids: entries sorted by
// (list, label), e.g. the output of image_merge_sort + image_merge_gather over the
// new entries alone) into the current image: out_off = old_off + new_off, and
// every list of [lo, hi) interleaved by label, old entries first on equal labels
// -- the image a full re-sort of old + new gives, built by moving each entry once
// (no sort of the old entries).  max_list: the largest old + new list length.
struct ListMergeArgs {
  int nlist = 0, lo = 0, hi = 0, M = 0;
  int64_t max_list = 0;
  const int64_t* old_off = nullptr;
  const uint8_t* old_codes = nullptr;
  const int64_t* old_ids = nullptr;
  const int64_t* new_off = nullptr;
  const uint8_t* new_codes = nullptr;
  const int64_t* new_ids = nullptr;
  int64_t* out_off = nullptr;
  uint8_t* out_codes = nullptr;
  int64_t* out_ids = nullptr;
};
hipError_t image_merge_lists(const ListMergeArgs& g, hipStream_t s);
// *count += entries of lists[0, n) inside [lo, hi)
hipError_t count_kept(const int64_t* lists, int64_t n, int lo, int hi, unsigned long long* count, hipStream_t s);

}  // namespace chivf
