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

}  // namespace chivf
