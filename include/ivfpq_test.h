/*
 * ivfpq_test.h — test and diagnostic hooks of libivfpq.so.
 *
 * NOT part of the drop-in boundary (include/ivfpq.h): no Faiss call corresponds to
 * these, and a production caller has no reason to use them.  They exist so that the
 * test suite can drive the repair path of the probe merge (tests/test_gpu_repair.py),
 * check the bounded scan against seeded bounds ("Uniform
 * bounds") and inspect a workspace after a search.  None of them is reachable through
 * the faiss_amd surface used by the reference's callers.
 */
#ifndef CHAMELEON_IVFPQ_TEST_H
#define CHAMELEON_IVFPQ_TEST_H

#include "ivfpq.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Test hook for the repair path: every > 0 makes the list scan of later searches skip
 * the stores of the partial lists whose slot (pair * 4 + wave) % every == 1, as if
 * they were lost; 0 (default) turns it off.  Results must stay exact. */
int ivfpq_set_fault_injection(ivfpq_index* h, int every);
/* Diagnostics: copy (up to cap bytes of) one per-batch buffer of workspace ws (0..2) as the
 * last search on it left it -- what: 0 partial-list records, 1 partial-list counts, 2 probe
 * masks, 3 tau words, 4 header words, 5 coarse lists, 6 coarse dis0; 7 / 8: the epoch of the
 * last batch planned there / the stream it ran on (8 bytes each); *bytes = its size. */
int ivfpq_debug_workspace(ivfpq_index* h, int ws, int what, void* dst, int64_t cap, int64_t* bytes);
/* Test hook for the cross-workgroup bound: the next device search (of exactly n queries)
 * starts with query i's shared bound tau_i = keys[i] instead of +inf (one-shot).  Any
 * keys[i] >= that query's true k-th key is a valid bound, and results must not change. */
int ivfpq_debug_seed_tau(ivfpq_index* h, int64_t n, const float* keys);

#ifdef __cplusplus
}
#endif

#endif /* CHAMELEON_IVFPQ_TEST_H */
