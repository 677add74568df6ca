/*
 * ivfpq.h — C-ABI of libivfpq.so, the MI355X (gfx950) IVF-PQ engine.
 *
 * Drop-in boundary for the IVF-PQ search path that Chameleon reaches through
 * Faiss's Python surface.  Each entry point names the
 * Faiss / Chameleon interface it replaces.  Plain pointers and sizes only;
 * host entry points take host buffers (numpy), *_device entry points take
 * device pointers plus a hipStream_t passed as void*.
 *
 * Conventions (as faiss.IndexIVFPQ):
 *   x: float32 [n][d] row-major;  D: float32 [n][k] ascending L2 distances
 *   (METRIC_L2) or descending inner products (METRIC_INNER_PRODUCT);
 *   I: int64 [n][k] labels, -1 (with distance FLT_MAX, or -FLT_MAX for inner
 *   product: the Faiss heap's neutral element) where fewer than k results
 *   exist.  Ties are ordered by label.
 * Errors: every int-returning function returns 0 on success and -1 on error;
 * ivfpq_last_error() gives the thread-local message (the Python layer raises
 * RuntimeError, as Faiss's SWIG wrapper does for FaissException).
 * Thread-safety: one mutex per handle; train/add/search serialize on it.
 * Stream ordering: a handle's device searches may be issued on different
 * streams without synchronizing.  By default each one waits (hipStreamWaitEvent)
 * for every search of the handle still in flight on another stream.  With
 * batches in flight on (ivfpq_set_inflight, or IVFPQ_INFLIGHT=1 in the
 * environment when the handle is created) searches on up to three streams
 * overlap, each in the per-stream workspace it last used; a fourth stream takes
 * over the least recently used workspace after waiting on the host for its
 * last search.
 * Results under concurrent GPU work: the same in both modes and beside other
 * kernels on the GPU.  Round 4's rare wrong rows under concurrent kernels came
 * from per-lane reads of the scan's shared bounds ("Uniform
 * bounds"; fixed in round 5, 0 of 1 046 400 stressed batches since).  Every per-wave
 * partial list the merge reads is also a set of tagged records (batch epoch +
 * slot): an entry this batch's scan did not leave there is never used -- its probe
 * is rescanned on the device by the merge -- and such events are counted
 * (ivfpq_get_repair_stats; 0 in every real search since the fix, and the concurrency
 * gates of the test suite assert it).
 * Test and diagnostic hooks (fault injection, seeded bounds, workspace dumps) are not part
 * of this drop-in surface: they are declared in ivfpq_test.h, for the test suite only.
 */
#ifndef CHAMELEON_IVFPQ_H
#define CHAMELEON_IVFPQ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ivfpq_index ivfpq_index;

#define IVFPQ_METRIC_INNER_PRODUCT 0 /* faiss.METRIC_INNER_PRODUCT (beir faiss_search.py:170, 194) */
#define IVFPQ_METRIC_L2 1            /* faiss.METRIC_L2 */

/* Last error message of the calling thread ("" if none). */
const char* ivfpq_last_error(void);

/* Number of visible HIP devices (faiss.get_num_gpus, beir faiss_index.py:46). */
int ivfpq_device_count(void);

/* faiss.IndexIVFPQ(quantizer, d, nlist, M, nbits) / index_factory(d, "IVF<nlist>,PQ<M>")
 * (IVFPQ_random_dataset.py:22-24, bench_polysemous_1bn.py:272).  nbits must be 8. */
int ivfpq_create(int d, int nlist, int M, int nbits, int metric, int device, ivfpq_index** out);
int ivfpq_free(ivfpq_index* h);

/* Index.train(x)  (bench_polysemous_1bn.py:283; beir faiss_index.py FaissTrainIndex.build).
 * Lloyd k-means on the GPU: coarse (niter_coarse) then one per sub-space (niter_pq). */
int ivfpq_train(ivfpq_index* h, int64_t n, const float* x, int niter_coarse, int niter_pq, uint64_t seed);

/* Index.add(x) / add_with_ids(x, ids)  (bench_polysemous_1bn.py:343-345; beir faiss_index.py:41-42).
 * ids == NULL assigns ntotal, ntotal+1, ...  Encoding runs on the GPU. */
int ivfpq_add(ivfpq_index* h, int64_t n, const float* x, const int64_t* ids);

/* Index.add / add_with_ids with the vectors (and ids, nullable) already in HBM:
 * device pointers, on `stream` (NULL = the handle's stream).  Coarse assignment
 * on the matrix cores (the search's coarse kernels, top-1), PQ encode and the
 * merge into the device list image all run on the GPU (ivfpq_add takes the same
 * path from host buffers).  Reference: bench_gpu_1bn.py:598-658 (the 1e9 base
 * set added through the GPU index in slices).  Returns when the image is in place. */
int ivfpq_add_device(ivfpq_index* h, int64_t n, const float* x, const int64_t* ids, void* stream);

/* invlists.add_entries with precomputed (list, code, id) triples, e.g. from a
 * loaded Faiss index or another shard.  codes: uint8 [n][M]. */
int ivfpq_add_preencoded(ivfpq_index* h, int64_t n, const int64_t* list_no, const uint8_t* codes,
                         const int64_t* ids);

/* Index.reset(): drop all inverted-list entries, keep the trained quantizers. */
int ivfpq_reset(ivfpq_index* h);

/* index.nprobe = p / ParameterSpace().set_index_parameters(index, "nprobe=p")
 * (faiss_retriever.py:170-176, bench_polysemous_1bn.py:422).  Clamped to nlist at search. */
int ivfpq_set_nprobe(ivfpq_index* h, int nprobe);
int ivfpq_get_nprobe(const ivfpq_index* h);

/* Shard range: only inverted lists in [lo, hi) are stored and scanned (list-range sharding,
 * SURVEY.md §8(e); replaces IndexShards, bench_gpu_1bn.py:605-616).  Default [0, nlist). */
int ivfpq_set_list_range(ivfpq_index* h, int lo, int hi);

/* Index.search(x, k) -> (D, I)  (beir faiss_index.py:22, bench_polysemous_1bn.py:430,
 * faiss_retriever.py:254, faiss_server.py:197).  Host buffers. k <= 1024. */
int ivfpq_search(ivfpq_index* h, int64_t n, const float* x, int k, float* D, int64_t* I);

/* IndexIVF::search_preassigned(n, x, k, Iq, Dq, D, I, store_pairs=False)
 * (faiss_retriever.py:217-223) and faiss.contrib.ivf_tools.search_preassigned
 * (faiss_retriever.py:265).  Iq: int64 [n][nprobe] list ids (-1 = skip);
 * Dq: float32 [n][nprobe] coarse distances, NULL = zeros (the upstream default). */
int ivfpq_search_preassigned(ivfpq_index* h, int64_t n, const float* x, int k, const int64_t* Iq, const float* Dq,
                             float* D, int64_t* I);

/* Device-pointer variants (inputs already resident in HBM; stream = hipStream_t, NULL = default).
 * The whole search: coarse probe, T3, fused LUT + scan + top-k. */
int ivfpq_search_device(ivfpq_index* h, int64_t n, const float* x, int k, float* D, int64_t* I, void* stream);
int ivfpq_search_preassigned_device(ivfpq_index* h, int64_t n, const float* x, int k, const int64_t* Iq,
                                    const float* Dq, float* D, int64_t* I, void* stream);
/* FaissServer request handling in the RALM wire format: decode_request[_with_lists] +
 * retrieve / retrieve_with_lists + encode_answer (ralm/server/faiss_server.py:170-277;
 * formats ralm/retriever/serialization_utils.py:17-35, 38-94, 173-258).  Header integers
 * are big-endian int32, arrays native-order:
 *   with_lists = 0: msg = k | queries f32 [batch_size][dim]               -> search (nprobe of the index)
 *   with_lists = 1: msg = batch_size, dim, nprobe, k | queries | lists i64 [batch_size][nprobe]
 *                                                                          -> search_preassigned, Dq = NULL
 * The answer is written to `answer`: I i64 [batch_size][k] then D f32 [batch_size][k];
 * *answer_len (nullable) = batch_size * k * 12.  msg_len must equal the format's message
 * length for (batch_size, dim[, nprobe]), and the with-lists header must match them
 * (decode_request_with_lists asserts, serialization_utils.py:211-213). */
int ivfpq_serve_request(ivfpq_index* h, const uint8_t* msg, int64_t msg_len, int with_lists, int batch_size, int dim,
                        int nprobe, uint8_t* answer, int64_t answer_cap, int64_t* answer_len);

/* The inner-product tables T3 of n HBM-resident queries (1 <= n <= 16384 at M=16:
 * one 256 MB table buffer), computed on `stream` ahead of the preassigned search
 * of those queries.  *token receives the handle that search passes to
 * ivfpq_search_preassigned_tables_device, which consumes the tables (the queries
 * x must be unchanged in between).  The shard flow issues it on a side stream
 * while the coarse step and the probe all-gather run (T3 depends only on the
 * queries).  Up to three tables can be pending, so a shard loop can keep batches
 * in flight; a fourth precompute overwrites the oldest pending one (its token is
 * then rejected).  Training, set_trained and reset drop pending tables.
 * ivfpq_search_preassigned_device never uses precomputed tables.
 * Reference: IndexIVFPQ::search_preassigned's per-query precompute_list_tables
 * (bench_gpu_1bn.py:605-616 shard step). */
int ivfpq_precompute_tables_device(ivfpq_index* h, int64_t n, const float* x, void* stream, uint64_t* token);
int ivfpq_search_preassigned_tables_device(ivfpq_index* h, int64_t n, const float* x, int k, const int64_t* Iq,
                                           const float* Dq, float* D, int64_t* I, uint64_t token, void* stream);

/* Batches in flight (see "Stream ordering" above): 1 = device searches on different
 * streams overlap, 0 = each waits for the others (default, unless IVFPQ_INFLIGHT=1).
 * Waits for the handle's in-flight searches before switching.  Reference: the query
 * blocks streamed through one GPU index, bench_gpu_1bn.py:788-806. */
int ivfpq_set_inflight(ivfpq_index* h, int on);
int ivfpq_get_inflight(const ivfpq_index* h);
/* 1: the overlap is available (kept for callers of the r04 interface). */
int ivfpq_overlap_built(void);

/* Index checks of the merge kernels: code positions read back from partial lists
 * outside the image, partial-list lengths above k and pair ids outside the batch
 * are counted (and dropped, never dereferenced).  *out = the count since the
 * handle was created, over all its workspaces, after waiting for in-flight
 * searches.  0 on a correct run; the tests assert it. */
int ivfpq_get_error_count(ivfpq_index* h, int64_t* out);

/* Stale partial lists (see "Results under concurrent GPU work" above): *stale_reads =
 * queries (counted once per search) whose merge read an entry whose tag was not this batch's,
 * *repairs = probes the merge rescanned because of one; totals since the handle was
 * created, over all workspaces, after waiting for in-flight searches. */
int ivfpq_get_repair_stats(ivfpq_index* h, int64_t* stale_reads, int64_t* repairs);
/* The first stale-entry events (at most 64 per workspace), 8 uint32 each: merge site
 * (1 fast path, 2 full merge) | reader XCD << 8, query, list j | rank << 16, expected
 * tag, found tag (writer XCD in bits 28-31), found key bits, batch epoch, and the
 * number of system-scope re-reads until the tag was fresh (0xFFFFFFFF = never within
 * 2000; fast path: 1 = fresh at once, 0 = not).  *n_events = events copied to out
 * (out holds max_events x 8 words). */
int ivfpq_get_repair_log(ivfpq_index* h, uint32_t* out, int max_events, int* n_events);
/* Stage entry points of the same search (for per-stage timing): the coarse quantizer
 * (IndexFlatL2::search as in ralm/index_scanner/index_scanner.py:61-77) writing
 * Iq [n][nprobe] / Dq [n][nprobe]; and the per-query inner-product table T3. */
int ivfpq_coarse_device(ivfpq_index* h, int64_t n, const float* x, int64_t* Iq, float* Dq, void* stream);
/* The front half of one list-range shard step (the IndexShards step it replaces:
 * bench_gpu_1bn.py:605-616), on ONE stream: the coarse quantizer of this rank's n queries
 * x (-> Iq, Dq as ivfpq_coarse_device) and T3 of the n_tables queries x_tables of the
 * global batch (the table workgroups ride in the same launch as the key tiles at
 * nlist < 8192).  *token receives the tables for ivfpq_search_preassigned_tables_device
 * of exactly x_tables (same rules as ivfpq_precompute_tables_device); no side stream. */
int ivfpq_coarse_tables_device(ivfpq_index* h, int64_t n, const float* x, int64_t* Iq, float* Dq, int64_t n_tables,
                               const float* x_tables, void* stream, uint64_t* token);

/* Merge S sorted partial results [S][n][k] into [n][k] on the device (the IndexShards
 * merge, bench_gpu_1bn.py:605-616; host argsort merge, bench_multi_cpu_performance_OSDI.py:203-218).
 * metric: IVFPQ_METRIC_L2 (partials ascending) or IVFPQ_METRIC_INNER_PRODUCT (descending). */
int ivfpq_merge_topk_device(int S, int64_t n, int k, int metric, const float* Din, const int64_t* Iin, float* Dout,
                            int64_t* Iout, void* stream);

/* Linear pre-transform on device buffers (Faiss VectorTransform::apply for OPQMatrix /
 * LinearTransform: the "OPQ16" of "OPQ16,IVF262144,PQ16", bench_gpu_1bn.py:485-489,
 * extract_FPGA_required_data.py:162-165): y[i][j] = sum_t x[i][t] * A[j][t] (+ b[j]),
 * the sum a t-ordered fused-multiply-add chain from 0, bias added last (Faiss uses
 * sgemm, whose order BLAS leaves open; this is the order of oracle/ivfpq_oracle.c).
 * AT = A transposed, [d_in][d_out]; b nullable; x [n][d_in], y [n][d_out]. */
int ivfpq_linear_transform_device(int64_t n, int d_in, int d_out, const float* AT, const float* b, const float* x,
                                  float* y, void* stream);

/* Per-stage device timing (the nsys stage split of MICRO_GPU_profiling/classify_stages.py:113-181,
 * measured live with HIP events recorded on the launch stream around each stage).
 * get_timing waits for the recorded events, returns per-stage sums in ms and launch counts
 * for stages {0: coarse probe, 1: inner-product table T3, 2: LUT + scan + top-k (all of it:
 * bucketing, seed pass, list scan, probe merge), 3: the list-scan kernel k_scan_lists alone
 * (list-major path; count 0 otherwise)}; both arrays hold 4 entries.  Resets.
 * on = 1: all stages; on = 2: only stage 3 (two events per batch: each recorded event
 * costs a few microseconds of stream time, so throughput runs time the list scan alone). */
int ivfpq_set_timing(ivfpq_index* h, int on);
int ivfpq_get_timing(ivfpq_index* h, double* ms, int64_t* count);

/* Accessors (extract_FPGA_required_data.py:174-248; bench_polysemous_1bn.py:368). */
int64_t ivfpq_ntotal(const ivfpq_index* h);
int ivfpq_is_trained(const ivfpq_index* h);
int ivfpq_get_dims(const ivfpq_index* h, int* d, int* nlist, int* M, int* nbits, int* metric);
int ivfpq_get_centroids(const ivfpq_index* h, float* out);  /* [nlist][d]  (quantizer.xb) */
int ivfpq_get_codebook(const ivfpq_index* h, float* out);   /* [M][256][d/M]  (pq.centroids) */
/* Install trained quantizers (e.g. from a Faiss .index or another process); builds T1 on the GPU. */
int ivfpq_set_trained(ivfpq_index* h, const float* centroids, const float* codebook);
int ivfpq_get_list_sizes(const ivfpq_index* h, int64_t* out); /* [nlist] (invlists.list_size) */
int ivfpq_get_list(const ivfpq_index* h, int list, uint8_t* codes, int64_t* ids); /* get_codes / get_ids */
/* T1 = precomputed_table [nlist][M][256] (IndexIVFPQ::precomputed_table), copied to the host. */
int ivfpq_get_precomputed_table(ivfpq_index* h, float* out);

/* faiss.write_index / read_index (bench_polysemous_1bn.py:287-290; beir faiss_index.py:29)
 * in this engine's own binary format ("CHIVFPQ1"). */
int ivfpq_save(ivfpq_index* h, const char* path);
int ivfpq_load(const char* path, int device, ivfpq_index** out);

/* Brute-force exact k-NN on the GPU: IndexFlatL2::search (metric L2; the coarse-quantizer
 * service of ralm/index_scanner/index_scanner.py:61-77) or IndexFlatIP::search (metric
 * INNER_PRODUCT; beir faiss_search.py's flat IP indexes).  Host buffers. */
int ivfpq_flat_search(int device, int d, int64_t nb, const float* xb, int64_t n, const float* x, int k, int metric,
                      float* D, int64_t* I);

#ifdef __cplusplus
}
#endif

#endif /* CHAMELEON_IVFPQ_H */
