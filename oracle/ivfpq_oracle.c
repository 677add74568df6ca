/*
 * ivfpq_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the IVF-PQ search path that Chameleon runs on Faiss
 * (faiss-cpu 1.7.1, Chameleon/Faiss_experiments/README.md:18; not vendored in
 * the reference and not installed here), used as the parity checker for the
 * MI355X HIP engine and as the `cpu_baseline` ("port") leg of bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may load it.
 * The product (chameleon-rag-acceleration_amd/) never links or calls this file.
 *
 * Pinning: see DESIGN.md §Oracle.  Faiss itself cannot run here, so the
 * bit-level operation order below is the Faiss-1.7.1 AVX order restated in
 * SURVEY.md Appendix A ("parity unpinned" at the Faiss boundary).  The
 * semantics are pinned by (1) golden vectors produced by the reference's own
 * NumPy IVF-PQ search (my_faiss_extract_scripts/IVFPQ_1B_search.ipynb, cell 20:
 * construct_distance_table :7929, estimate_distance(s) :7948-7985,
 * search_single_query :7986-8018) executed in this container by
 * tests/golden/make_golden.py, and (2) the FPGA LUT known-answer test
 * (retrieval_accelerator/LUT_construction_PEs/LUT_construction_PE_D128_M32/
 * src/host.cpp:44-109).
 *
 * Operation order (all fp32, compiled with -ffp-contract=off):
 *  - tree(x, y, d): Faiss fvec_inner_product / fvec_norm_L2sqr / fvec_L2sqr
 *    AVX order: 8 interleaved accumulators over full 8-chunks, then
 *    hi+lo fold to 4, 4-wide remainder, masked tail, two horizontal adds.
 *    For d = 8: ((p0+p4)+(p1+p5)) + ((p2+p6)+(p3+p7))  (SURVEY App. A.2).
 *  - coarse distance (IndexFlatL2 BLAS path, n >= 20):
 *    dis = (|x|^2 + |c|^2) - 2*ip, ip = k-ordered fmaf chain, clamp at 0
 *    (the chain is what f32 MFMA / sgemm-style kernels do).
 *  - T1[l][m][j] = |C_mj|^2 + 2 * tree_ip(c_l[m], C_mj)   (precompute_table)
 *  - T3[q][m][j] = tree_ip(q[m], C_mj)                   (compute_inner_prod_table)
 *  - LUT = T1[l] + (-2) * T3                               (fvec_madd, bf = -2)
 *  - per code: dis = dis0; dis += LUT[m][code[m]] for m = 0..M-1 in order
 *    (scan_list_with_table, 1.7.1; the FPGA PE sums the same table,
 *    retrieval_accelerator/entire_accelerator_final_SIFT_M16/src/ADC.hpp:86-90)
 *  - top-k: the k smallest (dis, label) pairs, lexicographic;
 *    missing results are (FLT_MAX, -1).
 *  - METRIC_INNER_PRODUCT (beir's default, beir/beir/retrieval/search/dense/
 *    faiss_search.py:170, 194), Faiss 1.7.1 by-residual IP semantics
 *    (IVFPQScanner<METRIC_INNER_PRODUCT, CMin>, precompute_list_tables_IP):
 *    coarse = IndexFlatIP (k-ordered fmaf chain, the nprobe LARGEST);
 *    per query LUT = T3 (no precomputed table); per probe
 *    dis0 = tree_ip(q, c_l) over d (the coarse similarity is not reused);
 *    per code dis = dis0 + sum_m T3[m][code[m]] in order; the k LARGEST,
 *    ties by label; missing results are (-FLT_MAX, -1) (CMin's neutral).
 *    Parity unpinned: the reference's NumPy oracle and the FPGA are L2-only.
 *  - encode (add): coarse top-1, residual r = x - c, per sub-quantizer the
 *    first argmin of tree_L2(r_m, C_mj)   (ProductQuantizer::compute_code).
 *  - k-means: this build's own deterministic Lloyd k-means (Faiss training is
 *    BLAS-dependent and cannot be reproduced without Faiss).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { OR_IP = 0, OR_L2 = 1, OR_NORM = 2 };

static inline float or_term(const float *x, const float *y, int i, int kind) {
    if (kind == OR_IP) return x[i] * y[i];
    if (kind == OR_L2) {
        float t = x[i] - y[i];
        return t * t;
    }
    return x[i] * x[i];
}

/* Faiss 1.7.1 AVX reduction order (utils/distances_simd.cpp, fvec_*). */
float or_tree(const float *x, const float *y, int d, int kind) {
    float a8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int i = 0;
    for (; i + 8 <= d; i += 8)
        for (int j = 0; j < 8; j++) a8[j] = a8[j] + or_term(x, y, i + j, kind);
    float a4[4];
    for (int j = 0; j < 4; j++) a4[j] = a8[j + 4] + a8[j];
    if (i + 4 <= d) {
        for (int j = 0; j < 4; j++) a4[j] = a4[j] + or_term(x, y, i + j, kind);
        i += 4;
    }
    for (int j = 0; i + j < d; j++) a4[j] = a4[j] + or_term(x, y, i + j, kind);
    float h0 = a4[0] + a4[1];
    float h1 = a4[2] + a4[3];
    return h0 + h1;
}

/* k-ordered fmaf chain (one rounding per product, k ascending). */
static inline float or_fma_dot(const float *x, const float *y, int d) {
    float acc = 0.0f;
    for (int k = 0; k < d; k++) acc = fmaf(x[k], y[k], acc);
    return acc;
}

void or_norms(const float *x, int64_t n, int d, float *out) {
    for (int64_t i = 0; i < n; i++) out[i] = or_tree(x + i * d, x + i * d, d, OR_NORM);
}

static inline float or_coarse_dis(const float *x, float xn, const float *c, float cn, int d) {
    float ip = or_fma_dot(x, c, d);
    float dis = (xn + cn) - 2.0f * ip;
    if (dis < 0) dis = 0;
    return dis;
}

/* ---------------- bounded top-k, lexicographic (dis, label) ---------------- */

static inline int or_less(float da, int64_t ia, float db, int64_t ib) {
    return da < db || (da == db && ia < ib);
}

/* "a ranks before b": L2 ascending distance, IP descending similarity; ties by label */
static inline int or_before(int ip, float da, int64_t ia, float db, int64_t ib) {
    if (ip) return da > db || (da == db && ia < ib);
    return or_less(da, ia, db, ib);
}

/* bounded heap on (dis, label) whose root is the worst kept element:
 * L2 a max-heap of distances (Faiss CMax), IP a min-heap of similarities (CMin) */
static void or_heap_push(int ip, float *hd, int64_t *hi, int *sz, int k, float d, int64_t id) {
    if (*sz < k) {
        int i = (*sz)++;
        while (i > 0) {
            int p = (i - 1) / 2;
            if (!or_before(ip, hd[p], hi[p], d, id)) break;
            hd[i] = hd[p];
            hi[i] = hi[p];
            i = p;
        }
        hd[i] = d;
        hi[i] = id;
        return;
    }
    if (!or_before(ip, d, id, hd[0], hi[0])) return;
    int i = 0;
    for (;;) {
        int l = 2 * i + 1, r = l + 1, c = i;
        float cd = d;
        int64_t ci = id;
        if (l < k && or_before(ip, cd, ci, hd[l], hi[l])) { c = l; cd = hd[l]; ci = hi[l]; }
        if (r < k && or_before(ip, cd, ci, hd[r], hi[r])) { c = r; }
        if (c == i) break;
        hd[i] = hd[c];
        hi[i] = hi[c];
        i = c;
    }
    hd[i] = d;
    hi[i] = id;
}

static void or_heap_sort_out(int ip, float *hd, int64_t *hi, int sz, int k, float *D, int64_t *I) {
    /* pop the worst repeatedly into the back */
    for (int n = sz; n > 0; n--) {
        float md = hd[0];
        int64_t mi = hi[0];
        float ld = hd[n - 1];
        int64_t li = hi[n - 1];
        int i = 0, m = n - 1;
        for (;;) {
            int l = 2 * i + 1, r = l + 1, c = i;
            float cd = ld;
            int64_t ci = li;
            if (l < m && or_before(ip, cd, ci, hd[l], hi[l])) { c = l; cd = hd[l]; ci = hi[l]; }
            if (r < m && or_before(ip, cd, ci, hd[r], hi[r])) { c = r; }
            if (c == i) break;
            hd[i] = hd[c];
            hi[i] = hi[c];
            i = c;
        }
        if (m > 0) { hd[i] = ld; hi[i] = li; }
        D[n - 1] = md;
        I[n - 1] = mi;
    }
    for (int j = sz; j < k; j++) { D[j] = ip ? -FLT_MAX : FLT_MAX; I[j] = -1; }
}

/* ---------------- coarse quantizer (IndexFlatL2::search) ---------------- */

/* For each query the `nprobe` best coarse lists: L2 the smallest distances,
 * ascending by (dis, list id); IP (metric 0) the largest inner products,
 * descending, ties by list id.  Reference call site: bench_polysemous_1bn.py:430
 * → IndexIVF::search → quantizer->search. */
void or_coarse_search_metric(const float *x, int64_t n, int d, const float *cent, const float *cnorm,
                             int nlist, int nprobe, int64_t *lists, float *dis, int nthreads, int metric) {
    const int ip = metric == 0;
    if (nprobe > nlist) nprobe = nlist;
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
    {
        float *hd = (float *)malloc(sizeof(float) * nprobe);
        int64_t *hi = (int64_t *)malloc(sizeof(int64_t) * nprobe);
#pragma omp for schedule(dynamic, 4)
        for (int64_t q = 0; q < n; q++) {
            const float *xq = x + q * d;
            float xn = or_tree(xq, xq, d, OR_NORM);
            int sz = 0;
            for (int c = 0; c < nlist; c++) {
                const float *cc = cent + (int64_t)c * d;
                float dd = ip ? or_fma_dot(xq, cc, d) : or_coarse_dis(xq, xn, cc, cnorm[c], d);
                or_heap_push(ip, hd, hi, &sz, nprobe, dd, c);
            }
            or_heap_sort_out(ip, hd, hi, sz, nprobe, dis + q * nprobe, lists + q * nprobe);
        }
        free(hd);
        free(hi);
    }
}

void or_coarse_search(const float *x, int64_t n, int d, const float *cent, const float *cnorm,
                      int nlist, int nprobe, int64_t *lists, float *dis, int nthreads) {
    or_coarse_search_metric(x, n, d, cent, cnorm, nlist, nprobe, lists, dis, nthreads, 1);
}

/* ---------------- linear pre-transform ---------------- */

/* y[i][j] = sum_t x[i][t] A[j][t] (+ b[j]): VectorTransform::apply of an
 * OPQMatrix / LinearTransform (Faiss LinearTransform::apply_noalloc does this
 * with sgemm, whose summation order BLAS leaves open; this restatement fixes it
 * as a t-ordered fmaf chain from 0 with the bias added last -- the order the GPU
 * kernel uses; parity with Faiss itself is unpinned).  A: [d_out][d_in]. */
void or_linear_transform(const float *x, int64_t n, int d_in, const float *A, const float *b, int d_out, float *y) {
    for (int64_t i = 0; i < n; i++)
        for (int j = 0; j < d_out; j++) {
            float acc = 0.0f;
            for (int t = 0; t < d_in; t++) acc = fmaf(x[i * d_in + t], A[(int64_t)j * d_in + t], acc);
            y[i * d_out + j] = b ? acc + b[j] : acc;
        }
}

/* ---------------- PQ tables ---------------- */

/* T3[q][m][j] = <q_m, C_mj>  (ProductQuantizer::compute_inner_prod_table) */
void or_ip_table(const float *x, int64_t n, int d, const float *codebook, int M, int ksub, float *out) {
    int dsub = d / M;
    for (int64_t q = 0; q < n; q++)
        for (int m = 0; m < M; m++)
            for (int j = 0; j < ksub; j++)
                out[(q * M + m) * ksub + j] =
                    or_tree(x + q * d + m * dsub, codebook + ((int64_t)m * ksub + j) * dsub, dsub, OR_IP);
}

/* T1[l][m][j] = |C_mj|^2 + 2 <c_l[m], C_mj>  (IndexIVFPQ::precompute_table) */
void or_precompute_T1(const float *cent, int nlist, int d, const float *codebook, int M, int ksub, float *T1) {
    int dsub = d / M;
    float *rn = (float *)malloc(sizeof(float) * M * ksub);
    for (int m = 0; m < M; m++)
        for (int j = 0; j < ksub; j++) {
            const float *cw = codebook + ((int64_t)m * ksub + j) * dsub;
            rn[m * ksub + j] = or_tree(cw, cw, dsub, OR_NORM);
        }
    /* lists are independent (a nlist = 262144 table is 4 GB): one thread per list range */
#pragma omp parallel for schedule(static)
    for (int l = 0; l < nlist; l++)
        for (int m = 0; m < M; m++)
            for (int j = 0; j < ksub; j++) {
                float ip = or_tree(cent + (int64_t)l * d + m * dsub, codebook + ((int64_t)m * ksub + j) * dsub,
                                   dsub, OR_IP);
                T1[((int64_t)l * M + m) * ksub + j] = rn[m * ksub + j] + 2.0f * ip;
            }
    free(rn);
}

/* ---------------- encode (add path) ---------------- */

/* coarse assignment of one vector: L2 the first nearest centroid, IP (metric 0)
 * the first largest inner product (IndexFlatIP as the IVF quantizer) */
static inline int or_assign(const float *xi, float xn, const float *cent, const float *cnorm, int nlist, int d,
                            int ip) {
    int best = 0;
    float bd = 0;
    for (int c = 0; c < nlist; c++) {
        const float *cc = cent + (int64_t)c * d;
        if (ip) {
            float dd = or_fma_dot(xi, cc, d);
            if (c == 0 || dd > bd) { bd = dd; best = c; }
        } else {
            float dd = or_coarse_dis(xi, xn, cc, cnorm[c], d);
            if (c == 0 || dd < bd) { bd = dd; best = c; }
        }
    }
    return best;
}

void or_encode_metric(const float *x, int64_t n, int d, const float *cent, const float *cnorm, int nlist,
                      const float *codebook, int M, int ksub, int64_t *list_no, uint8_t *codes, int nthreads,
                      int metric);

void or_encode(const float *x, int64_t n, int d, const float *cent, const float *cnorm, int nlist,
               const float *codebook, int M, int ksub, int64_t *list_no, uint8_t *codes, int nthreads) {
    or_encode_metric(x, n, d, cent, cnorm, nlist, codebook, M, ksub, list_no, codes, nthreads, 1);
}

void or_encode_metric(const float *x, int64_t n, int d, const float *cent, const float *cnorm, int nlist,
                      const float *codebook, int M, int ksub, int64_t *list_no, uint8_t *codes, int nthreads,
                      int metric) {
    int dsub = d / M;
    const int ip = metric == 0;
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
    {
        float *r = (float *)malloc(sizeof(float) * d);
#pragma omp for schedule(dynamic, 64)
        for (int64_t i = 0; i < n; i++) {
            const float *xi = x + i * d;
            float xn = or_tree(xi, xi, d, OR_NORM);
            int best = or_assign(xi, xn, cent, cnorm, nlist, d, ip);
            list_no[i] = best;
            const float *cb = cent + (int64_t)best * d;
            for (int t = 0; t < d; t++) r[t] = xi[t] - cb[t];
            for (int m = 0; m < M; m++) {
                int bj = 0;
                float bjd = 0;
                for (int j = 0; j < ksub; j++) {
                    float dd = or_tree(r + m * dsub, codebook + ((int64_t)m * ksub + j) * dsub, dsub, OR_L2);
                    if (j == 0 || dd < bjd) { bjd = dd; bj = j; }
                }
                codes[i * M + m] = (uint8_t)bj;
            }
        }
        free(r);
    }
}

/* ---------------- search over inverted lists ---------------- */

/* IndexIVF::search_preassigned + IVFPQScanner (precompute mode 2).
 * lists / dis0: [n][nprobe]; list id < 0 = skipped probe.
 * list_off: [nlist+1] offsets into codes (in codes) and ids.
 * metric 1 (L2): LUT = T1[l] + (-2) T3, dis0 = the given coarse distance.
 * metric 0 (IP): LUT = T3, dis0 = tree_ip(q, centroid l) over d (cent), the
 * given dis0 is ignored (precompute_list_tables_IP). */
void or_search_preassigned_metric(const float *x, int64_t n, int d, const float *T1, const float *codebook,
                                  int M, int ksub, const int64_t *list_off, const uint8_t *codes,
                                  const int64_t *ids, int nprobe, const int64_t *lists, const float *dis0,
                                  int k, float *D, int64_t *I, int nthreads, int metric, const float *cent) {
    const int ip = metric == 0;
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
    {
        float *t3 = (float *)malloc(sizeof(float) * M * ksub);
        float *lut = (float *)malloc(sizeof(float) * M * ksub);
        float *hd = (float *)malloc(sizeof(float) * k);
        int64_t *hi = (int64_t *)malloc(sizeof(int64_t) * k);
#pragma omp for schedule(dynamic, 1)
        for (int64_t q = 0; q < n; q++) {
            const float *xq = x + q * d;
            or_ip_table(xq, 1, d, codebook, M, ksub, t3);
            int sz = 0;
            for (int p = 0; p < nprobe; p++) {
                int64_t l = lists[q * nprobe + p];
                if (l < 0) continue;
                int dup = 0; /* a list repeated in the row is scanned once */
                for (int j = 0; j < p && !dup; j++) dup = lists[q * nprobe + j] == l;
                if (dup) continue;
                float d0;
                const float *tab;
                if (ip) {
                    d0 = or_tree(xq, cent + l * d, d, OR_IP);
                    tab = t3;
                } else {
                    d0 = dis0 ? dis0[q * nprobe + p] : 0.0f;
                    const float *t1 = T1 + l * M * ksub;
                    for (int e = 0; e < M * ksub; e++) lut[e] = t1[e] + (-2.0f * t3[e]);
                    tab = lut;
                }
                int64_t beg = list_off[l], end = list_off[l + 1];
                for (int64_t i = beg; i < end; i++) {
                    const uint8_t *c = codes + i * M;
                    float dis = d0;
                    for (int m = 0; m < M; m++) dis = dis + tab[m * ksub + c[m]];
                    or_heap_push(ip, hd, hi, &sz, k, dis, ids[i]);
                }
            }
            or_heap_sort_out(ip, hd, hi, sz, k, D + q * k, I + q * k);
        }
        free(t3);
        free(lut);
        free(hd);
        free(hi);
    }
}

void or_search_preassigned(const float *x, int64_t n, int d, const float *T1, const float *codebook,
                           int M, int ksub, const int64_t *list_off, const uint8_t *codes,
                           const int64_t *ids, int nprobe, const int64_t *lists, const float *dis0,
                           int k, float *D, int64_t *I, int nthreads) {
    or_search_preassigned_metric(x, n, d, T1, codebook, M, ksub, list_off, codes, ids, nprobe, lists, dis0, k, D, I,
                                 nthreads, 1, NULL);
}

/* ---------------- k-means (this build's own training) ---------------- */

static uint64_t or_splitmix(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* first k entries of a seeded partial Fisher-Yates permutation of [0, n) */
void or_rand_perm_prefix(int64_t n, int64_t k, uint64_t seed, int64_t *out) {
    int64_t *p = (int64_t *)malloc(sizeof(int64_t) * n);
    for (int64_t i = 0; i < n; i++) p[i] = i;
    uint64_t s = seed;
    for (int64_t i = 0; i < k; i++) {
        int64_t j = i + (int64_t)(or_splitmix(&s) % (uint64_t)(n - i));
        int64_t t = p[i];
        p[i] = p[j];
        p[j] = t;
        out[i] = p[i];
    }
    free(p);
}

/* Centroid update: per-centroid double sums in ascending point order, then
 * empty clusters are split off the largest one (smallest index on ties) with a
 * +-1/1024 relative perturbation alternating per dimension. */
void or_kmeans_update(const float *x, int64_t n, int d, int k, const int64_t *assign, float *cent) {
    double *sum = (double *)calloc((size_t)k * d, sizeof(double));
    int64_t *cnt = (int64_t *)calloc(k, sizeof(int64_t));
    for (int64_t i = 0; i < n; i++) {
        int64_t c = assign[i];
        cnt[c]++;
        for (int t = 0; t < d; t++) sum[c * d + t] += (double)x[i * d + t];
    }
    for (int c = 0; c < k; c++)
        if (cnt[c] > 0)
            for (int t = 0; t < d; t++) cent[(int64_t)c * d + t] = (float)(sum[(int64_t)c * d + t] / (double)cnt[c]);
    const float eps = 1.0f / 1024.0f;
    for (int c = 0; c < k; c++) {
        if (cnt[c] != 0) continue;
        int big = 0;
        for (int j = 1; j < k; j++)
            if (cnt[j] > cnt[big]) big = j;
        for (int t = 0; t < d; t++) {
            float v = cent[(int64_t)big * d + t];
            if (t % 2 == 0) {
                cent[(int64_t)c * d + t] = v * (1.0f + eps);
                cent[(int64_t)big * d + t] = v * (1.0f - eps);
            } else {
                cent[(int64_t)c * d + t] = v * (1.0f - eps);
                cent[(int64_t)big * d + t] = v * (1.0f + eps);
            }
        }
        cnt[c] = cnt[big] / 2;
        cnt[big] -= cnt[c];
    }
    free(sum);
    free(cnt);
}

/* Spherical step (Faiss Clustering::spherical, set by IndexIVF for
 * METRIC_INNER_PRODUCT; fvec_renorm_L2): each row scaled to unit L2 norm,
 * inv = 1.0 / sqrtf(|x|^2) as Faiss computes it.  Sequential float norm (the same
 * code as renorm_rows in csrc/ivfpq_index.cpp). */
void or_renorm_rows(float *x, int64_t n, int d) {
    for (int64_t i = 0; i < n; i++) {
        float *xi = x + i * d;
        float nr = 0.f;
        for (int t = 0; t < d; t++) nr += xi[t] * xi[t];
        if (nr > 0.f) {
            const float inv = (float)(1.0 / (double)sqrtf(nr));
            for (int t = 0; t < d; t++) xi[t] *= inv;
        }
    }
}

/* Lloyd k-means, niter rounds of (assign: first nearest centroid by coarse
 * distance, or for IP (metric 0) first largest inner product; update).  IP is
 * spherical: centroids renormalized after the initialization and every update. */
void or_kmeans_metric(const float *x, int64_t n, int d, int k, int niter, uint64_t seed, float *cent, int nthreads,
                      int metric) {
    const int ip = metric == 0;
    int64_t *init = (int64_t *)malloc(sizeof(int64_t) * k);
    or_rand_perm_prefix(n, k, seed, init);
    for (int c = 0; c < k; c++) memcpy(cent + (int64_t)c * d, x + init[c] * d, sizeof(float) * d);
    free(init);
    if (ip) or_renorm_rows(cent, k, d);
    int64_t *assign = (int64_t *)malloc(sizeof(int64_t) * n);
    float *cn = (float *)malloc(sizeof(float) * k);
    for (int it = 0; it < niter; it++) {
        or_norms(cent, k, d, cn);
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(dynamic, 256)
        for (int64_t i = 0; i < n; i++) {
            const float *xi = x + i * d;
            float xn = or_tree(xi, xi, d, OR_NORM);
            assign[i] = or_assign(xi, xn, cent, cn, k, d, ip);
        }
        or_kmeans_update(x, n, d, k, assign, cent);
        if (ip) or_renorm_rows(cent, k, d);
    }
    free(assign);
    free(cn);
}

void or_kmeans(const float *x, int64_t n, int d, int k, int niter, uint64_t seed, float *cent, int nthreads) {
    or_kmeans_metric(x, n, d, k, niter, seed, cent, nthreads, 1);
}

/* IVF-PQ training: coarse k-means (assignment by the index metric), residuals
 * to the assigned centroid, then one 2^nbits-centroid L2 k-means per sub-space
 * (seed + 1 + m; Faiss trains the product quantizer in L2 for both metrics). */
void or_train_ivfpq_metric(const float *x, int64_t n, int d, int nlist, int M, int ksub, int niter_coarse,
                           int niter_pq, uint64_t seed, float *cent, float *codebook, int nthreads, int metric) {
    int dsub = d / M;
    const int ip = metric == 0;
    or_kmeans_metric(x, n, d, nlist, niter_coarse, seed, cent, nthreads, metric);
    float *cn = (float *)malloc(sizeof(float) * nlist);
    or_norms(cent, nlist, d, cn);
    float *r = (float *)malloc(sizeof(float) * n * d);
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(dynamic, 256)
    for (int64_t i = 0; i < n; i++) {
        const float *xi = x + i * d;
        float xn = or_tree(xi, xi, d, OR_NORM);
        int best = or_assign(xi, xn, cent, cn, nlist, d, ip);
        for (int t = 0; t < d; t++) r[i * d + t] = xi[t] - cent[(int64_t)best * d + t];
    }
    float *sub = (float *)malloc(sizeof(float) * n * dsub);
    for (int m = 0; m < M; m++) {
        for (int64_t i = 0; i < n; i++) memcpy(sub + i * dsub, r + i * d + m * dsub, sizeof(float) * dsub);
        or_kmeans(sub, n, dsub, ksub, niter_pq, seed + 1 + (uint64_t)m, codebook + (int64_t)m * ksub * dsub,
                  nthreads);
    }
    free(sub);
    free(r);
    free(cn);
}

void or_train_ivfpq(const float *x, int64_t n, int d, int nlist, int M, int ksub, int niter_coarse,
                    int niter_pq, uint64_t seed, float *cent, float *codebook, int nthreads) {
    or_train_ivfpq_metric(x, n, d, nlist, M, ksub, niter_coarse, niter_pq, seed, cent, codebook, nthreads, 1);
}

/* recall helpers */
double or_recall_1_at_k(const int64_t *I, int64_t n, int k, int kk, const int64_t *gt, int gt_stride) {
    int64_t ok = 0;
    for (int64_t q = 0; q < n; q++)
        for (int j = 0; j < kk && j < k; j++)
            if (I[q * k + j] == gt[q * gt_stride]) { ok++; break; }
    return (double)ok / (double)n;
}
