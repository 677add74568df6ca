// Host side of libivfpq.so: the index object behind the C-ABI of include/ivfpq.h.
//
// Owns the trained quantizers and inverted lists on the host (insertion
// order per list, as Faiss ArrayInvertedLists) and their device images in
// HBM, and drives the gfx950 kernels of ivfpq_kernels.hip.  Training and
// encoding run on the GPU; only the k-means centroid update (a per-cluster
// double-precision mean) and list bookkeeping run on the host.
//
// HBM layout (DESIGN.md §Data layout):
//   centroids f32[nlist][d], |c|^2 f32[nlist], codebook f32[M][256][d/M],
//   T1 f32[nlist][M][256] (Faiss precomputed_table), codes u8[ntotal][M]
//   with lists concatenated in list order, ids i64[ntotal] alongside,
//   list offsets i64[nlist+1].
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "ivfpq.h"
#include "ivfpq_test.h"  // the test hooks are defined here too (not part of the drop-in header)
#include "ivfpq_kernels.h"
#include "ivfpq_build.h"

using namespace chivf;

namespace {

thread_local std::string g_err;

#define HIPCHECK(x)                                                                          \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

void require(bool ok, const std::string& msg) {
  if (!ok) throw std::runtime_error(msg);
}

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t b) {
    if (b <= bytes && p) return;
    release();
    if (b == 0) b = 16;
    HIPCHECK(hipMalloc(&p, b));
    bytes = b;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
};

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    HIPCHECK(hipGetDevice(&prev));
    if (prev != dev) HIPCHECK(hipSetDevice(dev));
  }
  ~DeviceGuard() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
  }
};

// Same generator and update rule as the oracle (oracle/ivfpq_oracle.c,
// or_rand_perm_prefix / or_kmeans_update) so GPU-trained and oracle-trained
// indexes are identical for identical input.
uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

std::vector<int64_t> rand_perm_prefix(int64_t n, int64_t k, uint64_t seed) {
  std::vector<int64_t> p(n), out(k);
  for (int64_t i = 0; i < n; i++) p[i] = i;
  uint64_t s = seed;
  for (int64_t i = 0; i < k; i++) {
    int64_t j = i + (int64_t)(splitmix(&s) % (uint64_t)(n - i));
    std::swap(p[i], p[j]);
    out[i] = p[i];
  }
  return out;
}

// Spherical k-means step (Faiss Clustering with spherical = true, which IndexIVF
// sets for METRIC_INNER_PRODUCT; fvec_renorm_L2): every centroid scaled to unit
// L2 norm.  Same arithmetic as or_renorm_rows in oracle/ivfpq_oracle.c.
void renorm_rows(float* x, int64_t n, int d) {
  for (int64_t i = 0; i < n; i++) {
    float* xi = x + i * d;
    float nr = 0.f;
    for (int t = 0; t < d; t++) nr += xi[t] * xi[t];
    if (nr > 0.f) {
      const float inv = (float)(1.0 / (double)sqrtf(nr));
      for (int t = 0; t < d; t++) xi[t] *= inv;
    }
  }
}

void kmeans_update(const float* x, int64_t n, int d, int k, const int64_t* assign, float* cent) {
  std::vector<double> sum((size_t)k * d, 0.0);
  std::vector<int64_t> cnt(k, 0);
  for (int64_t i = 0; i < n; i++) {
    const int64_t c = assign[i];
    cnt[c]++;
    double* s = &sum[(size_t)c * d];
    const float* xi = x + i * d;
    for (int t = 0; t < d; t++) s[t] += (double)xi[t];
  }
  for (int c = 0; c < k; c++)
    if (cnt[c] > 0)
      for (int t = 0; t < d; t++) cent[(size_t)c * d + t] = (float)(sum[(size_t)c * d + t] / (double)cnt[c]);
  const float eps = 1.0f / 1024.0f;
  for (int c = 0; c < k; c++) {
    if (cnt[c] != 0) continue;
    int big = 0;
    for (int j = 1; j < k; j++)
      if (cnt[j] > cnt[big]) big = j;
    for (int t = 0; t < d; t++) {
      const float v = cent[(size_t)big * d + t];
      if (t % 2 == 0) {
        cent[(size_t)c * d + t] = v * (1.0f + eps);
        cent[(size_t)big * d + t] = v * (1.0f - eps);
      } else {
        cent[(size_t)c * d + t] = v * (1.0f - eps);
        cent[(size_t)big * d + t] = v * (1.0f + eps);
      }
    }
    cnt[c] = cnt[big] / 2;
    cnt[big] -= cnt[c];
  }
}

constexpr size_t kChunkBytes = size_t(256) << 20;    // bound for [rows][cols] fp32 scratch
constexpr size_t kPartialBytes = size_t(2048) << 20;  // bound for a chunk's per-wave partial top-k lists
// from this nlist on, the coarse quantizer never writes the key matrix (r03 A/B at
// C2, nlist 1024: segmented 22.5 + 8.5 us + a separate T3 launch 13.0 us vs key
// matrix 17.8 + 10.0 us with T3 in the same launch)
constexpr int kSegmentedNlist = 8192;
// Default of a handle's batches-in-flight switch (ivfpq_set_inflight): with it
// on, device searches on different streams overlap, each on its own per-stream
// workspace; off, a search is ordered after every search still in flight on
// another stream.  IVFPQ_INFLIGHT=1 in the environment turns it on for new handles.
constexpr int kInflightFreeCus = 16;

bool inflight_default() {
  const char* e = std::getenv("IVFPQ_INFLIGHT");
  return e && e[0] == '1';
}

}  // namespace

struct ivfpq_index {
  int d = 0, nlist = 0, M = 0, nbits = 8, ksub = 256, metric = IVFPQ_METRIC_L2, device = 0;
  int nprobe = 1;
  int list_lo = 0, list_hi = 0;
  bool trained = false;
  std::vector<float> centroids, codebook;
  std::vector<std::vector<uint8_t>> lcodes;
  std::vector<std::vector<int64_t>> lids;
  int64_t ntotal = 0;
  int64_t next_id = 0;

  DevBuf d_cent, d_centT, d_cnorm, d_cb, d_T1, d_codes, d_ids, d_off, d_order;
  bool dirty = true;
  hipStream_t stream = nullptr;
  // scratch
  DevBuf w_x, w_xn, w_D, w_I, w_lno, w_codes, w_cent, w_cn;
  DevBuf h_D, h_I, h_Iq, h_Dq;  // device staging of the host-buffer entry points
  // device-side adds not yet merged into the image (add_dev / flush_pending): list
  // numbers (any list; entries outside [list_lo, list_hi) are dropped at the merge),
  // labels and codes, q_n of them (q_kept inside the range); a_off: small scratch
  DevBuf q_lists, q_ids, q_codes, a_off;
  int64_t q_n = 0, q_kept = 0, q_cap = 0;
  int64_t img_n = 0;  // entries in the device image (ntotal = img_n + q_kept)
  bool host_stale = false;  // the device image holds entries the host lists lack (device-side adds)
  // T3 of a batch computed ahead (ivfpq_precompute_tables_device), handed to a
  // preassigned search by the token that call returned (seq)
  struct PreT3 {
    DevBuf buf;
    int64_t n = 0;
    uint64_t seq = 0;  // the token; 0 = free
    uint64_t freed_seq = 0;  // order in which free entries were consumed (reuse the longest-free one)
    hipEvent_t ready = nullptr;  // recorded after the table launch
    hipStream_t ready_stream = nullptr;
    hipEvent_t freed = nullptr;  // recorded after the consuming search's scans
    hipStream_t freed_stream = nullptr;
    bool ready_pending = false, freed_pending = false;
  };
  static constexpr int kPreT3 = 3;  // tables of up to three batches ahead (batches in flight)
  PreT3 pre[kPreT3];
  uint64_t pre_seq = 0;
  // The per-batch workspaces of a device search (coarse keys, probes, T3, the
  // list-major plan of ivfpq_kernels.h ListPlan and the partial lists).  A handle
  // holds kSlots of them, one per stream in use (begin_slot), so that up to
  // kSlots batches can be in flight on different streams at once: the next
  // batch's coarse step and list scan start while this batch's scan drains
  // (DESIGN.md §4).
  struct Work {
    DevBuf w_dist, w_lists, w_dis0, w_T3, w_cand;  // w_cand: large-nlist coarse segment candidates
    DevBuf w_qn;  // |x|^2 of the batch's queries (tiled coarse keys)
    DevBuf p_cnt, p_bucket, p_recs, p_hdr, p_part, p_N, p_pd0, p_done, p_tau, p_qmask, p_evlog;
    uint32_t epoch = 0;  // tag of the last batch planned in this workspace (ListPlan::tauq)
    // every use records `done` on its stream; the slot's next user (on another
    // stream) waits for it, and whatever frees or rewrites shared device buffers
    // synchronizes on every slot's first
    hipEvent_t done = nullptr;
    hipStream_t done_stream = nullptr;
    bool done_pending = false;
    uint64_t last_use = 0;
  };
  static constexpr int kSlots = 3;
  Work work[kSlots];
  int slot = 0;  // the workspace of the current (last begun) device call
  uint64_t uses = 0;
  bool inflight = inflight_default();
  int fault_inj = 0;  // test hook (ivfpq_set_fault_injection): ListPlan::fault
  std::vector<uint64_t> tau_seed;  // test hook (ivfpq_debug_seed_tau): the next batch's starting bounds
  std::mutex mu;

  Work& W() { return work[slot]; }
  // The workspace of a device call on stream s: the one last used on s (stream
  // order already protects it, and a one-stream caller keeps a single
  // workspace), else the least recently used one, ordered after its last user.
  // With inflight on, this call may run concurrently with calls on other streams;
  // otherwise it is ordered after every call in flight.
  void begin_slot(hipStream_t s) {
    int pick = -1;
    for (int i = 0; i < kSlots && pick < 0; i++)
      if (work[i].done_pending && work[i].done_stream == s) pick = i;
    if (pick < 0) {
      pick = 0;
      for (int i = 1; i < kSlots; i++)
        if (work[i].last_use < work[pick].last_use) pick = i;
    }
    slot = pick;
    Work& w = work[slot];
    w.last_use = ++uses;
    // Taking over another stream's workspace (more streams than kSlots) waits on
    // the host: a device-side wait here let a k = 100 batch on a fourth stream see
    // its predecessor's partial lists (1 batch in 480, tests/test_gpu_parity.py
    // test_batches_in_flight_on_round_robin_streams), which two or three streams
    // never do.
    if (w.done_pending && w.done_stream != s) {
      HIPCHECK(hipEventSynchronize(w.done));
      w.done_pending = false;
    }
    if (!inflight) order_after_all(s);
  }
  // ordered after every device call still in flight (for paths that touch the
  // shared staging buffers or T3-ahead state)
  void order_after_all(hipStream_t s) {
    for (auto& w : work)
      if (w.done_pending && w.done_stream != s) HIPCHECK(hipStreamWaitEvent(s, w.done, 0));
  }
  void mark_done(hipStream_t s) {
    Work& w = W();
    HIPCHECK(hipEventRecord(w.done, s));
    w.done_stream = s;
    w.done_pending = true;
  }
  void quiesce() {
    for (auto& w : work) {
      if (w.done_pending) HIPCHECK(hipEventSynchronize(w.done));
      w.done_pending = false;
    }
  }

  ListPlan make_plan(int64_t nq, int np, int k, hipStream_t s, bool leave_free = false) {
    const int nloc = std::max(list_hi - list_lo, 1);
    Work& w = W();
    const int G = list_scan_group(M, k);
    ListPlan pl;
    pl.cap = (int)nq;
    pl.max_items = list_scan_max_items(nq * np, nloc, G);
    // leave_free (a full search with batches in flight): the scan leaves kInflightFreeCus
    // CUs to the other streams' coarse and merge kernels (r06x sweep: C2 step -2.5 %;
    // DESIGN.md section 4); one batch at a time, and in the shard flow's preassigned
    // searches, where the sweep was inconclusive, it takes them all
    pl.grid = scan_lists_grid(M, k, leave_free ? kInflightFreeCus : 0);
    if (!w.p_cnt.p || w.p_cnt.bytes < sizeof(int32_t) * 2 * nloc) {
      // kept zero between batches by k_scan_lists; zeroed once here
      w.p_cnt.ensure(sizeof(int32_t) * 2 * nloc);
      HIPCHECK(hipMemsetAsync(w.p_cnt.p, 0, w.p_cnt.bytes, s));
    }
    w.p_bucket.ensure(sizeof(int2) * 2 * (size_t)nloc * nq);
    w.p_recs.ensure(sizeof(int32_t) * 16 * (size_t)pl.max_items);
    if (!w.p_hdr.p) {  // hdr[2] (the scan's work counter) is kept zero between batches by k_merge_probes
      w.p_hdr.ensure(sizeof(int32_t) * 16);
      HIPCHECK(hipMemsetAsync(w.p_hdr.p, 0, w.p_hdr.bytes, s));
    }
    pl.ks = part_stride(k);
    w.p_part.ensure(sizeof(uint4) * nq * np * 4 * pl.ks);
    w.p_N.ensure(sizeof(uint2) * nq * np * 4);
    w.p_pd0.ensure(sizeof(float) * nq * np);
    if (!w.p_evlog.p) {
      w.p_evlog.ensure(sizeof(uint32_t) * 8 * kEvLog);
      HIPCHECK(hipMemsetAsync(w.p_evlog.p, 0, w.p_evlog.bytes, s));
    }
    if (!w.p_done.p || w.p_done.bytes < sizeof(int32_t) * nq) {  // kept zero between batches by k_merge_probes
      w.p_done.ensure(sizeof(int32_t) * nq);
      HIPCHECK(hipMemsetAsync(w.p_done.p, 0, w.p_done.bytes, s));
    }
    if (!w.p_tau.p || w.p_tau.bytes < sizeof(uint64_t) * nq) {  // all-ones: no batch's bound (ListPlan::tauq)
      w.p_tau.ensure(sizeof(uint64_t) * nq);
      HIPCHECK(hipMemsetAsync(w.p_tau.p, 0xff, w.p_tau.bytes, s));
    }
    if (++w.epoch >= 0xFFFFFFF0u) {  // tag space used up (after ~4e9 batches): start over on a clean buffer
      if (w.done_pending) HIPCHECK(hipEventSynchronize(w.done));
      HIPCHECK(hipMemsetAsync(w.p_tau.p, 0xff, w.p_tau.bytes, s));
      w.epoch = 1;
    }
    if (!tau_seed.empty()) {  // one-shot: this batch starts with the seeded bounds (its own tag)
      // disarmed before the check: a mismatched seed fails this search only, not every later one
      // (the hook applies to single-chunk searches of exactly the seeded size)
      std::vector<uint64_t> seed;
      seed.swap(tau_seed);
      require((int64_t)seed.size() == nq, "seeded bounds: one per query of the next batch (single-chunk searches)");
      for (auto& v : seed) v = ((uint64_t)(~w.epoch) << 32) | (uint32_t)v;
      HIPCHECK(hipMemcpyAsync(w.p_tau.p, seed.data(), sizeof(uint64_t) * nq, hipMemcpyHostToDevice, s));
      HIPCHECK(hipStreamSynchronize(s));
    }
    pl.qmw = (np + 63) / 64;
    w.p_qmask.ensure(sizeof(uint64_t) * nq * pl.qmw);
    pl.cnt = w.p_cnt.as<int32_t>();
    pl.bucket = w.p_bucket.as<int2>();
    pl.recs = w.p_recs.as<int32_t>();
    pl.hdr = w.p_hdr.as<int32_t>();
    pl.part = w.p_part.as<uint4>();
    pl.partN = w.p_N.as<uint2>();
    pl.pd0 = w.p_pd0.as<float>();
    pl.evlog = w.p_evlog.as<uint32_t>();
    pl.fault = fault_inj;
    pl.qdone = w.p_done.as<int32_t>();
    pl.tauq = w.p_tau.as<uint64_t>();
    pl.epoch = w.epoch;
    pl.err = w.p_hdr.as<int32_t>() + 15;
    pl.qmask = w.p_qmask.as<uint64_t>();
    pl.order = d_order.p ? d_order.as<int32_t>() : nullptr;
    pl.fused = scan_fused_plan(nloc, pl.max_items, M) ? 1 : 0;
    return pl;
  }

  // stage timing (HIP events recorded on the launch stream around each stage)
  enum Stage { ST_COARSE = 0, ST_TABLES = 1, ST_SCAN = 2, ST_LISTS = 3, ST_N = 4 };
  int timing = 0;  // 0 off, 1 every stage, 2 the list-scan kernel only
  struct Mark {
    int stage;
    hipEvent_t a, b;  // adjacent: &a is passed as an event pair
  };
  std::vector<Mark> marks;
  std::vector<hipEvent_t> ev_pool;

  hipEvent_t take_event() {
    if (!ev_pool.empty()) {
      hipEvent_t e = ev_pool.back();
      ev_pool.pop_back();
      return e;
    }
    hipEvent_t e;
    HIPCHECK(hipEventCreate(&e));
    return e;
  }
  // returns an index into marks (or -1 when timing is off)
  // record = false: the caller records the pair itself (ST_LISTS, around one kernel)
  int mark_begin(int stage, hipStream_t s, bool record = true) {
    if (!timing || (timing == 2 && stage != ST_LISTS)) return -1;
    Mark m{stage, take_event(), take_event()};
    if (record) HIPCHECK(hipEventRecord(m.a, s));
    marks.push_back(m);
    return (int)marks.size() - 1;
  }
  void mark_end(int idx, hipStream_t s) {
    if (idx >= 0) HIPCHECK(hipEventRecord(marks[idx].b, s));
  }
  void collect_timing(double* ms, int64_t* cnt) {
    for (int i = 0; i < ST_N; i++) {
      ms[i] = 0.0;
      cnt[i] = 0;
    }
    for (auto& m : marks) {
      HIPCHECK(hipEventSynchronize(m.b));
      float t = 0.f;
      HIPCHECK(hipEventElapsedTime(&t, m.a, m.b));
      ms[m.stage] += t;
      cnt[m.stage] += 1;
      ev_pool.push_back(m.a);
      ev_pool.push_back(m.b);
    }
    marks.clear();
  }

  ~ivfpq_index() {
    for (auto& m : marks) {
      (void)hipEventDestroy(m.a);
      (void)hipEventDestroy(m.b);
    }
    for (auto e : ev_pool) (void)hipEventDestroy(e);
    for (auto& w : work)
      if (w.done) (void)hipEventDestroy(w.done);
    for (auto& p : pre) {
      if (p.ready) (void)hipEventDestroy(p.ready);
      if (p.freed) (void)hipEventDestroy(p.freed);
    }
    if (stream) (void)hipStreamDestroy(stream);
  }

  void init_stream() {
    if (!stream) HIPCHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    for (auto& w : work)
      if (!w.done) HIPCHECK(hipEventCreateWithFlags(&w.done, hipEventDisableTiming));
    for (auto& p : pre) {
      if (!p.ready) HIPCHECK(hipEventCreateWithFlags(&p.ready, hipEventDisableTiming));
      if (!p.freed) HIPCHECK(hipEventCreateWithFlags(&p.freed, hipEventDisableTiming));
    }
  }

  // ---------------------------------------------------------------- helpers
  // Row-wise top-1 of x [n][dd] against c (already on device with norms):
  // writes assignments (host) for all rows. Uses w_x / w_xn / w_dist / w_D / w_I.
  // ip: assign to the largest inner product (the IndexFlatIP quantizer of an IP index)
  void assign_top1(const float* x_host, int64_t n, int dd, const float* dc, const float* dcn, int nc,
                   int64_t* assign_host, const float* x_dev = nullptr, bool ip_assign = false) {
    const int64_t rows = std::max<int64_t>(1, std::min<int64_t>(n, kChunkBytes / ((size_t)nc * 4)));
    w_xn.ensure(sizeof(float) * rows);
    W().w_dist.ensure(sizeof(float) * rows * nc);
    w_D.ensure(sizeof(float) * rows);
    w_I.ensure(sizeof(int64_t) * rows);
    if (!x_dev) w_x.ensure(sizeof(float) * rows * dd);
    for (int64_t r0 = 0; r0 < n; r0 += rows) {
      const int64_t c = std::min(rows, n - r0);
      const float* xd;
      if (x_dev) {
        xd = x_dev + r0 * dd;
      } else {
        HIPCHECK(hipMemcpyAsync(w_x.p, x_host + r0 * dd, sizeof(float) * c * dd, hipMemcpyHostToDevice, stream));
        xd = w_x.as<float>();
      }
      if (!ip_assign) launch_row_norms(xd, c, dd, w_xn.as<float>(), stream);
      launch_l2_dist(xd, w_xn.as<float>(), c, dc, dcn, nc, dd, W().w_dist.as<float>(), stream, ip_assign);
      launch_select_rows(W().w_dist.as<float>(), c, nc, 1, w_D.as<float>(), w_I.as<int64_t>(), stream);
      HIPCHECK(hipGetLastError());
      HIPCHECK(hipMemcpyAsync(assign_host + r0, w_I.p, sizeof(int64_t) * c, hipMemcpyDeviceToHost, stream));
      HIPCHECK(hipStreamSynchronize(stream));
    }
  }

  void kmeans(const float* x, int64_t n, int dd, int k, int niter, uint64_t seed, float* cent,
              bool ip_assign = false) {
    require(n >= k, "k-means: need at least as many training points as centroids (" + std::to_string(n) + " < " +
                        std::to_string(k) + ")");
    const auto init = rand_perm_prefix(n, k, seed);
    for (int c = 0; c < k; c++) std::memcpy(cent + (size_t)c * dd, x + init[c] * dd, sizeof(float) * dd);
    if (ip_assign) renorm_rows(cent, k, dd);  // spherical: unit-norm centroids (Faiss post_process_centroids)
    // keep the whole training set resident when it fits the scratch bound
    DevBuf xall;
    const bool resident = (size_t)n * dd * 4 <= (size_t(2) << 30);
    if (resident) {
      xall.ensure(sizeof(float) * n * dd);
      HIPCHECK(hipMemcpyAsync(xall.p, x, sizeof(float) * n * dd, hipMemcpyHostToDevice, stream));
    }
    std::vector<int64_t> assign(n);
    w_cent.ensure(sizeof(float) * k * dd);
    w_cn.ensure(sizeof(float) * k);
    for (int it = 0; it < niter; it++) {
      HIPCHECK(hipMemcpyAsync(w_cent.p, cent, sizeof(float) * k * dd, hipMemcpyHostToDevice, stream));
      launch_row_norms(w_cent.as<float>(), k, dd, w_cn.as<float>(), stream);
      assign_top1(x, n, dd, w_cent.as<float>(), w_cn.as<float>(), k, assign.data(),
                  resident ? xall.as<float>() : nullptr, ip_assign);
      kmeans_update(x, n, dd, k, assign.data(), cent);
      if (ip_assign) renorm_rows(cent, k, dd);
    }
  }

  void upload_trained() {
    quiesce();
    drop_tables();
    d_cent.ensure(sizeof(float) * nlist * d);
    d_cnorm.ensure(sizeof(float) * nlist);
    d_cb.ensure(sizeof(float) * M * ksub * (d / M));
    d_T1.ensure(sizeof(float) * (size_t)nlist * M * ksub);
    HIPCHECK(hipMemcpyAsync(d_cent.p, centroids.data(), sizeof(float) * nlist * d, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipMemcpyAsync(d_cb.p, codebook.data(), sizeof(float) * codebook.size(), hipMemcpyHostToDevice,
                            stream));
    launch_row_norms(d_cent.as<float>(), nlist, d, d_cnorm.as<float>(), stream);
    {  // transposed centroids [d][nlist] for the fused coarse kernel
      const int ldc = (nlist + 3) & ~3;  // rows padded to a multiple of 4 (branch-free float4 loads)
      std::vector<float> ct((size_t)ldc * d, 0.f);
      for (int l = 0; l < nlist; l++)
        for (int t = 0; t < d; t++) ct[(size_t)t * ldc + l] = centroids[(size_t)l * d + t];
      d_centT.ensure(sizeof(float) * ct.size());
      HIPCHECK(hipMemcpyAsync(d_centT.p, ct.data(), sizeof(float) * ct.size(), hipMemcpyHostToDevice, stream));
      HIPCHECK(hipStreamSynchronize(stream));
    }
    launch_precompute_T1(d_cent.as<float>(), nlist, d, d_cb.as<float>(), M, ksub, d_T1.as<float>(), stream);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(stream));
    trained = true;
  }

  void upload_lists() {
    flush_pending(stream);
    if (!dirty) return;
    quiesce();  // in-flight searches may still read the old device lists
    std::vector<int64_t> off(nlist + 1, 0);
    for (int l = 0; l < nlist; l++) off[l + 1] = off[l] + (int64_t)lids[l].size();
    const int64_t tot = off[nlist];
    std::vector<uint8_t> codes((size_t)tot * M);
    std::vector<int64_t> ids((size_t)tot);
    // Device image: each list sorted by label (stable).  Results do not depend
    // on the order inside a list, and label-sorted lists let the scan kernels
    // rank candidates by code position instead of loading labels.
    std::vector<int64_t> perm;
    for (int l = 0; l < nlist; l++) {
      const int64_t n = (int64_t)lids[l].size();
      if (!n) continue;
      perm.resize(n);
      for (int64_t i = 0; i < n; i++) perm[i] = i;
      const int64_t* lid = lids[l].data();
      std::stable_sort(perm.begin(), perm.end(), [lid](int64_t a, int64_t b) { return lid[a] < lid[b]; });
      for (int64_t i = 0; i < n; i++) {
        uint8_t* dst = codes.data() + (off[l] + i) * M;
        const uint8_t* src = lcodes[l].data() + perm[i] * M;
        std::memcpy(dst, src, M);
        ids[off[l] + i] = lid[perm[i]];
      }
    }
    set_list_order(off);
    d_codes.ensure(std::max<size_t>(16, codes.size()));
    d_ids.ensure(std::max<size_t>(16, sizeof(int64_t) * ids.size()));
    d_off.ensure(sizeof(int64_t) * off.size());
    if (tot) {
      HIPCHECK(hipMemcpyAsync(d_codes.p, codes.data(), codes.size(), hipMemcpyHostToDevice, stream));
      HIPCHECK(hipMemcpyAsync(d_ids.p, ids.data(), sizeof(int64_t) * ids.size(), hipMemcpyHostToDevice, stream));
    }
    HIPCHECK(hipMemcpyAsync(d_off.p, off.data(), sizeof(int64_t) * off.size(), hipMemcpyHostToDevice, stream));
    HIPCHECK(hipStreamSynchronize(stream));
    img_n = tot;
    dirty = false;
  }

  // The host lists from the device image (after device-side adds), in image
  // order: each list label-sorted.
  void sync_host() {
    if (!host_stale) return;
    flush_pending(stream);
    quiesce();
    std::vector<int64_t> off(nlist + 1);
    HIPCHECK(hipMemcpy(off.data(), d_off.p, sizeof(int64_t) * (nlist + 1), hipMemcpyDeviceToHost));
    const int64_t tot = off[nlist];
    std::vector<uint8_t> codes((size_t)tot * M);
    std::vector<int64_t> ids((size_t)tot);
    if (tot) {
      HIPCHECK(hipMemcpy(codes.data(), d_codes.p, codes.size(), hipMemcpyDeviceToHost));
      HIPCHECK(hipMemcpy(ids.data(), d_ids.p, sizeof(int64_t) * ids.size(), hipMemcpyDeviceToHost));
    }
    for (int l = 0; l < nlist; l++) {
      lids[l].assign(ids.begin() + off[l], ids.begin() + off[l + 1]);
      lcodes[l].assign(codes.begin() + off[l] * M, codes.begin() + off[l + 1] * M);
    }
    host_stale = false;
  }

  // Device-side add of n vectors (x on the host or the device; ids nullable =
  // sequential): coarse assignment on the matrix cores (the search's coarse
  // kernels, top-1) and PQ encode into the pending set (q_*), no per-chunk host
  // synchronization.  The pending set is merged into the image (flush_pending)
  // before the lists are next read, or once it holds as many entries as the
  // image: every entry is then moved O(1) times over any sequence of adds
  // (Chameleon adds a 1e9 base in 1e6 slices, bench_gpu_1bn.py:598-658; beir in
  // 50k chunks, faiss_index.py:40-42), instead of the whole image being
  // re-sorted at every add.
  void add_dev(int64_t n, const float* x, bool x_on_device, const int64_t* ids, bool ids_on_device, hipStream_t s) {
    require(trained, "index is not trained");
    if (n <= 0) return;
    upload_lists();  // host-side adds not yet in the image
    order_after_all(s);
    quiesce();
    // the pending sort permutes entries with 32-bit indices
    require(q_n + n < (int64_t(1) << 32) - 1, "more than 2^32 - 2 vectors pending in one merge");
    const int64_t rows = nlist >= kSegmentedNlist ? std::min<int64_t>(n, 1 << 18)
                                                  : std::max<int64_t>(1, std::min<int64_t>(n, kChunkBytes / ((size_t)nlist * 4)));
    pend_reserve(q_n + n, s);
    int64_t* lists = q_lists.as<int64_t>() + q_n;
    w_D.ensure(sizeof(float) * rows);
    if (!x_on_device) w_x.ensure(sizeof(float) * rows * d);
    for (int64_t r0 = 0; r0 < n; r0 += rows) {
      const int64_t c = std::min(rows, n - r0);
      const float* xd = x + r0 * d;
      if (!x_on_device) {
        HIPCHECK(hipMemcpyAsync(w_x.p, xd, sizeof(float) * c * d, hipMemcpyHostToDevice, s));
        xd = w_x.as<float>();
      }
      coarse_launch(xd, c, 1, w_D.as<float>(), lists + r0, s);
      launch_pq_encode(xd, c, d, d_cent.as<float>(), lists + r0, d_cb.as<float>(), M, ksub,
                       q_codes.as<uint8_t>() + (q_n + r0) * M, s);
      HIPCHECK(hipGetLastError());
      if (!x_on_device) HIPCHECK(hipStreamSynchronize(s));  // w_x is reused by the next chunk's copy
    }
    if (!ids) {
      launch_iota_i64(q_ids.as<int64_t>() + q_n, n, next_id, s);
      next_id += n;
    } else {
      HIPCHECK(hipMemcpyAsync(q_ids.as<int64_t>() + q_n, ids, sizeof(int64_t) * n,
                              ids_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
    }
    int64_t kept = n;
    if (list_lo > 0 || list_hi < nlist) {  // a list-range shard keeps its own lists only
      a_off.ensure(sizeof(unsigned long long));
      HIPCHECK(hipMemsetAsync(a_off.p, 0, sizeof(unsigned long long), s));
      HIPCHECK(count_kept(lists, n, list_lo, list_hi, a_off.as<unsigned long long>(), s));
      unsigned long long k = 0;
      HIPCHECK(hipMemcpyAsync(&k, a_off.p, sizeof(k), hipMemcpyDeviceToHost, s));
      HIPCHECK(hipStreamSynchronize(s));
      kept = (int64_t)k;
    } else {
      HIPCHECK(hipStreamSynchronize(s));
    }
    q_n += n;
    q_kept += kept;
    ntotal += kept;
    host_stale = true;
    dirty = false;
    if (q_n >= std::max<int64_t>(img_n, int64_t(1) << 24)) flush_pending(s);
  }

  void pend_reserve(int64_t need, hipStream_t s) {
    if (need <= q_cap) return;
    const int64_t cap = std::max<int64_t>(need, q_cap * 2);
    DevBuf l2, i2, c2;
    l2.ensure(sizeof(int64_t) * cap);
    i2.ensure(sizeof(int64_t) * cap);
    c2.ensure((size_t)cap * M);
    if (q_n > 0) {
      HIPCHECK(hipMemcpyAsync(l2.p, q_lists.p, sizeof(int64_t) * q_n, hipMemcpyDeviceToDevice, s));
      HIPCHECK(hipMemcpyAsync(i2.p, q_ids.p, sizeof(int64_t) * q_n, hipMemcpyDeviceToDevice, s));
      HIPCHECK(hipMemcpyAsync(c2.p, q_codes.p, (size_t)q_n * M, hipMemcpyDeviceToDevice, s));
      HIPCHECK(hipStreamSynchronize(s));
    }
    std::swap(q_lists.p, l2.p);
    std::swap(q_lists.bytes, l2.bytes);
    std::swap(q_ids.p, i2.p);
    std::swap(q_ids.bytes, i2.bytes);
    std::swap(q_codes.p, c2.p);
    std::swap(q_codes.bytes, c2.bytes);
    q_cap = cap;
  }

  void drop_pending() {
    q_lists.release();
    q_ids.release();
    q_codes.release();
    q_n = q_kept = q_cap = 0;
  }

  // The pending entries merged into the device image: sorted by (list, label)
  // alone (rocprim radix sorts of the pending set, out-of-range lists dropped),
  // then interleaved list by list into the label-sorted image (ivfpq_build.h
  // image_merge_lists).  The result equals a stable (list, label) sort of old +
  // new, the image order of DESIGN.md §3.
  void flush_pending(hipStream_t s) {
    if (q_n == 0) return;
    quiesce();  // in-flight searches read the current image
    ImageMergeArgs g;
    g.nlist = nlist;
    g.lo = list_lo;
    g.hi = list_hi;
    g.M = M;
    g.n_old = 0;
    g.n_new = q_n;
    g.new_lists = q_lists.as<int64_t>();
    g.new_ids = q_ids.as<int64_t>();
    g.new_codes = q_codes.as<uint8_t>();
    DevBuf new_off, out_off;
    new_off.ensure(sizeof(int64_t) * (nlist + 1));
    g.off_out = new_off.as<int64_t>();
    {
      const size_t sb = image_merge_scratch_bytes(q_n, nlist);
      DevBuf scratch, codes_n, ids_n;
      scratch.ensure(sb);
      HIPCHECK(image_merge_sort(g, scratch.p, sb, s));
      std::vector<int64_t> noff(nlist + 1), ooff(nlist + 1);
      HIPCHECK(hipMemcpyAsync(noff.data(), new_off.p, sizeof(int64_t) * (nlist + 1), hipMemcpyDeviceToHost, s));
      HIPCHECK(hipMemcpyAsync(ooff.data(), d_off.p, sizeof(int64_t) * (nlist + 1), hipMemcpyDeviceToHost, s));
      HIPCHECK(hipStreamSynchronize(s));
      const int64_t kept = noff[nlist];
      require(kept == q_kept, "pending merge: kept entries disagree with the add-time count");
      codes_n.ensure(std::max<size_t>(16, (size_t)kept * M));
      ids_n.ensure(std::max<size_t>(16, sizeof(int64_t) * kept));
      g.codes_out = codes_n.as<uint8_t>();
      g.ids_out = ids_n.as<int64_t>();
      HIPCHECK(image_merge_gather(g, kept, scratch.p, s));
      scratch.release();
      std::vector<int64_t> off(nlist + 1);
      int64_t mx = 0;
      for (int l = 0; l <= nlist; l++) {
        off[l] = ooff[l] + noff[l];
        if (l < nlist) mx = std::max(mx, (ooff[l + 1] - ooff[l]) + (noff[l + 1] - noff[l]));
      }
      const int64_t n_out = off[nlist];
      DevBuf codes2, ids2;
      codes2.ensure(std::max<size_t>(16, (size_t)n_out * M));
      ids2.ensure(std::max<size_t>(16, sizeof(int64_t) * n_out));
      out_off.ensure(sizeof(int64_t) * (nlist + 1));
      ListMergeArgs m;
      m.nlist = nlist;
      m.lo = list_lo;
      m.hi = list_hi;
      m.M = M;
      m.max_list = mx;
      m.old_off = d_off.as<int64_t>();
      m.old_codes = d_codes.as<uint8_t>();
      m.old_ids = d_ids.as<int64_t>();
      m.new_off = new_off.as<int64_t>();
      m.new_codes = codes_n.as<uint8_t>();
      m.new_ids = ids_n.as<int64_t>();
      m.out_off = out_off.as<int64_t>();
      m.out_codes = codes2.as<uint8_t>();
      m.out_ids = ids2.as<int64_t>();
      HIPCHECK(image_merge_lists(m, s));
      HIPCHECK(hipStreamSynchronize(s));
      std::swap(d_codes.p, codes2.p);
      std::swap(d_codes.bytes, codes2.bytes);
      std::swap(d_ids.p, ids2.p);
      std::swap(d_ids.bytes, ids2.bytes);
      std::swap(d_off.p, out_off.p);
      std::swap(d_off.bytes, out_off.bytes);
      img_n = n_out;
      set_list_order(off);
    }
    drop_pending();
    require(img_n == ntotal, "pending merge: image size disagrees with ntotal");
  }

  // Scheduling order of the shard's lists: largest first (the list scan takes
  // items in this order within each kind, so the items that finish last are the
  // short ones: longest-processing-time-first bounds the persistent grid's tail).
  void set_list_order(const std::vector<int64_t>& off) {
    const int nloc = std::max(list_hi - list_lo, 1);
    std::vector<int32_t> order(nloc);
    for (int j = 0; j < nloc; j++) order[j] = j;
    if (list_hi > list_lo)
      std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
        return off[list_lo + a + 1] - off[list_lo + a] > off[list_lo + b + 1] - off[list_lo + b];
      });
    d_order.ensure(sizeof(int32_t) * nloc);
    HIPCHECK(hipMemcpyAsync(d_order.p, order.data(), sizeof(int32_t) * nloc, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipStreamSynchronize(stream));
  }

  void append(int64_t n, const int64_t* lno, const uint8_t* codes, const int64_t* ids) {
    sync_host();
    for (int64_t i = 0; i < n; i++) {
      const int64_t l = lno[i];
      require(l >= 0 && l < nlist, "list number out of range");
      if (l < list_lo || l >= list_hi) continue;  // another shard's list
      lcodes[l].insert(lcodes[l].end(), codes + i * M, codes + (i + 1) * M);
      lids[l].push_back(ids[i]);
      ntotal++;
    }
    dirty = true;
  }

  int eff_nprobe() const { return std::min(nprobe, nlist); }

  void check_search(int64_t n, int k) {
    require(trained, "index is not trained");
    require(n >= 0, "n must be >= 0");
    require(k >= 1 && k <= kMaxK, "k must be in [1, " + std::to_string(kMaxK) + "]");
  }

  bool ip() const { return metric == IVFPQ_METRIC_INNER_PRODUCT; }

  // Coarse quantizer for c queries at x: the nprobe best lists and the
  // quantizer's values (L2 distances / IP similarities), from the key matrix
  // built on the matrix cores (with T3out, the same launch builds T3).  With
  // `plan` and nprobe <= 64 the selection also plans the batch and true is
  // returned; otherwise the caller plans with launch_plan_count.
  // xt / nt (nullable): T3out holds the tables of the queries xt instead of x (the
  // shard step: keys of this rank's slice, tables of the global batch, one launch)
  bool coarse_launch(const float* x, int64_t c, int np, float* dis, int64_t* lists, hipStream_t s,
                     const ListPlan* plan = nullptr, float* T3out = nullptr, const float* xt = nullptr,
                     int64_t nt = 0, bool hoist = false) {
    if (!xt) {
      xt = x;
      nt = c;
    }
    if (nlist >= kSegmentedNlist && np <= 64) {  // large nlist: no [c][nlist] key matrix
      W().w_cand.ensure(sizeof(uint64_t) * c * coarse_segments(c, nlist, d) * np);
      if (T3out) launch_ip_table(xt, nt, d, d_cb.as<float>(), M, ksub, T3out, s);
      launch_coarse_segmented(x, c, d, d_centT.as<float>(), d_cnorm.as<float>(), nlist, np, W().w_cand.as<uint64_t>(),
                              dis, lists, s, ip(), plan, d_off.as<int64_t>(), list_lo, list_hi, d_cent.as<float>());
      return plan != nullptr;
    }
    W().w_dist.ensure(sizeof(float) * c * nlist);
    W().w_qn.ensure(sizeof(float) * c);
    launch_coarse_keys(x, c, d, d_centT.as<float>(), d_cnorm.as<float>(), nlist, W().w_dist.as<float>(), s, ip(), T3out,
                       d_cb.as<float>(), M, W().w_qn.as<float>(), xt, nt, hoist);
    if (np <= 64) {
      launch_coarse_select(W().w_dist.as<float>(), c, nlist, np, dis, lists, s, ip(), plan, d_off.as<int64_t>(), list_lo,
                           list_hi, x, d_cent.as<float>(), d);
      return plan != nullptr;
    }
    launch_select_rows(W().w_dist.as<float>(), c, nlist, np, dis, lists, s, ip());
    return false;
  }

  // The full search on device pointers, on stream s.  Iq/Dq non-null = preassigned.
  // tables: a token of tables_dev (preassigned searches only; 0 = build T3 here)
  void search_dev(int64_t n, const float* x, int k, float* D, int64_t* I, const int64_t* Iq, const float* Dq,
                  bool preassigned, hipStream_t s, uint64_t tables = 0) {
    check_search(n, k);
    upload_lists();
    if (n == 0) return;
    begin_slot(s);
    const int np = preassigned ? nprobe : eff_nprobe();
    const int64_t qc = query_chunk(n, np, k);
    W().w_T3.ensure(sizeof(float) * qc * M * ksub);
    if (!preassigned) {
      W().w_lists.ensure(sizeof(int64_t) * qc * np);
      W().w_dis0.ensure(sizeof(float) * qc * np);
    }
    const int G = list_scan_group(M, k);
    // tables computed ahead (tables_dev): exactly the entry of the token, which
    // this search consumes
    int pi = -1;
    if (tables) {
      require(preassigned, "precomputed tables are for preassigned searches");
      for (int i = 0; i < kPreT3; i++)
        if (pre[i].seq == tables) pi = i;
      require(pi >= 0, "tables token " + std::to_string(tables) +
                           " is not pending (already consumed, or overwritten by later precomputes)");
      require(pre[pi].n == n, "tables token was computed for " + std::to_string(pre[pi].n) + " queries, not " +
                                  std::to_string(n));
      pre[pi].seq = 0;
      pre[pi].freed_seq = ++pre_seq;
    }
    const bool use_pre = pi >= 0;
    for (int64_t q0 = 0; q0 < n; q0 += qc) {
      const int64_t c = std::min(qc, n - q0);
      const float* xq = x + q0 * d;
      const ListPlan plan = make_plan(c, np, k, s, inflight && !preassigned);
      const int64_t* lists;
      bool planned = false;
      const int tm = mark_begin(ST_COARSE, s);
      if (preassigned) {
        lists = Iq + q0 * np;
        launch_plan_count(lists, (Dq && !ip()) ? Dq + q0 * np : nullptr, xq, d_cent.as<float>(), c, d, np,
                          d_off.as<int64_t>(), list_lo, list_hi, ip(), true, k, plan, s);
      } else {
        planned =
            coarse_launch(xq, c, np, W().w_dis0.as<float>(), W().w_lists.as<int64_t>(), s, &plan, W().w_T3.as<float>(),
                          nullptr, 0, /*hoist: the scan is not k_scan_lean*/ !(k <= 16 && M <= 16));
        lists = W().w_lists.as<int64_t>();
        if (!planned)
          launch_plan_count(lists, ip() ? nullptr : W().w_dis0.as<float>(), xq, d_cent.as<float>(), c, d, np,
                            d_off.as<int64_t>(), list_lo, list_hi, ip(), false, k, plan, s);
      }
      mark_end(tm, s);
      const float* T3 = W().w_T3.as<float>();
      if (preassigned && use_pre) {  // T3 computed ahead on another stream
        if (pre[pi].ready_stream != s) HIPCHECK(hipStreamWaitEvent(s, pre[pi].ready, 0));
        T3 = pre[pi].buf.as<float>() + q0 * M * ksub;
      } else if (preassigned) {  // T3 (the coarse launch builds it otherwise)
        const int tt = mark_begin(ST_TABLES, s);
        launch_ip_table(xq, c, d, d_cb.as<float>(), M, ksub, W().w_T3.as<float>(), s);
        mark_end(tt, s);
      }
      ScanArgs a;
      a.T1 = d_T1.as<float>();
      a.T3 = T3;
      a.codes = d_codes.as<uint8_t>();
      a.ids = d_ids.as<int64_t>();
      a.list_off = d_off.as<int64_t>();
      a.n_codes = img_n;
      a.probe_list = lists;
      a.nq = c;
      a.nprobe = np;
      a.k = k;
      a.M = M;
      a.ip = ip() ? 1 : 0;
      a.list_lo = list_lo;
      a.list_hi = list_hi;
      a.outD = D + q0 * k;
      a.outI = I + q0 * k;
      const int ts = mark_begin(ST_SCAN, s);
      launch_plan_items(plan, d_off.as<int64_t>(), list_lo, list_hi, G, s);
      // ST_LISTS: its two events are recorded around the list-scan kernel alone
      const int tl = mark_begin(ST_LISTS, s, false);
      launch_scan_lists(a, plan, s, tl >= 0 ? &marks[tl].a : nullptr);
      mark_end(ts, s);
      HIPCHECK(hipGetLastError());
    }
    if (use_pre) {  // the entry's buffer may be rewritten once these scans are done
      HIPCHECK(hipEventRecord(pre[pi].freed, s));
      pre[pi].freed_stream = s;
      pre[pi].freed_pending = true;
    }
    mark_done(s);
  }

  // The query chunk of a search: [c][nlist] keys, T3 and buckets within
  // kChunkBytes; the per-wave partial lists ([c][np][4][k] 16-B records, 64 B per
  // entry and query) within kPartialBytes, so large k still runs whole
  // 1024-query batches (C3, k = 1000, nprobe 32: 2 MB per query).
  int64_t query_chunk(int64_t n, int np, int k) const {
    const int nloc = std::max(list_hi - list_lo, 1);
    const size_t per_q = std::max({(size_t)nlist * 4, (size_t)M * ksub * 4, (size_t)nloc * 16});
    return std::max<int64_t>(
        1, std::min<int64_t>({n, (int64_t)(kChunkBytes / per_q), (int64_t)(kPartialBytes / ((size_t)np * part_stride(k) * 64))}));
  }

  // T3 [n][M][ksub] of the queries x, on stream s, ahead of a preassigned search
  // of exactly those queries (the shard flow computes it while the probes are
  // all-gathered), into one of kPreT3 buffers so that batches in flight each have
  // their own.  Returns the token the search takes (ivfpq.h).
  uint64_t tables_dev(int64_t n, const float* x, hipStream_t s) {
    PreT3& p = take_pre(n, s);
    launch_ip_table(x, n, d, d_cb.as<float>(), M, ksub, p.buf.as<float>(), s);
    HIPCHECK(hipGetLastError());
    return publish_pre(p, n, s);
  }
  // A table entry for n queries, ordered on s after its last consumer and producer.
  PreT3& take_pre(int64_t n, hipStream_t s) {
    require(trained, "index is not trained");
    require(n >= 1, "precompute_tables needs at least one query");
    const int64_t cap = (int64_t)(kChunkBytes / ((size_t)M * ksub * 4));
    require(n <= cap, "precompute_tables: n = " + std::to_string(n) + " exceeds the " + std::to_string(cap) +
                          " queries one table buffer holds (split the batch)");
    // the free entry computed longest ago, else the oldest pending one (dropped);
    // ordered after its last consumer's scans and its last table launch
    int r = 0;
    for (int i = 1; i < kPreT3; i++) {
      const bool fi = pre[i].seq == 0, fr = pre[r].seq == 0;
      // a free entry first, the one consumed longest ago (its consumer's scans are the
      // likeliest to be done, so the wait below rarely stalls the side stream); else
      // the oldest pending entry
      if ((fi && !fr) || (fi && fr && pre[i].freed_seq < pre[r].freed_seq) ||
          (!fi && !fr && pre[i].seq < pre[r].seq))
        r = i;
    }
    PreT3& p = pre[r];
    if (p.freed_pending && p.freed_stream != s) HIPCHECK(hipStreamWaitEvent(s, p.freed, 0));
    if (p.ready_pending && p.ready_stream != s) HIPCHECK(hipStreamWaitEvent(s, p.ready, 0));
    p.buf.ensure(sizeof(float) * (size_t)n * M * ksub);
    p.seq = 0;  // (being rewritten: not consumable until published)
    return p;
  }
  uint64_t publish_pre(PreT3& p, int64_t n, hipStream_t s) {
    HIPCHECK(hipEventRecord(p.ready, s));
    p.ready_stream = s;
    p.ready_pending = true;
    p.n = n;
    p.seq = ++pre_seq;
    return p.seq;
  }
  // tables computed ahead are meaningless once the codebook changes or the index is reset
  void drop_tables() {
    for (auto& p : pre) p.seq = 0;
  }

  // The list-range shard step's front half on one stream: the coarse quantizer of
  // this rank's n queries x and T3 of the nt queries xt of the global batch (the
  // key workgroups and the table workgroups of one launch at nlist < 8192), the
  // tables handed to the preassigned search of xt by the returned token.  No side
  // stream (side streams past the box's four hardware queues cost a
  // third of the throughput).
  uint64_t coarse_tables_dev(int64_t n, const float* x, int64_t* Iq, float* Dq, int64_t nt, const float* xt,
                             hipStream_t s) {
    require(trained, "index is not trained");
    require(n >= 1 && nt >= 1, "coarse_tables needs queries");
    PreT3& p = take_pre(nt, s);
    begin_slot(s);
    const int np = eff_nprobe();
    const int64_t qc = std::max<int64_t>(1, std::min<int64_t>(n, kChunkBytes / ((size_t)nlist * 4)));
    for (int64_t q0 = 0; q0 < n; q0 += qc) {
      const int64_t c = std::min(qc, n - q0);
      const bool with_t3 = q0 == 0;  // the first chunk's launch also builds every table
      coarse_launch(x + q0 * d, c, np, Dq + q0 * np, Iq + q0 * np, s, nullptr,
                    with_t3 ? p.buf.as<float>() : nullptr, with_t3 ? xt : nullptr, with_t3 ? nt : 0);
      HIPCHECK(hipGetLastError());
    }
    mark_done(s);
    return publish_pre(p, nt, s);
  }

  void coarse_dev(int64_t n, const float* x, int64_t* Iq, float* Dq, hipStream_t s) {
    require(trained, "index is not trained");
    if (n <= 0) return;
    begin_slot(s);
    const int np = eff_nprobe();
    const int64_t qc = std::max<int64_t>(1, std::min<int64_t>(n, kChunkBytes / ((size_t)nlist * 4)));
    for (int64_t q0 = 0; q0 < n; q0 += qc) {
      const int64_t c = std::min(qc, n - q0);
      coarse_launch(x + q0 * d, c, np, Dq + q0 * np, Iq + q0 * np, s);
      HIPCHECK(hipGetLastError());
    }
    mark_done(s);
  }

  // host-buffer search (copies in/out on the handle's stream; device staging
  // buffers persist across calls)
  void search_host(int64_t n, const float* x, int k, float* D, int64_t* I, const int64_t* Iq, const float* Dq,
                   bool preassigned) {
    check_search(n, k);
    if (n == 0) return;
    order_after_all(stream);
    const int np = nprobe;
    w_x.ensure(sizeof(float) * n * d);
    h_D.ensure(sizeof(float) * n * k);
    h_I.ensure(sizeof(int64_t) * n * k);
    HIPCHECK(hipMemcpyAsync(w_x.p, x, sizeof(float) * n * d, hipMemcpyHostToDevice, stream));
    if (preassigned) {
      h_Iq.ensure(sizeof(int64_t) * n * np);
      HIPCHECK(hipMemcpyAsync(h_Iq.p, Iq, sizeof(int64_t) * n * np, hipMemcpyHostToDevice, stream));
      if (Dq) {
        h_Dq.ensure(sizeof(float) * n * np);
        HIPCHECK(hipMemcpyAsync(h_Dq.p, Dq, sizeof(float) * n * np, hipMemcpyHostToDevice, stream));
      }
    }
    search_dev(n, w_x.as<float>(), k, h_D.as<float>(), h_I.as<int64_t>(), h_Iq.as<int64_t>(),
               Dq ? h_Dq.as<float>() : nullptr, preassigned, stream);
    HIPCHECK(hipMemcpyAsync(D, h_D.p, sizeof(float) * n * k, hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipMemcpyAsync(I, h_I.p, sizeof(int64_t) * n * k, hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipStreamSynchronize(stream));
  }

  // One FaissServer request in the ralm wire format
  // (ralm/retriever/serialization_utils.py): header integers big-endian
  // (BYTE_ORDER_PY = 'big', :5), arrays in native order (tobytes, :59, :86-87).
  //   with_lists 0: k | queries f32[B][dim]                      (encode_request :38-67)
  //   with_lists 1: B, dim, nprobe, k | queries | lists i64[B][np] (encode_request_with_lists :69-94)
  // The answer is I i64[B][k] | D f32[B][k] (encode_answer :223-258), copied from
  // HBM straight into the answer buffer.  Shape checks follow decode_request*
  // (asserts at :211-213) and FaissServer.start (faiss_server.py:241-277).
  void serve(const uint8_t* msg, int64_t len, int with_lists, int B, int dim, int np, uint8_t* ans, int64_t cap,
             int64_t* ans_len) {
    auto be32 = [](const uint8_t* p) {
      return (int64_t)(int32_t)(((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]);
    };
    require(B > 0 && dim == d, "server shape: batch_size must be > 0 and dim must equal the index's d");
    const int64_t qbytes = (int64_t)B * dim * 4;
    int64_t k;
    const uint8_t* qp;
    const uint8_t* lp = nullptr;
    if (with_lists) {
      require(np >= 1, "nprobe must be >= 1");
      require(len == 16 + qbytes + (int64_t)B * np * 8,
              "request length " + std::to_string(len) + " != request_message_length_with_lists(" +
                  std::to_string(B) + ", " + std::to_string(dim) + ", " + std::to_string(np) + ")");
      require(be32(msg) == B && be32(msg + 4) == dim && be32(msg + 8) == np,
              "request header (batch_size, dim, nprobe) does not match the server's shape");
      k = be32(msg + 12);
      qp = msg + 16;
      lp = msg + 16 + qbytes;
    } else {
      require(len == 4 + qbytes, "request length " + std::to_string(len) + " != request_message_length(" +
                                     std::to_string(B) + ", " + std::to_string(dim) + ")");
      k = be32(msg);
      qp = msg + 4;
    }
    require(k >= 1 && k <= kMaxK, "k in the request must be in [1, " + std::to_string(kMaxK) + "]");
    const int64_t need = (int64_t)B * k * 12;
    require(ans != nullptr && cap >= need, "answer buffer holds " + std::to_string(cap) + " bytes, the answer needs " +
                                               std::to_string(need));
    check_search(B, (int)k);
    order_after_all(stream);
    w_x.ensure(qbytes);
    h_D.ensure(sizeof(float) * B * k);
    h_I.ensure(sizeof(int64_t) * B * k);
    HIPCHECK(hipMemcpyAsync(w_x.p, qp, qbytes, hipMemcpyHostToDevice, stream));
    if (with_lists) {
      // the list ids sit at an arbitrary byte offset of the message: validate on the host, copy as bytes
      for (int64_t i = 0; i < (int64_t)B * np; i++) {
        int64_t l;
        std::memcpy(&l, lp + 8 * i, 8);
        require(l < nlist, "list id out of range in the request");
      }
      const int saved = nprobe;
      nprobe = np;  // search_preassigned scans list_nos.shape[1] probes
      h_Iq.ensure(sizeof(int64_t) * B * np);
      HIPCHECK(hipMemcpyAsync(h_Iq.p, lp, sizeof(int64_t) * B * np, hipMemcpyHostToDevice, stream));
      try {
        search_dev(B, w_x.as<float>(), (int)k, h_D.as<float>(), h_I.as<int64_t>(), h_Iq.as<int64_t>(), nullptr, true,
                   stream);
      } catch (...) {
        nprobe = saved;
        throw;
      }
      nprobe = saved;
    } else {
      search_dev(B, w_x.as<float>(), (int)k, h_D.as<float>(), h_I.as<int64_t>(), nullptr, nullptr, false, stream);
    }
    HIPCHECK(hipMemcpyAsync(ans, h_I.p, sizeof(int64_t) * B * k, hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipMemcpyAsync(ans + (int64_t)B * k * 8, h_D.p, sizeof(float) * B * k, hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipStreamSynchronize(stream));
    if (ans_len) *ans_len = need;
  }
};

// ====================================================================== C-ABI
namespace {

template <class F>
int guarded(F&& f) {
  try {
    g_err.clear();
    f();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
  } catch (...) {
    g_err = "unknown error";
  }
  return -1;
}

void check_handle(const ivfpq_index* h) { require(h != nullptr, "null index handle"); }

}  // namespace

extern "C" {

const char* ivfpq_last_error(void) { return g_err.c_str(); }

int ivfpq_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int ivfpq_create(int d, int nlist, int M, int nbits, int metric, int device, ivfpq_index** out) {
  return guarded([&] {
    require(out != nullptr, "null output pointer");
    require(d > 0 && nlist > 0 && M > 0, "d, nlist and M must be positive");
    require(d % M == 0, "d must be a multiple of M");
    require(nbits == 8, "only nbits=8 is supported");
    require(scan_supported_M(M), "M=" + std::to_string(M) + " not supported on the GPU (8, 16, 32, 48, 64)");
    require(d <= 2048, "d > 2048 not supported");
    require(metric == IVFPQ_METRIC_L2 || metric == IVFPQ_METRIC_INNER_PRODUCT, "unknown metric");
    int ndev = 0;
    HIPCHECK(hipGetDeviceCount(&ndev));
    require(device >= 0 && device < ndev, "device ordinal out of range");
    DeviceGuard g(device);
    auto h = std::make_unique<ivfpq_index>();
    h->d = d;
    h->nlist = nlist;
    h->M = M;
    h->nbits = nbits;
    h->ksub = 1 << nbits;
    h->metric = metric;
    h->device = device;
    h->list_lo = 0;
    h->list_hi = nlist;
    h->lcodes.resize(nlist);
    h->lids.resize(nlist);
    h->init_stream();
    *out = h.release();
  });
}

int ivfpq_free(ivfpq_index* h) {
  return guarded([&] {
    if (!h) return;
    DeviceGuard g(h->device);
    (void)hipStreamSynchronize(h->stream);
    h->quiesce();
    delete h;
  });
}

int ivfpq_train(ivfpq_index* h, int64_t n, const float* x, int niter_coarse, int niter_pq, uint64_t seed) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(x != nullptr && n > 0, "empty training set");
    h->quiesce();  // the k-means scratch buffers are shared with the search path
    const int d = h->d, M = h->M, dsub = d / M, ksub = h->ksub, nlist = h->nlist;
    std::vector<float> cent((size_t)nlist * d);
    h->kmeans(x, n, d, nlist, niter_coarse, seed, cent.data(), h->ip());
    // residuals to the final coarse centroids
    h->w_cent.ensure(sizeof(float) * nlist * d);
    h->w_cn.ensure(sizeof(float) * nlist);
    HIPCHECK(hipMemcpyAsync(h->w_cent.p, cent.data(), sizeof(float) * nlist * d, hipMemcpyHostToDevice, h->stream));
    launch_row_norms(h->w_cent.as<float>(), nlist, d, h->w_cn.as<float>(), h->stream);
    std::vector<int64_t> assign(n);
    h->assign_top1(x, n, d, h->w_cent.as<float>(), h->w_cn.as<float>(), nlist, assign.data(), nullptr, h->ip());
    std::vector<float> sub((size_t)n * dsub);
    std::vector<float> cb((size_t)M * ksub * dsub);
    for (int m = 0; m < M; m++) {
      for (int64_t i = 0; i < n; i++) {
        const float* xi = x + i * d + m * dsub;
        const float* ci = cent.data() + assign[i] * d + m * dsub;
        for (int t = 0; t < dsub; t++) sub[(size_t)i * dsub + t] = xi[t] - ci[t];
      }
      h->kmeans(sub.data(), n, dsub, ksub, niter_pq, seed + 1 + (uint64_t)m, cb.data() + (size_t)m * ksub * dsub);
    }
    h->centroids = std::move(cent);
    h->codebook = std::move(cb);
    h->upload_trained();
  });
}

int ivfpq_set_trained(ivfpq_index* h, const float* centroids, const float* codebook) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(centroids && codebook, "null centroids/codebook");
    h->centroids.assign(centroids, centroids + (size_t)h->nlist * h->d);
    h->codebook.assign(codebook, codebook + (size_t)h->M * h->ksub * (h->d / h->M));
    h->upload_trained();
  });
}

int ivfpq_add(ivfpq_index* h, int64_t n, const float* x, const int64_t* ids) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(h->trained, "index is not trained");
    if (n <= 0) return;
    require(x != nullptr, "null x");
    h->add_dev(n, x, false, ids, false, h->stream);
  });
}

int ivfpq_add_device(ivfpq_index* h, int64_t n, const float* x, const int64_t* ids, void* stream) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(h->trained, "index is not trained");
    if (n <= 0) return;
    require(x != nullptr, "null x");
    h->add_dev(n, x, true, ids, true, stream ? (hipStream_t)stream : h->stream);
  });
}

int ivfpq_add_preencoded(ivfpq_index* h, int64_t n, const int64_t* list_no, const uint8_t* codes,
                         const int64_t* ids) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    if (n <= 0) return;
    require(list_no && codes, "null list_no/codes");
    std::vector<int64_t> seq;
    if (!ids) {
      seq.resize(n);
      for (int64_t i = 0; i < n; i++) seq[i] = h->next_id + i;
      ids = seq.data();
      h->next_id += n;
    }
    h->append(n, list_no, codes, ids);
  });
}

int ivfpq_reset(ivfpq_index* h) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    for (auto& v : h->lcodes) v.clear();
    for (auto& v : h->lids) v.clear();
    DeviceGuard g(h->device);
    h->quiesce();
    h->drop_tables();
    h->drop_pending();
    h->host_stale = false;
    h->ntotal = 0;
    h->next_id = 0;
    h->dirty = true;
  });
}

int ivfpq_set_nprobe(ivfpq_index* h, int nprobe) {
  return guarded([&] {
    check_handle(h);
    require(nprobe >= 1 && nprobe <= kMaxK, "nprobe must be in [1, " + std::to_string(kMaxK) + "]");
    h->nprobe = nprobe;
  });
}

int ivfpq_get_nprobe(const ivfpq_index* h) { return h ? h->nprobe : -1; }

int ivfpq_set_list_range(ivfpq_index* h, int lo, int hi) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    require(0 <= lo && lo <= hi && hi <= h->nlist, "invalid list range");
    require(h->ntotal == 0 && h->q_n == 0, "set the list range before adding vectors");
    h->list_lo = lo;
    h->list_hi = hi;
    h->dirty = true;  // the device image (list order) follows the range
  });
}

int ivfpq_search(ivfpq_index* h, int64_t n, const float* x, int k, float* D, int64_t* I) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(n == 0 || (x && D && I), "null buffer");
    h->search_host(n, x, k, D, I, nullptr, nullptr, false);
  });
}

int ivfpq_search_preassigned(ivfpq_index* h, int64_t n, const float* x, int k, const int64_t* Iq, const float* Dq,
                             float* D, int64_t* I) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(n == 0 || (x && Iq && D && I), "null buffer");
    for (int64_t i = 0; i < n * h->nprobe; i++)
      require(Iq[i] < h->nlist, "list id out of range in Iq");
    h->search_host(n, x, k, D, I, Iq, Dq, true);
  });
}

int ivfpq_search_device(ivfpq_index* h, int64_t n, const float* x, int k, float* D, int64_t* I, void* stream) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    h->search_dev(n, x, k, D, I, nullptr, nullptr, false, (hipStream_t)stream);
  });
}

int ivfpq_search_preassigned_device(ivfpq_index* h, int64_t n, const float* x, int k, const int64_t* Iq,
                                    const float* Dq, float* D, int64_t* I, void* stream) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    h->search_dev(n, x, k, D, I, Iq, Dq, true, (hipStream_t)stream);
  });
}

int ivfpq_serve_request(ivfpq_index* h, const uint8_t* msg, int64_t msg_len, int with_lists, int batch_size, int dim,
                        int nprobe, uint8_t* answer, int64_t answer_cap, int64_t* answer_len) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(msg != nullptr, "null request message");
    h->serve(msg, msg_len, with_lists, batch_size, dim, nprobe, answer, answer_cap, answer_len);
  });
}

int ivfpq_precompute_tables_device(ivfpq_index* h, int64_t n, const float* x, void* stream, uint64_t* token) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(x != nullptr && token != nullptr, "null x or token");
    *token = h->tables_dev(n, x, stream ? (hipStream_t)stream : h->stream);
  });
}

int ivfpq_search_preassigned_tables_device(ivfpq_index* h, int64_t n, const float* x, int k, const int64_t* Iq,
                                           const float* Dq, float* D, int64_t* I, uint64_t token, void* stream) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(token != 0, "tables token 0 (use ivfpq_search_preassigned_device without tables)");
    h->search_dev(n, x, k, D, I, Iq, Dq, true, (hipStream_t)stream, token);
  });
}

int ivfpq_set_inflight(ivfpq_index* h, int on) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(on == 0 || on == 1, "inflight must be 0 or 1");
    h->quiesce();  // searches issued under the previous setting complete first
    h->inflight = on == 1;
  });
}

int ivfpq_get_inflight(const ivfpq_index* h) { return h ? (h->inflight ? 1 : 0) : -1; }

int ivfpq_overlap_built(void) { return 1; }

int ivfpq_get_error_count(ivfpq_index* h, int64_t* out) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(out != nullptr, "null output");
    h->quiesce();
    int64_t tot = 0;
    for (auto& w : h->work) {
      if (!w.p_hdr.p) continue;
      int32_t hdr[16];
      HIPCHECK(hipMemcpy(hdr, w.p_hdr.p, sizeof(hdr), hipMemcpyDeviceToHost));
      tot += hdr[15];
    }
    *out = tot;
  });
}

int ivfpq_get_repair_stats(ivfpq_index* h, int64_t* stale_reads, int64_t* repairs) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(stale_reads != nullptr && repairs != nullptr, "null output");
    h->quiesce();
    int64_t st = 0, rp = 0;
    for (auto& w : h->work) {
      if (!w.p_hdr.p) continue;
      int32_t hdr[16];
      HIPCHECK(hipMemcpy(hdr, w.p_hdr.p, sizeof(hdr), hipMemcpyDeviceToHost));
      st += hdr[kHdrStale];
      rp += hdr[kHdrRepair];
    }
    *stale_reads = st;
    *repairs = rp;
  });
}

int ivfpq_get_repair_log(ivfpq_index* h, uint32_t* out, int max_events, int* n_events) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(n_events != nullptr && (out != nullptr || max_events == 0) && max_events >= 0, "bad output arguments");
    h->quiesce();
    int got = 0;
    for (auto& w : h->work) {
      if (!w.p_hdr.p || !w.p_evlog.p) continue;
      int32_t hdr[16];
      HIPCHECK(hipMemcpy(hdr, w.p_hdr.p, sizeof(hdr), hipMemcpyDeviceToHost));
      const int kept = std::min(hdr[kHdrLog], kEvLog);
      std::vector<uint32_t> ev((size_t)8 * kEvLog);
      HIPCHECK(hipMemcpy(ev.data(), w.p_evlog.p, ev.size() * 4, hipMemcpyDeviceToHost));
      for (int e = 0; e < kept && got < max_events; e++, got++) std::memcpy(out + 8 * got, &ev[8 * e], 32);
    }
    *n_events = got;
  });
}

int ivfpq_debug_workspace(ivfpq_index* h, int ws, int what, void* dst, int64_t cap, int64_t* bytes) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(ws >= 0 && ws < ivfpq_index::kSlots && bytes != nullptr, "bad workspace index");
    h->quiesce();
    auto& w = h->work[ws];
    if (what >= 7) {  // host words: 7 the epoch of the last batch planned there, 8 the stream it ran on
      const uint64_t v = what == 7 ? (uint64_t)w.epoch : (uint64_t)(uintptr_t)w.done_stream;
      *bytes = 8;
      if (dst && cap >= 8) std::memcpy(dst, &v, 8);
      return;
    }
    const DevBuf* b = what == 0 ? &w.p_part : what == 1 ? &w.p_N : what == 2 ? &w.p_qmask : what == 3 ? &w.p_tau
                    : what == 4 ? &w.p_hdr : what == 5 ? &w.w_lists : &w.w_dis0;
    *bytes = (int64_t)b->bytes;
    if (dst && b->p) HIPCHECK(hipMemcpy(dst, b->p, std::min<size_t>(b->bytes, (size_t)cap), hipMemcpyDeviceToHost));
  });
}

int ivfpq_set_fault_injection(ivfpq_index* h, int every) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    require(every >= 0, "fault injection period must be >= 0");
    h->fault_inj = every;
  });
}

int ivfpq_debug_seed_tau(ivfpq_index* h, int64_t n, const float* keys) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    require(n >= 0 && (n == 0 || keys), "null buffer");
    h->tau_seed.resize(n);
    for (int64_t i = 0; i < n; i++) {  // the ordered-int word of the key (ivfpq_kernels.hip tau_lower)
      int32_t b;
      std::memcpy(&b, keys + i, 4);
      const int32_t o = b >= 0 ? b : b ^ 0x7FFFFFFF;
      h->tau_seed[i] = (uint32_t)o ^ 0x80000000u;
    }
  });
}

int ivfpq_coarse_tables_device(ivfpq_index* h, int64_t n, const float* x, int64_t* Iq, float* Dq, int64_t n_tables,
                               const float* x_tables, void* stream, uint64_t* token) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(x != nullptr && Iq != nullptr && Dq != nullptr && x_tables != nullptr && token != nullptr,
            "null pointer argument");
    *token = h->coarse_tables_dev(n, x, Iq, Dq, n_tables, x_tables, stream ? (hipStream_t)stream : h->stream);
  });
}

int ivfpq_coarse_device(ivfpq_index* h, int64_t n, const float* x, int64_t* Iq, float* Dq, void* stream) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    h->coarse_dev(n, x, Iq, Dq, (hipStream_t)stream);
  });
}

int ivfpq_merge_topk_device(int S, int64_t n, int k, int metric, const float* Din, const int64_t* Iin, float* Dout,
                            int64_t* Iout, void* stream) {
  return guarded([&] {
    require(S >= 1 && k >= 1 && n >= 0, "invalid merge shape");
    require(metric == IVFPQ_METRIC_L2 || metric == IVFPQ_METRIC_INNER_PRODUCT, "unknown metric");
    launch_merge_topk(S, n, k, Din, Iin, Dout, Iout, (hipStream_t)stream, metric == IVFPQ_METRIC_INNER_PRODUCT);
    HIPCHECK(hipGetLastError());
  });
}

int ivfpq_linear_transform_device(int64_t n, int d_in, int d_out, const float* AT, const float* b, const float* x,
                                  float* y, void* stream) {
  return guarded([&] {
    require(n >= 0 && d_in >= 1 && d_out >= 1, "invalid transform shape");
    require(n == 0 || (AT && x && y), "null buffer");
    launch_linear_transform(x, n, d_in, AT, b, d_out, y, (hipStream_t)stream);
    HIPCHECK(hipGetLastError());
  });
}

int ivfpq_set_timing(ivfpq_index* h, int on) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    require(on >= 0 && on <= 2, "timing mode must be 0, 1 or 2");
    h->timing = on;
  });
}

int ivfpq_get_timing(ivfpq_index* h, double* ms, int64_t* count) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(ms && count, "null output");
    h->collect_timing(ms, count);
  });
}

int64_t ivfpq_ntotal(const ivfpq_index* h) { return h ? h->ntotal : -1; }

int ivfpq_is_trained(const ivfpq_index* h) { return h && h->trained ? 1 : 0; }

int ivfpq_get_dims(const ivfpq_index* h, int* d, int* nlist, int* M, int* nbits, int* metric) {
  return guarded([&] {
    check_handle(h);
    if (d) *d = h->d;
    if (nlist) *nlist = h->nlist;
    if (M) *M = h->M;
    if (nbits) *nbits = h->nbits;
    if (metric) *metric = h->metric;
  });
}

int ivfpq_get_centroids(const ivfpq_index* h, float* out) {
  return guarded([&] {
    check_handle(h);
    require(h->trained, "index is not trained");
    std::memcpy(out, h->centroids.data(), sizeof(float) * h->centroids.size());
  });
}

int ivfpq_get_codebook(const ivfpq_index* h, float* out) {
  return guarded([&] {
    check_handle(h);
    require(h->trained, "index is not trained");
    std::memcpy(out, h->codebook.data(), sizeof(float) * h->codebook.size());
  });
}

int ivfpq_get_list_sizes(const ivfpq_index* ch, int64_t* out) {
  return guarded([&] {
    check_handle(ch);
    auto* h = const_cast<ivfpq_index*>(ch);  // the host lists are a cache of the device image
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    if (h->host_stale) {  // from the device image's offsets (no download of the lists)
      h->flush_pending(h->stream);
      h->quiesce();
      std::vector<int64_t> off(h->nlist + 1);
      HIPCHECK(hipMemcpy(off.data(), h->d_off.p, sizeof(int64_t) * (h->nlist + 1), hipMemcpyDeviceToHost));
      for (int l = 0; l < h->nlist; l++) out[l] = off[l + 1] - off[l];
      return;
    }
    for (int l = 0; l < h->nlist; l++) out[l] = (int64_t)h->lids[l].size();
  });
}

int ivfpq_get_list(const ivfpq_index* ch, int list, uint8_t* codes, int64_t* ids) {
  return guarded([&] {
    check_handle(ch);
    auto* h = const_cast<ivfpq_index*>(ch);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    h->sync_host();
    require(list >= 0 && list < h->nlist, "list id out of range");
    if (codes) std::memcpy(codes, h->lcodes[list].data(), h->lcodes[list].size());
    if (ids) std::memcpy(ids, h->lids[list].data(), sizeof(int64_t) * h->lids[list].size());
  });
}

int ivfpq_get_precomputed_table(ivfpq_index* h, float* out) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    require(h->trained, "index is not trained");
    HIPCHECK(hipMemcpy(out, h->d_T1.p, sizeof(float) * (size_t)h->nlist * h->M * h->ksub, hipMemcpyDeviceToHost));
  });
}

// ----------------------------------------------------------------- save/load
namespace {
constexpr char kMagic[8] = {'C', 'H', 'I', 'V', 'F', 'P', 'Q', '1'};

struct File {
  FILE* f;
  File(const char* p, const char* m) : f(std::fopen(p, m)) {
    require(f != nullptr, std::string("cannot open ") + p);
  }
  ~File() {
    if (f) std::fclose(f);
  }
  void w(const void* p, size_t n) { require(std::fwrite(p, 1, n, f) == n, "write failed"); }
  void r(void* p, size_t n) { require(std::fread(p, 1, n, f) == n, "truncated index file"); }
};
}  // namespace

int ivfpq_save(ivfpq_index* h, const char* path) {
  return guarded([&] {
    check_handle(h);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    h->sync_host();
    File f(path, "wb");
    f.w(kMagic, 8);
    int32_t hdr[8] = {h->d, h->nlist, h->M, h->nbits, h->metric, h->nprobe, h->trained ? 1 : 0, 0};
    f.w(hdr, sizeof(hdr));
    int64_t cnt[2] = {h->ntotal, h->next_id};
    f.w(cnt, sizeof(cnt));
    if (h->trained) {
      f.w(h->centroids.data(), sizeof(float) * h->centroids.size());
      f.w(h->codebook.data(), sizeof(float) * h->codebook.size());
    }
    for (int l = 0; l < h->nlist; l++) {
      int64_t sz = (int64_t)h->lids[l].size();
      f.w(&sz, 8);
      if (sz) {
        f.w(h->lcodes[l].data(), h->lcodes[l].size());
        f.w(h->lids[l].data(), sizeof(int64_t) * sz);
      }
    }
  });
}

int ivfpq_load(const char* path, int device, ivfpq_index** out) {
  ivfpq_index* h = nullptr;
  int rc = guarded([&] {
    File f(path, "rb");
    char magic[8];
    f.r(magic, 8);
    require(std::memcmp(magic, kMagic, 8) == 0, "not a CHIVFPQ1 index file");
    int32_t hdr[8];
    f.r(hdr, sizeof(hdr));
    int64_t cnt[2];
    f.r(cnt, sizeof(cnt));
    if (ivfpq_create(hdr[0], hdr[1], hdr[2], hdr[3], hdr[4], device, &h) != 0) throw std::runtime_error(g_err);
    h->nprobe = hdr[5];
    DeviceGuard g(device);
    if (hdr[6]) {
      h->centroids.resize((size_t)h->nlist * h->d);
      h->codebook.resize((size_t)h->M * h->ksub * (h->d / h->M));
      f.r(h->centroids.data(), sizeof(float) * h->centroids.size());
      f.r(h->codebook.data(), sizeof(float) * h->codebook.size());
      h->upload_trained();
    }
    for (int l = 0; l < h->nlist; l++) {
      int64_t sz;
      f.r(&sz, 8);
      require(sz >= 0, "corrupt list size");
      h->lcodes[l].resize((size_t)sz * h->M);
      h->lids[l].resize((size_t)sz);
      if (sz) {
        f.r(h->lcodes[l].data(), h->lcodes[l].size());
        f.r(h->lids[l].data(), sizeof(int64_t) * sz);
      }
    }
    h->ntotal = cnt[0];
    h->next_id = cnt[1];
    h->dirty = true;
    *out = h;
  });
  if (rc != 0 && h) {
    std::string e = g_err;
    ivfpq_free(h);
    g_err = e;
  }
  return rc;
}

int ivfpq_flat_search(int device, int d, int64_t nb, const float* xb, int64_t n, const float* x, int k, int metric,
                      float* D, int64_t* I) {
  return guarded([&] {
    require(d > 0 && nb >= 0 && n >= 0, "invalid shape");
    require(metric == IVFPQ_METRIC_L2 || metric == IVFPQ_METRIC_INNER_PRODUCT, "unknown metric");
    const bool ip = metric == IVFPQ_METRIC_INNER_PRODUCT;
    require(k >= 1 && k <= kMaxK, "k must be in [1, " + std::to_string(kMaxK) + "]");
    if (n == 0) return;
    DeviceGuard g(device);
    hipStream_t s;
    HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::unique_ptr<void, void (*)(void*)> sguard((void*)s, [](void* p) { (void)hipStreamDestroy((hipStream_t)p); });
    DevBuf dxb, dbn, dx, dxn, ddist, dD, dI;
    const int64_t nbb = std::max<int64_t>(nb, 1);
    dxb.ensure(sizeof(float) * nbb * d);
    dbn.ensure(sizeof(float) * nbb);
    if (nb) HIPCHECK(hipMemcpyAsync(dxb.p, xb, sizeof(float) * nb * d, hipMemcpyHostToDevice, s));
    launch_row_norms(dxb.as<float>(), nb, d, dbn.as<float>(), s);
    const int64_t qc = std::max<int64_t>(1, std::min<int64_t>(n, kChunkBytes / ((size_t)nbb * 4)));
    dx.ensure(sizeof(float) * qc * d);
    dxn.ensure(sizeof(float) * qc);
    ddist.ensure(sizeof(float) * qc * nbb);
    dD.ensure(sizeof(float) * qc * k);
    dI.ensure(sizeof(int64_t) * qc * k);
    for (int64_t q0 = 0; q0 < n; q0 += qc) {
      const int64_t c = std::min(qc, n - q0);
      HIPCHECK(hipMemcpyAsync(dx.p, x + q0 * d, sizeof(float) * c * d, hipMemcpyHostToDevice, s));
      launch_row_norms(dx.as<float>(), c, d, dxn.as<float>(), s);
      launch_l2_dist(dx.as<float>(), dxn.as<float>(), c, dxb.as<float>(), dbn.as<float>(), (int)nb, d,
                     ddist.as<float>(), s, ip);
      launch_select_rows(ddist.as<float>(), c, (int)nb, k, dD.as<float>(), dI.as<int64_t>(), s, ip);
      HIPCHECK(hipGetLastError());
      HIPCHECK(hipMemcpyAsync(D + q0 * k, dD.p, sizeof(float) * c * k, hipMemcpyDeviceToHost, s));
      HIPCHECK(hipMemcpyAsync(I + q0 * k, dI.p, sizeof(int64_t) * c * k, hipMemcpyDeviceToHost, s));
      HIPCHECK(hipStreamSynchronize(s));
    }
  });
}

}  // extern "C"
