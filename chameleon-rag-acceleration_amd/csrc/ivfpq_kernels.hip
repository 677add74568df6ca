// gfx950 (MI355X, CDNA4) kernels for IVF-PQ search.
//
// Hot path: coarse probe -> distance LUT -> PQ-code scan
// -> top-k.  The reference runs it in Faiss (IndexIVFPQ::search ->
// IVFPQScanner::scan_list_with_table; faiss-gpu pqScanPrecomputedMultiPass +
// pass1/pass2SelectLists, Chameleon/Faiss_experiments/MICRO_GPU_profiling/
// classify_stages.py:127-136) and on the FPGA (retrieval_accelerator/
// entire_accelerator_final_SIFT_M16/src/{LUT_construction,ADC}.hpp).
//
// Design:
//  * one 256-thread workgroup per query; the query's inner-product table T3
//    (M x 256 fp32) is held in VGPRs; for every probed list the workgroup
//    forms LUT = T1[list] + (-2) T3 directly in LDS (the LUT never touches
//    HBM), then the four waves stream the list's PQ codes (16 B per lane,
//    coalesced 1 KiB per wave-instruction) and sum M LDS lookups per code;
//  * top-k is fused into the scan: each wave keeps its k best (dist, label)
//    pairs sorted across lanes in registers (R = ceil(k/64) rows) and admits a
//    candidate only if it beats the wave's current k-th; the four wave lists
//    are merged by rank at the end.  No distance is ever written to memory.
//  * every fp32 operation follows the oracle's order (oracle/ivfpq_oracle.c,
//    Faiss 1.7.1 AVX order); the library is compiled with -ffp-contract=off
//    and the only FMAs are the explicit fmaf() of the coarse inner product.
#include <float.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "ivfpq_kernels.h"

namespace chivf {

namespace {

constexpr float kInf = __builtin_huge_valf();

enum { K_IP = 0, K_L2 = 1, K_NORM = 2 };

// Faiss-1.7.1 AVX reduction order (see or_tree in oracle/ivfpq_oracle.c).
// fx(t), fy(t) return element t of the two operands.
template <int KIND, class FX, class FY>
__device__ __forceinline__ float tree(FX fx, FY fy, int d) {
  float a8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int i = 0;
  for (; i + 8 <= d; i += 8) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      float p;
      if (KIND == K_IP) {
        p = fx(i + j) * fy(i + j);
      } else if (KIND == K_L2) {
        float t = fx(i + j) - fy(i + j);
        p = t * t;
      } else {
        float v = fx(i + j);
        p = v * v;
      }
      a8[j] = a8[j] + p;
    }
  }
  float a4[4];
#pragma unroll
  for (int j = 0; j < 4; j++) a4[j] = a8[j + 4] + a8[j];
#pragma unroll
  for (int pass = 0; pass < 2; pass++) {
    // pass 0: the 4-wide remainder (d - i >= 4); pass 1: the masked tail
    if (pass == 0 && i + 4 > d) continue;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (i + j < d) {
        float p;
        if (KIND == K_IP) {
          p = fx(i + j) * fy(i + j);
        } else if (KIND == K_L2) {
          float t = fx(i + j) - fy(i + j);
          p = t * t;
        } else {
          float v = fx(i + j);
          p = v * v;
        }
        a4[j] = a4[j] + p;
      }
    }
    if (pass == 0) i += 4;
  }
  float h0 = a4[0] + a4[1];
  float h1 = a4[2] + a4[3];
  return h0 + h1;
}

__device__ __forceinline__ bool lexless(float ad, int64_t ai, float bd, int64_t bi) {
  return ad < bd || (ad == bd && ai < bi);
}

__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

__device__ __forceinline__ int64_t readlane_i64(int64_t v, int lane) {
  const uint64_t u = (uint64_t)v;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), lane);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ float shfl_up1_f(float v) { return __shfl_up(v, 1, 64); }

__device__ __forceinline__ int64_t shfl_up1_i64(int64_t v) {
  const uint64_t u = (uint64_t)v;
  const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)u, 1, 64);
  const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(u >> 32), 1, 64);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// A wave's running k best (dist, label) pairs, sorted ascending across
// R rows x 64 lanes (logical index r*64 + lane).  Requires k <= 64*R.
template <int R>
struct WaveTopK {
  float d[R];
  int64_t id[R];
  float td;     // current k-th best (the admission threshold)
  int64_t ti;
  int krow, klane;

  __device__ __forceinline__ void init(int k) {
#pragma unroll
    for (int r = 0; r < R; r++) {
      d[r] = kInf;
      id[r] = kSentinelId;
    }
    td = kInf;
    ti = kSentinelId;
    krow = (k - 1) >> 6;
    klane = (k - 1) & 63;
  }

  __device__ __forceinline__ void refresh_tau() {
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (r == krow) {
        td = readlane_f(d[r], klane);
        ti = readlane_i64(id[r], klane);
      }
    }
  }

  // Insert the candidates (cd, ci) of the lanes set in `mask` (wave-uniform).
  __device__ __forceinline__ void insert(uint64_t mask, float cd, int64_t ci, int lane) {
    while (mask) {
      const int src = __builtin_ctzll(mask);
      mask &= mask - 1;
      const float vd = readlane_f(cd, src);
      const int64_t vi = readlane_i64(ci, src);
      if (!lexless(vd, vi, td, ti)) continue;  // overtaken by an earlier insert
      int pos = 0;
#pragma unroll
      for (int r = 0; r < R; r++) pos += __popcll(__ballot(lexless(d[r], id[r], vd, vi)));
#pragma unroll
      for (int r = R - 1; r >= 0; r--) {
        if ((r + 1) * 64 <= pos) continue;  // row entirely before the slot
        float cdd = vd;
        int64_t cii = vi;
        if (r > 0) {
          cdd = readlane_f(d[r - 1], 63);
          cii = readlane_i64(id[r - 1], 63);
        }
        float ud = shfl_up1_f(d[r]);
        int64_t ui = shfl_up1_i64(id[r]);
        if (lane == 0) {
          ud = cdd;
          ui = cii;
        }
        const int idx = r * 64 + lane;
        if (idx > pos) {
          d[r] = ud;
          id[r] = ui;
        } else if (idx == pos) {
          d[r] = vd;
          id[r] = vi;
        }
      }
      refresh_tau();
    }
  }
};

// ------------------------------------------------------------------ norms
__global__ __launch_bounds__(256) void k_row_norms(const float* __restrict__ x, int64_t n, int d,
                                                   float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float* xi = x + i * d;
  out[i] = tree<K_NORM>([&](int t) { return xi[t]; }, [&](int t) { return xi[t]; }, d);
}

// ------------------------------------------------- coarse L2 distance matrix
// 64 x 64 output tile per 256-thread workgroup, 4 x 4 per thread, K staged in
// LDS 16 at a time.  Each output's inner product is a k-ordered fmaf chain.
constexpr int DT_B = 64;
constexpr int DT_K = 16;

__global__ __launch_bounds__(256) void k_l2_dist(const float* __restrict__ x, const float* __restrict__ xn,
                                                 int64_t nx, const float* __restrict__ c,
                                                 const float* __restrict__ cn, int nc, int d,
                                                 float* __restrict__ out) {
  __shared__ float xs[DT_K][DT_B + 4];
  __shared__ float cs[DT_K][DT_B + 4];
  const int tid = threadIdx.x;
  const int tx = tid & 15, ty = tid >> 4;
  const int64_t row0 = (int64_t)blockIdx.y * DT_B;
  const int64_t col0 = (int64_t)blockIdx.x * DT_B;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[i][j] = 0.f;

  for (int k0 = 0; k0 < d; k0 += DT_K) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int e = tid + 256 * u;
      const int r = e >> 4, kk = e & 15;
      const bool kin = k0 + kk < d;
      xs[kk][r] = (row0 + r < nx && kin) ? x[(row0 + r) * d + k0 + kk] : 0.f;
      cs[kk][r] = (col0 + r < nc && kin) ? c[(col0 + r) * d + k0 + kk] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < DT_K; kk++) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; i++) a[i] = xs[kk][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; j++) b[j] = cs[kk][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = __builtin_fmaf(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int64_t r = row0 + ty * 4 + i;
    if (r >= nx) continue;
    const float xr = xn[r];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int64_t cc = col0 + tx * 4 + j;
      if (cc >= nc) continue;
      float dis = (xr + cn[cc]) - 2.0f * acc[i][j];
      if (dis < 0.f) dis = 0.f;
      out[r * nc + cc] = dis;
    }
  }
}

// ------------------------------------------------------------ row select
template <int R>
__global__ __launch_bounds__(256) void k_select_rows(const float* __restrict__ dist, int64_t nrows, int ncols,
                                                     int n, float* __restrict__ ov, int64_t* __restrict__ oc) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= nrows) return;  // wave-uniform
  WaveTopK<R> tk;
  tk.init(n);
  const float* drow = dist + row * ncols;
  for (int base = 0; base < ncols; base += 64) {
    const int cix = base + lane;
    const bool valid = cix < ncols;
    const float v = valid ? drow[cix] : kInf;
    const bool pass = valid && lexless(v, (int64_t)cix, tk.td, tk.ti);
    const uint64_t mask = __ballot(pass);
    if (mask) tk.insert(mask, v, (int64_t)cix, lane);
  }
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int idx = r * 64 + lane;
    if (idx < n) {
      const bool empty = tk.id[r] == kSentinelId;
      ov[row * n + idx] = empty ? FLT_MAX : tk.d[r];
      oc[row * n + idx] = empty ? -1 : tk.id[r];
    }
  }
}

// -------------------------------------------------------------- PQ tables
__global__ __launch_bounds__(256) void k_ip_table(const float* __restrict__ x, int64_t n, int d,
                                                  const float* __restrict__ cb, int M, int ksub,
                                                  float* __restrict__ out) {
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= n * M * ksub) return;
  const int j = (int)(gid % ksub);
  const int64_t t = gid / ksub;
  const int m = (int)(t % M);
  const int64_t q = t / M;
  const int dsub = d / M;
  const float* xq = x + q * d + m * dsub;
  const float* cw = cb + ((int64_t)m * ksub + j) * dsub;
  out[gid] = tree<K_IP>([&](int u) { return xq[u]; }, [&](int u) { return cw[u]; }, dsub);
}

__global__ __launch_bounds__(256) void k_precompute_T1(const float* __restrict__ cent, int nlist, int d,
                                                       const float* __restrict__ cb, int M, int ksub,
                                                       float* __restrict__ T1) {
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (int64_t)nlist * M * ksub) return;
  const int j = (int)(gid % ksub);
  const int64_t t = gid / ksub;
  const int m = (int)(t % M);
  const int64_t l = t / M;
  const int dsub = d / M;
  const float* cw = cb + ((int64_t)m * ksub + j) * dsub;
  const float* cl = cent + l * d + m * dsub;
  const float rn = tree<K_NORM>([&](int u) { return cw[u]; }, [&](int u) { return cw[u]; }, dsub);
  const float ip = tree<K_IP>([&](int u) { return cl[u]; }, [&](int u) { return cw[u]; }, dsub);
  T1[gid] = rn + 2.0f * ip;
}

// ---------------------------------------------------------------- encode
__global__ __launch_bounds__(256) void k_pq_encode(const float* __restrict__ x, int64_t n, int d,
                                                   const float* __restrict__ cent,
                                                   const int64_t* __restrict__ list_no,
                                                   const float* __restrict__ cb, int M, int ksub,
                                                   uint8_t* __restrict__ codes) {
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= n * M) return;
  const int m = (int)(gid % M);
  const int64_t i = gid / M;
  const int dsub = d / M;
  const float* xi = x + i * d + m * dsub;
  const float* ci = cent + list_no[i] * d + m * dsub;
  int best = 0;
  float bd = 0.f;
  for (int j = 0; j < ksub; j++) {
    const float* cw = cb + ((int64_t)m * ksub + j) * dsub;
    const float dd = tree<K_L2>([&](int u) { return xi[u] - ci[u]; }, [&](int u) { return cw[u]; }, dsub);
    if (j == 0 || dd < bd) {
      bd = dd;
      best = j;
    }
  }
  codes[gid] = (uint8_t)best;
}

// ------------------------------------------------------- fused scan + top-k
template <int M>
struct CodeWords {
  uint32_t w[M / 4];
  __device__ __forceinline__ void load(const uint8_t* p) {
    if constexpr (M % 16 == 0) {
#pragma unroll
      for (int v = 0; v < M / 16; v++) {
        const uint4 t = reinterpret_cast<const uint4*>(p)[v];
        w[4 * v + 0] = t.x;
        w[4 * v + 1] = t.y;
        w[4 * v + 2] = t.z;
        w[4 * v + 3] = t.w;
      }
    } else if constexpr (M % 8 == 0) {
#pragma unroll
      for (int v = 0; v < M / 8; v++) {
        const uint2 t = reinterpret_cast<const uint2*>(p)[v];
        w[2 * v + 0] = t.x;
        w[2 * v + 1] = t.y;
      }
    } else {
#pragma unroll
      for (int v = 0; v < M / 4; v++) w[v] = reinterpret_cast<const uint32_t*>(p)[v];
    }
  }
  __device__ __forceinline__ uint32_t byte(int m) const { return (w[m >> 2] >> ((m & 3) * 8)) & 0xffu; }
};

template <int M, int R>
__global__ __launch_bounds__(256) void k_scan_topk(ScanArgs a) {
  constexpr int LUTN = M * 256;  // fp32 entries per LUT
  constexpr int NV4 = M / 4;     // float4 per thread while forming the LUT
  constexpr int KP = R * 64;
  constexpr int LUT_BYTES = LUTN * 4;
  constexpr int MERGE_BYTES = 4 * KP * 12;
  constexpr int SMEM = LUT_BYTES > MERGE_BYTES ? LUT_BYTES : MERGE_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  float* lut = reinterpret_cast<float*>(smem);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int64_t q = blockIdx.x;
  const int k = a.k;

  // This thread's slice of the query's T3 (float4 index e*256 + tid).
  float4 t3[NV4];
  {
    const float4* T3q = reinterpret_cast<const float4*>(a.T3 + q * LUTN);
#pragma unroll
    for (int e = 0; e < NV4; e++) t3[e] = T3q[e * 256 + tid];
  }

  WaveTopK<R> tk;
  tk.init(k);

  for (int p = 0; p < a.nprobe; ++p) {
    const int64_t l = a.probe_list[q * a.nprobe + p];
    if (l < a.list_lo || l >= a.list_hi) continue;  // skipped probe (-1) or another shard's list
    const float d0 = a.probe_dis0 ? a.probe_dis0[q * a.nprobe + p] : 0.f;

    __syncthreads();  // every wave is done with the previous LUT
    {
      const float4* T1l = reinterpret_cast<const float4*>(a.T1 + l * LUTN);
      float4* lut4 = reinterpret_cast<float4*>(lut);
#pragma unroll
      for (int e = 0; e < NV4; e++) {
        float4 v = T1l[e * 256 + tid];
        const float4 t = t3[e];
        v.x = v.x + (-2.0f * t.x);
        v.y = v.y + (-2.0f * t.y);
        v.z = v.z + (-2.0f * t.z);
        v.w = v.w + (-2.0f * t.w);
        lut4[e * 256 + tid] = v;
      }
    }
    __syncthreads();

    const int64_t beg = a.list_off[l];
    const int64_t n = a.list_off[l + 1] - beg;
    const uint8_t* lc = a.codes + beg * M;
    const int64_t* lid = a.ids + beg;
    for (int64_t base = wave * 64; base < n; base += 256) {
      const int64_t i = base + lane;
      const bool valid = i < n;
      float dis = d0;
      if (valid) {
        CodeWords<M> cw;
        cw.load(lc + i * M);
#pragma unroll
        for (int m = 0; m < M; m++) dis = dis + lut[m * 256 + cw.byte(m)];
      }
      const bool maybe = valid && dis <= tk.td;
      int64_t id = kSentinelId;
      if (maybe) id = lid[i];
      const bool pass = maybe && lexless(dis, id, tk.td, tk.ti);
      const uint64_t mask = __ballot(pass);
      if (mask) tk.insert(mask, dis, id, lane);
    }
  }

  // ---- merge the four wave lists by rank
  __syncthreads();
  float* md = reinterpret_cast<float*>(smem);
  int64_t* mi = reinterpret_cast<int64_t*>(smem + 4 * KP * 4);
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int idx = r * 64 + lane;
    if (idx < k) {
      md[wave * KP + idx] = tk.d[r];
      mi[wave * KP + idx] = tk.id[r];
    }
  }
  __syncthreads();
  for (int e = tid; e < 4 * k; e += 256) {
    const int w = e / k;
    const int idx = e - w * k;
    const float vd = md[w * KP + idx];
    const int64_t vi = mi[w * KP + idx];
    int rank = idx;
#pragma unroll
    for (int w2 = 0; w2 < 4; w2++) {
      if (w2 == w) continue;
      int lo = 0, hi = k;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const float ed = md[w2 * KP + mid];
        const int64_t ei = mi[w2 * KP + mid];
        const bool before = (w2 < w) ? !lexless(vd, vi, ed, ei) : lexless(ed, ei, vd, vi);
        if (before)
          lo = mid + 1;
        else
          hi = mid;
      }
      rank += lo;
    }
    if (rank < k) {
      const bool empty = vi == kSentinelId;
      a.outD[q * k + rank] = empty ? FLT_MAX : vd;
      a.outI[q * k + rank] = empty ? -1 : vi;
    }
  }
}

// ------------------------------------------------------------ shard merge
__global__ __launch_bounds__(256) void k_merge_topk(int S, int64_t n, int k, const float* __restrict__ Din,
                                                    const int64_t* __restrict__ Iin, float* __restrict__ Dout,
                                                    int64_t* __restrict__ Iout) {
  const int64_t q = blockIdx.x;
  auto key_d = [&](int s, int j) { return Din[((int64_t)s * n + q) * k + j]; };
  auto key_i = [&](int s, int j) {
    const int64_t v = Iin[((int64_t)s * n + q) * k + j];
    return v < 0 ? kSentinelId : v;
  };
  for (int e = threadIdx.x; e < S * k; e += 256) {
    const int s = e / k;
    const int idx = e - s * k;
    const float vd = key_d(s, idx);
    const int64_t vi = key_i(s, idx);
    int rank = idx;
    for (int s2 = 0; s2 < S; s2++) {
      if (s2 == s) continue;
      int lo = 0, hi = k;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const float ed = key_d(s2, mid);
        const int64_t ei = key_i(s2, mid);
        const bool before = (s2 < s) ? !lexless(vd, vi, ed, ei) : lexless(ed, ei, vd, vi);
        if (before)
          lo = mid + 1;
        else
          hi = mid;
      }
      rank += lo;
    }
    if (rank < k) {
      const bool empty = vi == kSentinelId;
      Dout[q * k + rank] = empty ? FLT_MAX : vd;
      Iout[q * k + rank] = empty ? -1 : vi;
    }
  }
}

inline unsigned nblocks(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

inline int rows_for(int k) { return k <= 64 ? 1 : k <= 128 ? 2 : k <= 256 ? 4 : k <= 512 ? 8 : 16; }

}  // namespace

void launch_row_norms(const float* x, int64_t n, int d, float* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_row_norms, dim3(nblocks(n, 256)), dim3(256), 0, s, x, n, d, out);
}

void launch_l2_dist(const float* x, const float* xn, int64_t nx, const float* c, const float* cn, int nc, int d,
                    float* out, hipStream_t s) {
  if (nx <= 0 || nc <= 0) return;
  dim3 grid(nblocks(nc, DT_B), nblocks(nx, DT_B));
  hipLaunchKernelGGL(k_l2_dist, grid, dim3(256), 0, s, x, xn, nx, c, cn, nc, d, out);
}

void launch_select_rows(const float* dist, int64_t nrows, int ncols, int n, float* ov, int64_t* oc,
                        hipStream_t s) {
  if (nrows <= 0) return;
  const dim3 grid(nblocks(nrows, 4));
  switch (rows_for(n)) {
    case 1: hipLaunchKernelGGL(k_select_rows<1>, grid, dim3(256), 0, s, dist, nrows, ncols, n, ov, oc); break;
    case 2: hipLaunchKernelGGL(k_select_rows<2>, grid, dim3(256), 0, s, dist, nrows, ncols, n, ov, oc); break;
    case 4: hipLaunchKernelGGL(k_select_rows<4>, grid, dim3(256), 0, s, dist, nrows, ncols, n, ov, oc); break;
    case 8: hipLaunchKernelGGL(k_select_rows<8>, grid, dim3(256), 0, s, dist, nrows, ncols, n, ov, oc); break;
    default: hipLaunchKernelGGL(k_select_rows<16>, grid, dim3(256), 0, s, dist, nrows, ncols, n, ov, oc); break;
  }
}

void launch_ip_table(const float* x, int64_t n, int d, const float* cb, int M, int ksub, float* out,
                     hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_ip_table, dim3(nblocks(n * M * ksub, 256)), dim3(256), 0, s, x, n, d, cb, M, ksub, out);
}

void launch_precompute_T1(const float* cent, int nlist, int d, const float* cb, int M, int ksub, float* T1,
                          hipStream_t s) {
  hipLaunchKernelGGL(k_precompute_T1, dim3(nblocks((int64_t)nlist * M * ksub, 256)), dim3(256), 0, s, cent, nlist,
                     d, cb, M, ksub, T1);
}

void launch_pq_encode(const float* x, int64_t n, int d, const float* cent, const int64_t* list_no,
                      const float* cb, int M, int ksub, uint8_t* codes, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pq_encode, dim3(nblocks(n * M, 256)), dim3(256), 0, s, x, n, d, cent, list_no, cb, M, ksub,
                     codes);
}

bool scan_supported_M(int M) { return M == 8 || M == 16 || M == 32 || M == 48 || M == 64; }

template <int M>
static void launch_scan_M(const ScanArgs& a, hipStream_t s) {
  const dim3 grid((unsigned)a.nq);
  switch (rows_for(a.k)) {
    case 1: hipLaunchKernelGGL((k_scan_topk<M, 1>), grid, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL((k_scan_topk<M, 2>), grid, dim3(256), 0, s, a); break;
    case 4: hipLaunchKernelGGL((k_scan_topk<M, 4>), grid, dim3(256), 0, s, a); break;
    case 8: hipLaunchKernelGGL((k_scan_topk<M, 8>), grid, dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL((k_scan_topk<M, 16>), grid, dim3(256), 0, s, a); break;
  }
}

void launch_scan_topk(const ScanArgs& a, hipStream_t s) {
  if (a.nq <= 0) return;
  switch (a.M) {
    case 8: launch_scan_M<8>(a, s); break;
    case 16: launch_scan_M<16>(a, s); break;
    case 32: launch_scan_M<32>(a, s); break;
    case 48: launch_scan_M<48>(a, s); break;
    case 64: launch_scan_M<64>(a, s); break;
    default: break;
  }
}

void launch_merge_topk(int S, int64_t n, int k, const float* Din, const int64_t* Iin, float* Dout, int64_t* Iout,
                       hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_merge_topk, dim3((unsigned)n), dim3(256), 0, s, S, n, k, Din, Iin, Dout, Iout);
}

}  // namespace chivf
