#!/usr/bin/env python3
"""r05 race A/B: build experimental variants of libivfpq.so into lib/var/<name>/ by
patching a COPY of the shipped kernel source (the shipped ivfpq_kernels.hip stays
free of experiment switches).  Each variant changes how inter-kernel hand-off
data is stored or loaded:

  base      the shipped source, rebuilt (control)
  wt_part   per-wave partial-list records and counts stored write-through (sc1)
  wt_all    wt_part + every other inter-kernel hand-off store write-through: T3,
            coarse keys, bucket entries, per-pair dis0, probe masks, count / work
            counter zeroing, result D / I
  rel_end   every producer workgroup ends with an agent-scope release
            (buffer_wbl2 sc1 + s_waitcnt vmcnt(0)) -- coarse, select, scan, merges
  acq_start every consumer kernel starts with an agent-scope acquire per workgroup
  inv_sys   every consumer kernel starts with buffer_inv sc0 sc1 per workgroup

Usage: python profiles/race_variants.py base wt_part ...   (here, before gpurun)
"""
import os
import re
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C = os.path.join(R, "chameleon-rag-acceleration_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
F = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-I" + os.path.join(R, "include"),
     "-I" + C]

HELPERS = r'''
namespace chivf { namespace {
__device__ __forceinline__ void st_wt16(void* base, uint64_t byte_off, uint4 v) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const auto r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7FFFFFF0, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, r, (int)byte_off, 0, 16);
}
template <class T> __device__ __forceinline__ void st_ag(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_ag2(int2* p, int2 v) {
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), ((uint64_t)(uint32_t)v.y << 32) | (uint32_t)v.x,
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_ag2u(uint2* p, uint2 v) {
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), ((uint64_t)v.y << 32) | v.x, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void rel_agent() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
}}  // namespace chivf
'''


def sub(src, a, b, count=1):
    n = src.count(a)
    if n != count:
        raise SystemExit(f"patch anchor found {n} times (want {count}): {a[:80]!r}")
    return src.replace(a, b)


def wt_part(s):
    s = sub(s, "      o[ix] = part_rec(empty ? FLT_MAX : kc_key(tk.p[r]), tag, empty ? -1 : beg + (int64_t)(uint32_t)tk.p[r]);",
            "      st_wt16(pl.part, (uint64_t)(slot * pl.ks + ix) * 16,\n"
            "              part_rec(empty ? FLT_MAX : kc_key(tk.p[r]), tag, empty ? -1 : beg + (int64_t)(uint32_t)tk.p[r]));")
    s = sub(s, "    if (lane == 0) pl.partN[slot] = make_uint2((uint32_t)n, tag);",
            "    if (lane == 0) st_ag2u(pl.partN + slot, make_uint2((uint32_t)n, tag));")
    s = sub(s, "        pl.part[slot * pl.ks + re] =\n",
            "        st_wt16(pl.part, (uint64_t)(slot * pl.ks + re) * 16,\n")
    s = sub(s, "part_tag(pl.epoch, slot) | xcc_tag(), empty ? -1 : it.beg + (int64_t)(uint32_t)rk);",
            "part_tag(pl.epoch, slot) | xcc_tag(), empty ? -1 : it.beg + (int64_t)(uint32_t)rk));")
    return s


def wt_all(s):
    s = wt_part(s)
    # T3 (coarse launch's T3 role, k_ip_tiles, k_ip_table)
    s = sub(s, "        if (qq < nqq) t3.out[(q0 + qq) * total + e] = v;", "        if (qq < nqq) st_ag(t3.out + (q0 + qq) * total + e, v);")
    s = sub(s, "        t3.out[(q0 + qq) * total + e] = tree<K_IP>(", "        st_ag(t3.out + (q0 + qq) * total + e, tree<K_IP>(", 1)
    s = sub(s, "[&](int t) { return cwp[t]; }, dsub);\n      }\n    }\n    CDIAG(5);",
            "[&](int t) { return cwp[t]; }, dsub));\n      }\n    }\n    CDIAG(5);")
    s = sub(s, "    t3.out[(q0 + qq) * total + e] = tree<K_IP>([&](int t) { return xq[t]; }, [&](int t) { return cwp[t]; }, dsub);",
            "    st_ag(t3.out + (q0 + qq) * total + e, tree<K_IP>([&](int t) { return xq[t]; }, [&](int t) { return cwp[t]; }, dsub));")
    s = sub(s, "    out[(q0 + qq) * total + m * 256 + tid] =\n        tree<K_IP>([&](int t) { return xq[t]; }, [&](int t) { return cw[t]; }, DSUB);",
            "    st_ag(out + (q0 + qq) * total + m * 256 + tid,\n        tree<K_IP>([&](int t) { return xq[t]; }, [&](int t) { return cw[t]; }, DSUB));")
    # coarse keys
    s = sub(s, "      keys[(q0 + i) * nlist + c] = coarse_key(acc[t][r], xn[i], cnv, ip);",
            "      st_ag(keys + (q0 + i) * nlist + c, coarse_key(acc[t][r], xn[i], cnv, ip));")
    s = sub(s, "      keys[q * nlist + c] = coarse_key(acc[t][r], ip ? 0.f : xn[q], cnv, ip);",
            "      st_ag(keys + q * nlist + c, coarse_key(acc[t][r], ip ? 0.f : xn[q], cnv, ip));")
    # planning: bucket, pd0, qmask; coarse output lists / dis
    s = sub(s, "  if (s < pl.cap) pl.bucket[((int64_t)(l - lo) * 2 + kind) * pl.cap + s] = make_int2(pair, __float_as_int(dis0));\n  pl.pd0[pair] = dis0;",
            "  if (s < pl.cap) st_ag2(pl.bucket + ((int64_t)(l - lo) * 2 + kind) * pl.cap + s, make_int2(pair, __float_as_int(dis0)));\n  st_ag(pl.pd0 + pair, dis0);")
    s = sub(s, "    if (lane == 0) cp.pl.qmask[q * cp.pl.qmw] = um;", "    if (lane == 0) st_ag(cp.pl.qmask + q * cp.pl.qmw, um);")
    s = sub(s, "    if (lane == 0) pl.qmask[q * pl.qmw + (p0 >> 6)] = um;", "    if (lane == 0) st_ag(pl.qmask + q * pl.qmw + (p0 >> 6), um);")
    s = sub(s, "    out_dis[q * nprobe + lane] = empty ? (ip ? -FLT_MAX : FLT_MAX) : (ip ? -rd : rd);\n    out_list[q * nprobe + lane] = empty ? -1 : ri;",
            "    st_ag(out_dis + q * nprobe + lane, empty ? (ip ? -FLT_MAX : FLT_MAX) : (ip ? -rd : rd));\n    st_ag(out_list + q * nprobe + lane, empty ? (int64_t)-1 : ri);")
    # zeroing of counts and the work counter by the merge
    s = sub(s, "    for (int i = threadIdx.x; i < 2 * nloc; i += 256) pl.cnt[i] = 0;\n    if (threadIdx.x == 0) pl.hdr[2] = 0;",
            "    for (int i = threadIdx.x; i < 2 * nloc; i += 256) st_ag(pl.cnt + i, 0);\n    if (threadIdx.x == 0) st_ag(pl.hdr + 2, 0);")
    s = sub(s, "      if (lane == 0) pl.qdone[q] = 0;  // zero for the next batch", "      if (lane == 0) st_ag(pl.qdone + q, 0);")
    # results (fast path + full merge of k_merge_probes)
    s = sub(s, "          a.outD[q * k + lane] = empty ? pad : sgn * cd;\n          a.outI[q * k + lane] = empty ? -1 : ci;",
            "          st_ag(a.outD + q * k + lane, empty ? pad : sgn * cd);\n          st_ag(a.outI + q * k + lane, empty ? (int64_t)-1 : ci);")
    s = sub(s, "      a.outD[q * k + idx] = empty ? pad : sgn * tk.d[r];\n      a.outI[q * k + idx] = empty ? -1 : tk.id[r];",
            "      st_ag(a.outD + q * k + idx, empty ? pad : sgn * tk.d[r]);\n      st_ag(a.outI + q * k + idx, empty ? (int64_t)-1 : tk.id[r]);")
    return s


def rel_end(s):
    # list scan: after the item loop
    s = sub(s, "    it_no++;\n    cur = nxt;\n  }\n}", "    it_no++;\n    cur = nxt;\n  }\n  __syncthreads();\n  if (tid == 0) rel_agent();\n}")
    # coarse T3 role and key role
    s = sub(s, "    CDIAG(5);\n    return;\n  }", "    CDIAG(5);\n    __syncthreads();\n    if (tid == 0) rel_agent();\n    return;\n  }")
    s = sub(s, "      keys[(q0 + i) * nlist + c] = coarse_key(acc[t][r], xn[i], cnv, ip);\n    }\n  }\n  CDIAG(5);\n}",
            "      keys[(q0 + i) * nlist + c] = coarse_key(acc[t][r], xn[i], cnv, ip);\n    }\n  }\n  CDIAG(5);\n  rel_agent();\n}")
    s = sub(s, "  coarse_emit(run, q, lane, nprobe, out_dis, out_list, ip, x, d, cp);\n  SDIAG(5);\n}",
            "  coarse_emit(run, q, lane, nprobe, out_dis, out_list, ip, x, d, cp);\n  SDIAG(5);\n  rel_agent();\n}")
    return s


def kernel_start(s, stmt):
    for name in ["void k_scan_lists(ScanArgs a, ListPlan pl) {", "void k_merge_probes(ScanArgs a, ListPlan pl) {",
                 "void k_merge_radix(ScanArgs a, ListPlan pl) {", "void k_merge_big(ScanArgs a, ListPlan pl) {"]:
        s = sub(s, name, name + "\n  " + stmt)
    s = sub(s, "                                                       const float* __restrict__ x, int d, CoarsePlan cp) {\n  __shared__ uint64_t scratch[4][64];",
            "                                                       const float* __restrict__ x, int d, CoarsePlan cp) {\n  " + stmt + "\n  __shared__ uint64_t scratch[4][64];")
    return s



DBG_HELPERS = r"""
namespace chivf {
__device__ uint32_t g_dbg[1 + 64 * 48];
}
extern "C" int ivfpq_dbg_read(void* out, int zero) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(chivf::g_dbg), sizeof(uint32_t) * (1 + 64 * 48)) != hipSuccess) return -1;
  if (zero) {
    static uint32_t z[1 + 64 * 48];
    if (hipMemcpyToSymbol(HIP_SYMBOL(chivf::g_dbg), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
"""


def dbg(s):
    # scan: a record whose pair id is outside the batch -> log the raw record, the
    # counts and bucket slots re-read now (agent scope), and the work/prefix state
    s = sub(s, """    if (bad) {
      if (lane == 0) atomicAdd(pl.err, 1);
      it.cnt = 0;""", """    if (bad) {
      int e_ = 0;
      if (lane == 0) e_ = atomicAdd(&g_dbg[0], 1);
      e_ = __builtin_amdgcn_readfirstlane(e_);
      if (e_ < 64) {
        uint32_t* r_ = g_dbg + 1 + 48 * e_;
        const int kind_ = __builtin_amdgcn_readlane(rv, 13), t_ = __builtin_amdgcn_readlane(rv, 14);
        const int jl_ = it.l - a.list_lo;
        if (lane < 16) r_[lane] = (uint32_t)rv;
        if (lane == 16) r_[16] = 0xB0B0u;
        if (lane == 17) r_[17] = blockIdx.x;
        if (lane == 18) r_[18] = (uint32_t)n_items0;
        if (lane == 19) r_[19] = (uint32_t)n_items;
        if (lane == 20) r_[20] = (uint32_t)__hip_atomic_load(pl.cnt + kind_ * nloc + jl_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lane == 21) r_[21] = (uint32_t)__hip_atomic_load(pl.cnt + (1 - kind_) * nloc + jl_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lane >= 22 && lane < 26)
          r_[lane] = (uint32_t)__hip_atomic_load(reinterpret_cast<const int*>(pl.bucket) + 2 * (((int64_t)jl_ * 2 + kind_) * pl.cap + t_ * G + (lane - 22)),
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lane == 26) r_[26] = pl.epoch;
        if (lane == 27) r_[27] = (uint32_t)pl.cap;
        if (lane == 28) r_[28] = (uint32_t)s_ex[kind_][jl_ < nloc ? jl_ : 0];
        if (lane == 29) r_[29] = (uint32_t)nloc;
        if (lane == 30) r_[30] = ((uint32_t)__builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11)) & 15u);
      }
      if (lane == 0) atomicAdd(pl.err, 1);
      it.cnt = 0;""")
    return s


def w_unpack(s):  # every outstanding vector memory op done before the next record is unpacked
    return sub(s, "    if (nxt >= 0) {  // the next item's fields; with kEarly its first loads start here\n      unpack(nrec);",
               "    if (nxt >= 0) {  // the next item's fields; with kEarly its first loads start here\n"
               "      asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n      unpack(nrec);")


def w_fetch(s):  # the next record waited for right where it is fetched (no prefetch)
    return sub(s, "    const int nrec = fetch_rec(nxt >= 0 ? nxt : cur);  // the next record, in flight during the scan",
               "    const int nrec = fetch_rec(nxt >= 0 ? nxt : cur);  // the next record, in flight during the scan\n"
               "    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");")


def p_merge(s):  # perturbation outside the scan: a never-taken store in k_merge_probes
    return sub(s, "  const int64_t q = (int64_t)blockIdx.x * 4 + wave;\n  if (q >= a.nq) return;\n  const int k = a.k;",
               "  const int64_t q = (int64_t)blockIdx.x * 4 + wave;\n  if (q >= a.nq) return;\n  if (a.k < 0) pl.err[1] = 7;\n  const int k = a.k;")


def p_scan(s):  # perturbation inside the scan, away from the record: a never-taken store in write_partial
    return sub(s, "  if (pl.fault > 0 && slot % pl.fault == 1) return;  // (uniform; 0 in every real search)",
               "  if (pl.fault > 0 && slot % pl.fault == 1) return;  // (uniform; 0 in every real search)\n"
               "  if (k < 0) pl.err[1] = 7;")


def noswap(s):  # the lane ^ 16 / ^ 32 exchanges by ds_bpermute instead of v_permlane16/32_swap
    return sub(s, """  else if constexpr (J == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    return (int)((__lane_id() & 16) ? r[0] : r[1]);
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
    return (int)((__lane_id() & 32) ? r[0] : r[1]);
  }""", """  else return __shfl_xor(v, J, 64);""")


def notau(s):  # no cross-workgroup bound: tau_q never read (every item starts unbounded) nor lowered
    s = sub(s, "  return (uint32_t)(v >> 32) == ~pl.epoch ? (int)((uint32_t)v ^ 0x80000000u) : f2ord(kInf);",
            "  (void)v;\n  return f2ord(kInf);")
    s = sub(s, "  atomicMin(reinterpret_cast<unsigned long long*>(pl.tauq + q), (unsigned long long)w);",
            "  (void)w;")
    return s


def nowb(s):  # no cross-wave bound inside an item (s_wb never read)
    return sub(s, "        if (g < it.cnt) bound[g] = fminf(bound[g], ord2f(__builtin_amdgcn_readfirstlane(s_wb[g])));",
               "        (void)s_wb;")


TLOG_HELPERS = r"""
namespace chivf {
__device__ uint32_t* g_tlog;
__device__ uint32_t g_tlog_cap;
__device__ uint32_t g_tlog_n;
}
extern "C" int ivfpq_dbg_set_tlog(void* ptr, uint32_t cap) {
  uint32_t zero = 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(chivf::g_tlog), &ptr, sizeof(ptr)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(chivf::g_tlog_cap), &cap, sizeof(cap)) != hipSuccess) return -1;
  return hipMemcpyToSymbol(HIP_SYMBOL(chivf::g_tlog_n), &zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
extern "C" int ivfpq_dbg_tlog_count(uint32_t* n) {
  return hipMemcpyFromSymbol(n, HIP_SYMBOL(chivf::g_tlog_n), sizeof(uint32_t)) == hipSuccess ? 0 : -1;
}
"""


def taulog(s):
    # every tau lowering logged: (tauq address low word, epoch, query, value, site, pair, list, block | wave << 16)
    s = sub(s, "// a code position read back from a partial list, checked against the image",
            """__device__ __forceinline__ void tlog(const ListPlan& pl, const float* outD, int64_t q, int o, int site, int pair, int l) {
  if (!g_tlog) return;
  const uint32_t e = atomicAdd(&g_tlog_n, 1u);
  if (e >= g_tlog_cap) return;
  uint4* r = reinterpret_cast<uint4*>(g_tlog) + 2 * (size_t)e;
  r[0] = make_uint4((uint32_t)(uintptr_t)outD, pl.epoch, (uint32_t)q, (uint32_t)o);
  r[1] = make_uint4((uint32_t)site, (uint32_t)pair, (uint32_t)l, blockIdx.x | ((threadIdx.x >> 6) << 16));
}
// a code position read back from a partial list, checked against the image""")
    s = sub(s, """          atomicMin(&s_wb[g], f2ord(kc_key(tp)));
          tau_lower(pl, qix[g], f2ord(kc_key(tp)));""", """          atomicMin(&s_wb[g], f2ord(kc_key(tp)));
          tau_lower(pl, qix[g], f2ord(kc_key(tp)));
          tlog(pl, a.outD, qix[g], f2ord(kc_key(tp)), ROWK ? 11 : 12, it.pair[g], it.l);""")
    s = sub(s, """              atomicMin(&s_wb[g], f2ord(T));
              tau_lower(pl, qix[g], f2ord(T));""", """              atomicMin(&s_wb[g], f2ord(T));
              tau_lower(pl, qix[g], f2ord(T));
              tlog(pl, a.outD, qix[g], f2ord(T), 2, it.pair[g], it.l);""")
    s = sub(s, """              atomicMin(&s_wb[g], T);
              tau_lower(pl, qix[g], T);""", """              atomicMin(&s_wb[g], T);
              tau_lower(pl, qix[g], T);
              tlog(pl, a.outD, qix[g], T, 3, it.pair[g], it.l);""")
    return s


def tau_nop_after(s):  # 16 wait states right after every tau_q atomicMin (its data registers left alone that long)
    return sub(s, "  atomicMin(reinterpret_cast<unsigned long long*>(pl.tauq + q), (unsigned long long)w);",
               "  atomicMin(reinterpret_cast<unsigned long long*>(pl.tauq + q), (unsigned long long)w);\n"
               "  asm volatile(\"s_nop 7\\n\\ts_nop 7\" ::: \"memory\");")


def tau_nop_before(s):  # the same 16 wait states right before it (control: same perturbation, no protection after)
    return sub(s, "  atomicMin(reinterpret_cast<unsigned long long*>(pl.tauq + q), (unsigned long long)w);",
               "  asm volatile(\"s_nop 7\\n\\ts_nop 7\" ::: \"memory\");\n"
               "  atomicMin(reinterpret_cast<unsigned long long*>(pl.tauq + q), (unsigned long long)w);")


def nofast(s):  # keep tau, but never take the packed-prefix (fast) admission: per-chunk admission always
    return sub(s, "      } else if (!loose) {", "      } else if (!loose && a.k < 0) {")


def noloose(s):  # keep tau, but never derive bounds from the super-batch lane minima (loose path off)
    return sub(s, "        if (loose) {\n#pragma unroll\n          for (int g = 0; g < G; g++) {\n            if (bound[g] != kInf) continue;  // wave-uniform\n            float mn = kInf;",
               "        if (loose && a.k < 0) {\n#pragma unroll\n          for (int g = 0; g < G; g++) {\n            if (bound[g] != kInf) continue;  // wave-uniform\n            float mn = kInf;")


VARIANTS = {
    "base": lambda s: s,
    "wt_part": wt_part,
    "wt_all": wt_all,
    "rel_end": rel_end,
    "acq_start": lambda s: kernel_start(s, "{ if (threadIdx.x == 0) { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"agent\"); "
                                           "asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\"); } __syncthreads(); }"),
    "dbg": dbg,
    "nofast": nofast,
    "noloose": noloose,
    "tau_nop_after": tau_nop_after,
    "tau_nop_before": tau_nop_before,
    "taulog": taulog,
    "notau": notau,
    "nowb": nowb,
    "w_unpack": w_unpack,
    "w_fetch": w_fetch,
    "p_merge": p_merge,
    "p_scan": p_scan,
    "noswap": noswap,
    "inv_sys": lambda s: kernel_start(s, "{ if (threadIdx.x == 0) asm volatile(\"buffer_inv sc0 sc1\\n s_waitcnt vmcnt(0)\" ::: \"memory\"); "
                                         "__syncthreads(); }"),
}


def build(name):
    src = open(os.path.join(C, "ivfpq_kernels.hip")).read()
    src = VARIANTS[name](src)
    if name != "base":
        i = src.index("namespace chivf {")
        src = src[:i] + HELPERS + (DBG_HELPERS if name == "dbg" else "") + (TLOG_HELPERS if name == "taulog" else "") + src[i:]
    out = os.path.join(R, "chameleon-rag-acceleration_amd", "lib", "var", name)
    os.makedirs(out, exist_ok=True)
    kp = os.path.join(out, "ivfpq_kernels.hip")
    open(kp, "w").write(src)
    procs = [subprocess.Popen([HIPCC] + F + ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None", "-c", "-o",
                                             os.path.join(out, "k.o"), kp]),
             subprocess.Popen([HIPCC] + F + ["-x", "hip", "-c", "-o", os.path.join(out, "i.o"),
                                             os.path.join(C, "ivfpq_index.cpp")]),
             subprocess.Popen([HIPCC] + F + ["-c", "-o", os.path.join(out, "b.o"), os.path.join(C, "ivfpq_build.hip")])]
    if any(p.wait() for p in procs):
        raise SystemExit(f"build of {name} failed")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(out, "libivfpq.so"),
                           os.path.join(out, "k.o"), os.path.join(out, "b.o"), os.path.join(out, "i.o")])
    for f in ("k.o", "i.o", "b.o"):
        os.remove(os.path.join(out, f))
    print("built", name, flush=True)


if __name__ == "__main__":
    for n in sys.argv[1:]:
        build(n)
