"""Per-item phase breakdown of k_scan_lists from a DIAG_STAMPS build.

Slots per (workgroup, iteration), thread 0: 0 item start (barrier A), 1 LUT
built (barrier B), 2 scan done, 3 partial writes done, 4 codes, 5 pairs |
kind << 8, 6 wave 0's cycles in the super-batch gathers, 7 its admitted
candidates | drains << 32.

Usage (on the GPU box):
  bash profiles/build_variants.sh diag:"-DDIAG_STAMPS"     # here, before gpurun
  IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/diag/libivfpq.so python3 profiles/diag_stamps.py

Builds the C2 index (bench.py's workload), runs a few warm-up searches, then one
stamped search, and prints per phase (LUT build incl. its loads, scan, partial
writes) the cycle statistics split by item kind (0 = first probe, 1 = other),
the admitted-candidate counts (wave 0) and the per-workgroup busy fraction.
"""
import ctypes
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "chameleon-rag-acceleration_amd"))
WG, ITEMS, SLOTS = 1024, 64, 16  # ivfpq_diag.h kDiagWG, kDiagItems, kDiagSlots


def main():
    import torch

    import faiss_amd as faiss
    from faiss_amd import _lib, datasets

    nb = int(os.environ.get("NB", "1000000"))
    xt = datasets.synthetic_sift_like(100_000, 128, seed=4321)  # (bench.py's data: 200k centres)
    xb = datasets.synthetic_sift_like(nb, 128, seed=1234)
    xq = datasets.synthetic_sift_like(1024, 128, seed=123)
    ix = faiss.index_factory(128, "IVF1024,PQ16")
    ix.niter_coarse = ix.niter_pq = 25
    ix.train(xt)
    ix.add(xb)
    ix.nprobe = 16
    xd = torch.from_numpy(xq).cuda()
    L = _lib.load()
    fn = L.ivfpq_diag_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros(WG * ITEMS * SLOTS, np.uint64)
    for _ in range(5):
        ix.search_device(xd, 10)
    torch.cuda.synchronize()
    fn(buf.ctypes.data, buf.nbytes)  # clears
    ix.search_device(xd, 10)
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    a = buf.reshape(WG, ITEMS, SLOTS).astype(np.int64)
    valid = a[:, :, 0] > 0
    t0, t1, t2, t3, n, ck, push, tau = [a[:, :, i] for i in range(8)]
    kind = (ck >> 8) & 1
    cnt = ck & 0xFF
    print(f"items {valid.sum()} (kind0 {(valid & (kind == 0)).sum()}, kind1 {(valid & (kind == 1)).sum()}); "
          f"per-WG mean {valid.sum(1)[valid.any(1)].mean():.1f} max {valid.sum(1).max()}")
    for kname, sel in (("kind0", valid & (kind == 0)), ("kind1", valid & (kind == 1)), ("all", valid)):
        if not sel.any():
            continue
        print(f"-- {kname}: codes/item {n[sel].mean():.0f}, pairs/item {cnt[sel].mean():.2f}, "
              f"admitted (wave 0, all pairs) {(tau[sel] & 0xFFFFFFFF).mean():.1f}, drains {(tau[sel] >> 32).mean():.2f}, "
              f"gather cycles (wave 0) {push[sel].mean():.0f}")
        d_loose, d_admit, d_fdrain, t_loop = (a[:, :, i][sel] for i in (8, 9, 10, 11))
        print(f"   scan phase (wave 0): setup {(t_loop - t1[sel]).mean():.0f}, gathers {push[sel].mean():.0f}, "
              f"bounds {d_loose.mean():.0f}, admission {d_admit.mean():.0f}, final drain {d_fdrain.mean():.0f}")
        for name, v in (("build", (t1 - t0)[sel]), ("scan", (t2 - t1)[sel]), ("write", (t3 - t2)[sel])):
            print(f"   {name:6s} cycles mean {v.mean():8.0f} p50 {np.median(v):8.0f} p90 {np.percentile(v, 90):8.0f}")
        sc = (t2 - t1)[sel]
        print(f"   scan cycles per code-pair {sc.sum() / (n[sel] * cnt[sel]).sum():.2f}, per code {sc.sum() / n[sel].sum():.2f}")
    first = np.where(valid, t0, np.iinfo(np.int64).max).min(1)
    last = np.where(valid, t3, 0).max(1)
    act = valid.any(1)
    span = (last - first)[act]
    busy = ((t3 - t0) * valid).sum(1)[act]
    g0 = first[act].min()
    gend = last[act].max()
    print(f"WG span mean {span.mean():.0f} max {span.max():.0f} cycles; busy frac {busy.sum() / span.sum():.3f}; "
          f"kernel span {gend - g0} cycles")
    print(f"WG start offset p50 {np.median(first[act] - g0):.0f} max {(first[act] - g0).max():.0f}; "
          f"WG end offset p10 {np.percentile(last[act] - g0, 10):.0f} p50 {np.median(last[act] - g0):.0f}")
    # kind-1 items started before (within the kernel) vs after all kind-0 items ended
    k0_end = np.where(valid & (kind == 0), t3, 0).max()
    k1 = valid & (kind == 1)
    early = k1 & (t0 < k0_end)
    print(f"kind-1 items started before the last kind-0 item ended: {early.sum()} of {k1.sum()}; "
          f"their scan mean {(t2 - t1)[early].mean() if early.any() else 0:.0f} vs later "
          f"{(t2 - t1)[k1 & ~early].mean() if (k1 & ~early).any() else 0:.0f}")


if __name__ == "__main__":
    main()
