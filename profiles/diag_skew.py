"""Per-item phase breakdown of k_scan_skew16 (wave 0) from a DIAG_STAMPS build.

Slots per (workgroup, iteration): 0 arrive at barrier A, 1 leave A, 2 leave B (LUT built),
3 first block's code words ready, 4 scan done, 5 partial writes done, 6 n | kind << 32 |
pairs << 40 | blocks << 48, 7 cycles in the super-batch gathers.

Usage (GPU box): IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/diag/libivfpq.so python3 profiles/diag_skew.py
"""
import ctypes
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "chameleon-rag-acceleration_amd"))
WG, ITEMS, SLOTS = 1024, 64, 16


def main():
    import torch

    import faiss_amd as faiss
    from faiss_amd import _lib, datasets

    xt = datasets.synthetic_sift_like(100_000, 128, seed=4321)
    xb = datasets.synthetic_sift_like(1_000_000, 128, seed=1234)
    xq = datasets.synthetic_sift_like(1024, 128, seed=123)
    ix = faiss.index_factory(128, "IVF1024,PQ16")
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
    valid = a[:, :, 1] > 0
    t = [a[:, :, i] for i in range(6)]
    info = a[:, :, 6]
    n = info & 0xFFFFFFFF
    kind = (info >> 32) & 0xFF
    cnt = (info >> 40) & 0xFF
    nblk = (info >> 48) & 0xFFFF
    print(f"items {valid.sum()} (kind0 {(valid & (kind == 0)).sum()}); per-WG mean {valid.sum(1)[valid.any(1)].mean():.1f}")
    names = ["A wait", "build", "first codes", "scan", "writes"]
    for kname, sel in (("kind0", valid & (kind == 0)), ("kind1", valid & (kind == 1)), ("all", valid)):
        if not sel.any():
            continue
        print(f"-- {kname}: codes/item {n[sel].mean():.0f}, pairs {cnt[sel].mean():.2f}, blocks {nblk[sel].mean():.2f}")
        for i, nm in enumerate(names):
            v = (t[i + 1] - t[i])[sel]
            print(f"   {nm:12s} cycles mean {v.mean():8.0f} p50 {np.median(v):8.0f} p90 {np.percentile(v, 90):8.0f}")
        tg = a[:, :, 7][sel]
        print(f"   of scan: gathers {tg.mean():8.0f} ({(tg / np.maximum(nblk[sel], 1)).mean():.0f} per block), "
              f"admission + drains {((t[4] - t[3])[sel] - tg).mean():8.0f}")
        nd, td, npu, na = a[:, :, 8][sel], a[:, :, 9][sel], a[:, :, 10][sel], a[:, :, 11][sel]
        print(f"   drains/item {nd.mean():.2f} ({td.mean():.0f} cycles), pushed/item {npu.mean():.1f}, "
              f"super-batches with candidates {(na & 0xFFFF).mean():.2f}, loose {(na >> 16).mean():.2f}")
        tot = (t[5] - t[0])[sel]
        print(f"   item total   mean {tot.mean():8.0f}; scan cycles per block {((t[4] - t[3])[sel] / np.maximum(nblk[sel], 1)).mean():.0f}")
    first = np.where(valid, t[0], np.iinfo(np.int64).max).min(1)
    last = np.where(valid, t[5], 0).max(1)
    act = valid.any(1)
    g0 = first[act].min()
    print(f"kernel span {last[act].max() - g0} cycles; WG end offset p10 {np.percentile(last[act] - g0, 10):.0f} "
          f"p50 {np.median(last[act] - g0):.0f} max {(last[act] - g0).max()}")


if __name__ == "__main__":
    main()
