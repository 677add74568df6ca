"""Phase breakdown of k_coarse_fused from a DIAG_CSTAMPS build.

k_coarse_gemm slots per (workgroup, wave): 0 start, 1 after the query tile
fill, 2 after |x|^2 and the MFMA loop (key tiles), 5 at the end (stores drained).

Usage: bash profiles/build_variants.sh cdiag:"-DDIAG_CSTAMPS=1"   # here
       IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/cdiag/libivfpq.so python3 profiles/diag_coarse.py
"""
import ctypes
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "chameleon-rag-acceleration_amd"))
WG, ITEMS, SLOTS = 1024, 64, 8


def main():
    import torch

    import faiss_amd as faiss
    from faiss_amd import _lib, datasets

    nb = int(os.environ.get("NB", "1000000"))
    gen = dict(n_centres=200_000)  # bench.py's data
    xt = datasets.synthetic_sift_like(100_000, 128, seed=4321, **gen)
    xb = datasets.synthetic_sift_like(nb, 128, seed=1234, **gen)
    xq = datasets.synthetic_sift_like(1024, 128, seed=123, **gen)
    ix = faiss.index_factory(128, "IVF1024,PQ16")
    ix.train(xt)
    ix.add(xb)
    ix.nprobe = 16
    xd = torch.from_numpy(xq).cuda()
    fn = _lib.load().ivfpq_diag_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros(WG * ITEMS * SLOTS, np.uint64)
    for _ in range(5):
        ix.search_device(xd, 10)
    torch.cuda.synchronize()
    fn(buf.ctypes.data, buf.nbytes)
    mode = os.environ.get("MODE", "search")
    if mode == "search":  # stamps of a search's coarse kernels (after the previous search's merge)
        ix.search_device(xd, 10)
    else:  # MODE=coarse2: the coarse step twice back to back, stamps of the second (warm start)
        ix.coarse_device(xd)
        ix.coarse_device(xd)
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    full = buf.reshape(WG, ITEMS, SLOTS).astype(np.int64)
    a = full[:, :4, :6]
    b = full[:, 4:8, :6]
    ok = (b[:, :, 0] > 0) & (b[:, :, 5] > 0)
    if ok.any():
        print(f"-- select: waves {ok.sum()}")
        for i, j, nm in ((0, 1, "loads+min"), (1, 2, "kth"), (2, 3, "cut+sort"), (3, 5, "out+plan")):
            v = (b[:, :, j] - b[:, :, i])[ok]
            print(f"  {nm:13s} mean {v.mean():8.0f} p50 {np.median(v):8.0f} p90 {np.percentile(v, 90):8.0f} max {v.max():8.0f}")
    ngemm = int(os.environ.get("NGEMM", "256"))
    for role, rng, phases in (("keys", range(0, ngemm), [(0, 1, "fill"), (1, 2, "xn+mfma"), (2, 5, "epilogue")]),
                              ("T3", range(ngemm, WG), [(0, 1, "fill"), (1, 5, "trees+stores")])):
        sel = np.zeros(WG, bool)
        sel[list(rng)] = True
        ok = sel[:, None] & (a[:, :, 0] > 0) & (a[:, :, 5] > 0)
        if not ok.any():
            continue
        print(f"-- {role}: waves {ok.sum()}")
        for i, j, nm in phases:
            v = (a[:, :, j] - a[:, :, i])[ok]
            print(f"  {nm:13s} mean {v.mean():8.0f} p50 {np.median(v):8.0f} p90 {np.percentile(v, 90):8.0f} max {v.max():8.0f}")
        tot = (a[:, :, 5] - a[:, :, 0])[ok]
        print(f"  total         mean {tot.mean():8.0f} max {tot.max():8.0f} cycles")
        allok = (a[:, :, 0] > 0) & (a[:, :, 5] > 0)
        t0 = a[:, :, 0][allok].min()
        st, en = (a[:, :, 0] - t0)[ok], (a[:, :, 5] - t0)[ok]
        q = [0, 10, 50, 90, 100]
        print("  start (from the first wave) p0/10/50/90/100", [int(np.percentile(st, x)) for x in q])
        print("  end                          p0/10/50/90/100", [int(np.percentile(en, x)) for x in q])


if __name__ == "__main__":
    main()
