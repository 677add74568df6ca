#!/usr/bin/env python3
"""r05: which tau lowering is wrong?  Runs race_diag's index and k = 10 batches with
three streams in flight on a library built by `race_variants.py taulog`, which logs
every tau_q lowering (batch output pointer, epoch, query, value, site, pair, list,
workgroup | wave << 16).  A lowering is WRONG when its value is below the query's
true final k-th key (the batch searched alone): it can prune a true candidate.
Prints one JSON line: per site the lowerings and wrong ones, the mismatching
rows, and the first wrong records."""
import ctypes
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "chameleon-rag-acceleration_amd"))


def main():
    import numpy as np
    import torch

    import faiss_amd as faiss
    from faiss_amd import _lib, datasets

    k = int(os.environ.get("TL_K", "10"))
    nst = int(os.environ.get("TL_STREAMS", "3"))
    rounds = int(os.environ.get("TL_ROUNDS", "200"))
    lib = _lib.load()
    xt = datasets.synthetic_sift_like(20_000, 64, seed=4321, n_centres=20_000)
    xb = datasets.synthetic_sift_like(100_000, 64, seed=1234, n_centres=20_000)
    xq = datasets.synthetic_sift_like(24 * 256, 64, seed=123, n_centres=20_000)
    ix = faiss.index_factory(64, "IVF256,PQ8", device=0)
    ix.niter_coarse = ix.niter_pq = 8
    ix.train(xt)
    ix.add(xb)
    ix.nprobe = 12
    nb = 24
    xd = torch.from_numpy(xq).cuda().view(nb, 256, 64)
    ref = []
    for b in range(nb):
        D, I = ix.search_device(xd[b], k)
        torch.cuda.synchronize()
        ref.append((D.cpu().numpy(), I.cpu().numpy()))
    cap = 1 << 22
    logbuf = torch.zeros(cap * 8, dtype=torch.int32, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(nst)]
    sites = {}
    wrong_recs = []
    bad_rows = 0
    bad_with_wrong = 0
    for rnd in range(rounds):
        outs = [(torch.empty((256, k), device="cuda"), torch.empty((256, k), dtype=torch.int64, device="cuda"))
                for _ in range(nb)]
        bmap = {outs[b][0].data_ptr() & 0xFFFFFFFF: b for b in range(nb)}
        torch.cuda.synchronize()
        assert lib.ivfpq_dbg_set_tlog(ctypes.c_void_p(logbuf.data_ptr()), ctypes.c_uint32(cap)) == 0
        ix.inflight = nst > 1
        try:
            for b in range(nb):
                ix.search_device(xd[b], k, outs[b][0], outs[b][1], stream=streams[b % nst].cuda_stream)
            torch.cuda.synchronize()
        finally:
            ix.inflight = False
        n = ctypes.c_uint32(0)
        lib.ivfpq_dbg_tlog_count(ctypes.byref(n))
        n = min(n.value, cap)
        L = logbuf[:n * 8].view(n, 8).cpu().numpy().astype(np.uint32)
        assert lib.ivfpq_dbg_set_tlog(ctypes.c_void_p(0), ctypes.c_uint32(0)) == 0
        badset = set()
        for b in range(nb):
            I = outs[b][1].cpu().numpy()
            D = outs[b][0].cpu().numpy()
            rows = np.nonzero((I != ref[b][1]).any(1) | (D != ref[b][0]).any(1))[0]
            for r in rows:
                badset.add((b, int(r)))
        bad_rows += len(badset)
        # value (order-preserving int) -> float key
        o = L[:, 3].view(np.int32)
        key = np.where(o >= 0, o, o ^ 0x7FFFFFFF).astype(np.int32).view(np.float32)
        bsel = np.array([bmap.get(int(p), -1) for p in L[:, 0]])
        qs = L[:, 2].astype(np.int64)
        ok = (bsel >= 0) & (qs < 256)
        truth = np.full(n, np.inf, np.float32)
        for b in range(nb):
            m = ok & (bsel == b)
            truth[m] = ref[b][0][qs[m], k - 1]
        wrong = ok & (key < truth)
        for st in np.unique(L[:, 4]):
            m = L[:, 4] == st
            e = sites.setdefault(int(st), [0, 0])
            e[0] += int(m.sum())
            e[1] += int((m & wrong).sum())
        wq = set(zip(bsel[wrong].tolist(), qs[wrong].tolist()))
        bad_with_wrong += len(badset & wq)
        for i in np.nonzero(wrong)[0][:max(0, 40 - len(wrong_recs))]:
            b, q = int(bsel[i]), int(qs[i])
            wrong_recs.append({"round": rnd, "batch": b, "q": q, "value": float(key[i]), "truth_kth": float(truth[i]),
                               "site": int(L[i, 4]), "pair": int(L[i, 5]), "pair_q": int(L[i, 5]) // 12,
                               "pair_p": int(L[i, 5]) % 12, "list": int(L[i, 6]), "block": int(L[i, 7] & 0xFFFF),
                               "wave": int(L[i, 7] >> 16), "epoch": int(L[i, 1]), "row_bad": (b, q) in badset})
    print(json.dumps({"k": k, "streams": nst, "rounds": rounds, "bad_rows": bad_rows,
                      "bad_rows_with_wrong_lowering": bad_with_wrong, "sites": sites, "wrong": wrong_recs}), flush=True)


if __name__ == "__main__":
    main()
