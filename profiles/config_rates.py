#!/usr/bin/env python3
"""Search throughput at the other BASELINE.json configs (one GPU, device entry
points, queries resident in HBM), next to bench.py's C2 line:

  C1  SIFT1M-shaped IVF1024,PQ16, nprobe 8, k 10 (bench.py's index, other nprobe)
  C2  bench.py's index (200k centres), nprobe 16, k 10 and k 100
  C3  BEIR-NQ-shaped: d 768, nb 2.68 M, IVF4096,PQ64, nprobe 32, METRIC_INNER_PRODUCT,
      k 10 and k 1000 (beir EvaluateRetrieval's top_k, evaluation.py:13)
  C4  Deep1B-shaped single-GPU shard at reduced size: d 96, nb --c4-nb, IVF65536,PQ48,
      nprobe 32, k 10 (the 1e9 / 8-GPU case is not run here)

Synthetic clustered data (faiss_amd.datasets.synthetic_sift_like; for C3 centred and
normalised to unit rows like sentence embeddings), GPU-trained with
few iterations (rates do not depend on training quality).  Prints one JSON line per
(config, k): queries/s and ms per 1024-query batch, from torch events on the
launch stream over --reps batches, and the same with two batches in flight on two
streams (wall clock).
"""
import argparse
import json
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "chameleon-rag-acceleration_amd"))


def rate(ix, xq_dev, k, reps):
    import torch

    B = 1024
    nb = xq_dev.shape[0] // B
    D = torch.empty((B, k), dtype=torch.float32, device=xq_dev.device)
    I = torch.empty((B, k), dtype=torch.int64, device=xq_dev.device)
    for b in range(min(3, nb)):
        ix.search_device(xq_dev[b * B:(b + 1) * B], k, D, I)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for r in range(reps):
        b = r % nb
        ix.search_device(xq_dev[b * B:(b + 1) * B], k, D, I)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    # the same batches two in flight (batch r on stream r % 2, own outputs; wall clock
    # between device-wide synchronisations), as bench.py's timed region
    import faiss_amd

    if not faiss_amd.overlap_built():  # the experimental overlap is not in this build (-DIVFPQ_OVERLAP=1)
        return {"k": k, "ms_per_batch": ms, "queries_per_s": B / (ms * 1e-3)}
    ss = [torch.cuda.Stream() for _ in range(2)]
    outs = [(D, I), (torch.empty_like(D), torch.empty_like(I))]
    ix.inflight = True
    for r in range(4):  # warm: each stream's workspace allocated before timing
        ix.search_device(xq_dev[(r % nb) * B:(r % nb + 1) * B], k, *outs[r % 2], stream=ss[r % 2].cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(reps):
        b = r % nb
        ix.search_device(xq_dev[b * B:(b + 1) * B], k, *outs[r % 2], stream=ss[r % 2].cuda_stream)
    torch.cuda.synchronize()
    ms2 = (time.perf_counter() - t0) * 1000.0 / reps
    ix.inflight = False
    return {"k": k, "ms_per_batch": ms, "queries_per_s": B / (ms * 1e-3),
            "ms_per_batch_inflight2": ms2, "queries_per_s_inflight2": B / (ms2 * 1e-3)}


def roofline(ix, xq_dev, k, M, steps=10):
    """bench.py's roofline block for the list-scan kernel of this index: algorithmic code
    bytes per batch (sum over queries and probes of the probed list's size x code size)
    over the kernel's HIP-event duration (one batch at a time), and the stage split."""
    import numpy as np
    import torch

    B = 1024
    nb = xq_dev.shape[0] // B
    sizes = ix.invlists.list_sizes()
    alg = []
    for b in range(nb):
        _, Iq = ix.coarse_device(xq_dev[b * B:(b + 1) * B])
        Iq = Iq.cpu().numpy()
        alg.append(int(np.where(Iq >= 0, sizes[np.maximum(Iq, 0)], 0).sum()) * M)
    D = torch.empty((B, k), dtype=torch.float32, device=xq_dev.device)
    I = torch.empty((B, k), dtype=torch.int64, device=xq_dev.device)
    ix.search_device(xq_dev[:B], k, D, I)
    torch.cuda.synchronize()
    ix.set_timing(True, lists_only=True)
    for s in range(steps):
        b = s % nb
        ix.search_device(xq_dev[b * B:(b + 1) * B], k, D, I)
    torch.cuda.synchronize()
    ix.set_timing(False)
    ms, n = ix.get_timing()["lists"]
    avg = ms / max(n, 1)
    bpl = sum(alg[s % nb] for s in range(steps)) / steps
    ix.set_timing(True)
    for s in range(steps):
        b = s % nb
        ix.search_device(xq_dev[b * B:(b + 1) * B], k, D, I)
    torch.cuda.synchronize()
    ix.set_timing(False)
    split = {st: v[0] / max(v[1], 1) for st, v in ix.get_timing().items()}
    ach = bpl / (avg * 1e-3) / 1e9
    return {"roofline": {"bound": "hbm", "kernel": "k_scan_lists", "alg_bytes_per_launch": bpl, "avg_launch_ms": avg,
                         "achieved": ach, "peak": 8000.0, "unit": "GB/s", "frac": ach / 8000.0},
            "stages_ms": split}


def embed_like(x, mu):
    """Centred, unit-norm rows (sentence-embedding-like): inner-product k-means on the raw
    non-negative synthetic data would put almost every vector in a few lists."""
    import numpy as np

    y = x - mu
    return np.ascontiguousarray(y / np.maximum(np.linalg.norm(y, axis=1, keepdims=True), 1e-6), np.float32)


def build(faiss, datasets, d, nlist, M, nb, nt, niter, metric, n_centres, seed0=0):
    ix = faiss.index_factory(d, f"IVF{nlist},PQ{M}", metric, device=0)
    ix.niter_coarse = ix.niter_pq = niter
    xt = datasets.synthetic_sift_like(nt, d, seed=4321 + seed0, n_centres=n_centres)
    ip = metric == faiss.METRIC_INNER_PRODUCT
    mu = xt.mean(0, keepdims=True) if ip else None
    ix.train(embed_like(xt, mu) if ip else xt)
    step = 500_000
    for i0 in range(0, nb, step):
        xb = datasets.synthetic_sift_like(min(step, nb - i0), d, seed=1000 + seed0 + i0, n_centres=n_centres)
        ix.add(embed_like(xb, mu) if ip else xb)
        print(f"[rates] d={d} nlist={nlist}: added {ix.ntotal}", file=sys.stderr, flush=True)
    sizes = ix.invlists.list_sizes()
    print(f"[rates] list sizes: mean {sizes.mean():.0f} max {sizes.max()} (imbalance "
          f"{(sizes.astype(float) ** 2).sum() * len(sizes) / max(sizes.sum(), 1) ** 2:.2f})", file=sys.stderr, flush=True)
    return ix, mu


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--c3-nb", type=int, default=2_680_000)
    ap.add_argument("--c4-nb", type=int, default=10_000_000)
    ap.add_argument("--only", default="c1,c3,c4")
    a = ap.parse_args()
    import torch

    import faiss_amd as faiss
    from faiss_amd import datasets

    only = set(a.only.split(","))
    if "c1" in only:
        t0 = time.time()
        ix, _ = build(faiss, datasets, 128, 1024, 16, 1_000_000, 100_000, 25, faiss.METRIC_L2, 10000)
        xq = torch.from_numpy(datasets.synthetic_sift_like(10240, 128, seed=123)).cuda()
        ix.nprobe = 8
        r = rate(ix, xq, 10, a.reps)
        r.update(roofline(ix, xq, 10, 16))
        print(json.dumps({"config": "C1 shape on GPU: SIFT1M-shaped IVF1024,PQ16 nprobe 8", **r,
                          "setup_s": time.time() - t0}), flush=True)
        del ix, xq
    if "c2" in only:
        t0 = time.time()
        ix, _ = build(faiss, datasets, 128, 1024, 16, 1_000_000, 100_000, 25, faiss.METRIC_L2, 200_000)
        xq = torch.from_numpy(datasets.synthetic_sift_like(10240, 128, seed=123)).cuda()
        ix.nprobe = 16
        for k in (10, 100):
            r = rate(ix, xq, k, a.reps)
            print(json.dumps({"config": "C2: SIFT1M-shaped IVF1024,PQ16 nprobe 16 (bench.py's index)", **r,
                              "setup_s": time.time() - t0}), flush=True)
        del ix, xq
    if "c3" in only:
        t0 = time.time()
        # the index tests/test_gpu_fullsize.py checks against the oracle (datasets.c3_nq_shaped)
        xt, base, xq = datasets.c3_nq_shaped(nb=a.c3_nb)
        ix = faiss.index_factory(768, "IVF4096,PQ64", faiss.METRIC_INNER_PRODUCT, device=0)
        ix.niter_coarse = ix.niter_pq = 6
        ix.train(xt)
        for xb in base():
            ix.add(xb)
        xq = torch.from_numpy(xq).cuda()
        ix.nprobe = 32
        for k in (10, 1000):
            r = rate(ix, xq, k, a.reps)
            r.update(roofline(ix, xq, k, 64))
            print(json.dumps({"config": f"C3 shape: d 768, nb {ix.ntotal}, IVF4096,PQ64, nprobe 32, inner product",
                              **r, "setup_s": time.time() - t0}), flush=True)
        del ix, xq
    if "c4" in only:
        t0 = time.time()
        ix, _ = build(faiss, datasets, 96, 65536, 48, a.c4_nb, 300_000, 4, faiss.METRIC_L2, 200000, 11)
        xq = torch.from_numpy(datasets.synthetic_sift_like(4096, 96, seed=123, n_centres=200000)).cuda()
        ix.nprobe = 32
        r = rate(ix, xq, 10, a.reps)
        r.update(roofline(ix, xq, 10, 48))
        print(json.dumps({"config": f"C4 shape, one shard: d 96, nb {ix.ntotal}, IVF65536,PQ48, nprobe 32", **r,
                          "setup_s": time.time() - t0}), flush=True)


if __name__ == "__main__":
    main()
