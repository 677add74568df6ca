#!/usr/bin/env python3
"""C4 (BASELINE.json configs[3]) per-GPU shard at its real size, on one GPU.

Deep1B-shaped: d 96, nlist 65536, M 48 (48-B codes), nprobe 32, k 10, batches of
1024 queries.  C4 is 1e9 vectors list-range sharded over 8 GPUs; this run builds
rank 0's shard -- lists [0, 8192), about 1e9 / 8 = 125 M vectors, 6 GB of codes --
entirely on the GPU ("synthetic, generated per shard on
device"):

  1. train IVF65536,PQ48 on a 300k-vector sample of the synthetic Deep-like
     distribution (datasets.synthetic_sift_like, 200k centres) on the GPU;
  2. generate the shard's base vectors on the device, in slices, around the
     centroids of the shard's lists (c_l + N(0, 16^2), rounded and clipped like
     the generator), and add them with add_device: coarse assignment on the
     matrix cores, PQ encode, list-image merge -- vectors assigned outside the
     shard's range are dropped, as rank 0 of bench_gpu_1bn.py's sharded add keeps
     its own lists (reference: bench_gpu_1bn.py:598-658);
  3. search 1024-query batches from the global distribution with search_device
     (the shard scans only the probes landing in its lists, as in the shard flow);
     HIP events around the list-scan kernel give the roofline line.

Prints one JSON line in bench.py's format (config C4-shard), with the add
throughput and, with --check, a bit-exact check of 64 queries against the oracle.
"""
import argparse
import json
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "chameleon-rag-acceleration_amd"))
HBM_PEAK_GBPS = 8000.0


def log(*a):
    print("[c4]", *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nb", type=int, default=125_000_000, help="base vectors to generate for the shard")
    ap.add_argument("--slice", type=int, default=16_000_000)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--nt", type=int, default=300_000)
    ap.add_argument("--niter", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--nbatches", type=int, default=4)
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import torch

    import faiss_amd as faiss
    from faiss_amd import datasets

    d, nlist, M, nprobe, k, B = 96, 65536, 48, 32, 10, 1024
    dev = torch.device("cuda", 0)
    t0 = time.time()
    xt = datasets.synthetic_sift_like(a.nt, d, seed=4321 + 11, n_centres=200_000)
    ix = faiss.index_factory(d, f"IVF{nlist},PQ{M}", device=0)
    ix.niter_coarse = ix.niter_pq = a.niter
    ix.train(xt)
    log(f"trained in {time.time() - t0:.1f}s")
    lo, hi = 0, nlist // a.shards
    ix.set_list_range(lo, hi)
    cent = torch.from_numpy(ix.centroids()[lo:hi]).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    t0 = time.time()
    added = 0
    torch.cuda.synchronize()
    for i0 in range(0, a.nb, a.slice):
        n = min(a.slice, a.nb - i0)
        which = torch.randint(0, hi - lo, (n,), device=dev, generator=g)
        x = cent[which] + 16.0 * torch.randn((n, d), device=dev, generator=g)
        x = torch.clamp(torch.round(x), 0, 255).contiguous()
        ix.add_device(x)
        added += n
        del x, which
        log(f"generated {added}, shard holds {ix.ntotal} ({time.time() - t0:.1f}s)")
    torch.cuda.synchronize()
    t_add = time.time() - t0
    ix.nprobe = nprobe
    xq = torch.from_numpy(datasets.synthetic_sift_like(a.nbatches * B, d, seed=123, n_centres=200_000)).to(dev)
    xq = xq.view(a.nbatches, B, d)
    Dbuf = torch.empty((B, k), dtype=torch.float32, device=dev)
    Ibuf = torch.empty((B, k), dtype=torch.int64, device=dev)
    # algorithmic bytes per batch: codes of the probes that land in the shard's lists
    off_sizes = None
    bytes_alg = []
    for b in range(a.nbatches):
        _, Iq = ix.coarse_device(xq[b])
        Iq = Iq.cpu().numpy()
        if off_sizes is None:
            off_sizes = ix.invlists.list_sizes()  # from the device offsets
        sz = np.where(Iq >= 0, off_sizes[np.maximum(Iq, 0)], 0)
        bytes_alg.append(int(sz.sum()) * M)
    for w in range(3):
        ix.search_device(xq[w % a.nbatches], k, Dbuf, Ibuf)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(a.steps):
        ix.set_timing(True, lists_only=True)
        ix.search_device(xq[s % a.nbatches], k, Dbuf, Ibuf)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ix.set_timing(False)
    st = ix.get_timing()
    lists_ms, lists_n = st["lists"]
    avg = lists_ms / max(lists_n, 1)
    bpl = sum(bytes_alg[s % a.nbatches] for s in range(a.steps)) / a.steps
    ach = bpl / (avg * 1e-3) / 1e9
    check = None
    if a.check:
        from oracle import oracle as O

        log("oracle check: 64 queries")
        ox = O.OracleIVFPQ(d, nlist, M)
        ox.set_trained(ix.centroids(), ix.codebook())
        for l in range(lo, hi):
            ox.list_ids[l] = ix.invlists.get_ids(l)
            ox.list_codes[l] = ix.invlists.get_codes(l).reshape(-1, M)
        ox.ntotal = ix.ntotal
        ox.nprobe = nprobe
        q = xq[0, :64].cpu().numpy()
        D, I = ix.search(q, k)
        Dr, Ir = ox.search(q, k)
        check = {"queries": 64, "ids_equal": bool(np.array_equal(I, Ir)), "dist_equal": bool(np.array_equal(D, Dr))}
    out = {
        "metric": "queries/sec, Deep1B-shaped IVF-PQ shard (nlist=65536, M=48, nprobe=32)",
        "value": a.steps * B / el,
        "unit": "queries/s",
        "n_gpus": 1,
        "steps": a.steps,
        "ms_per_step": el * 1000 / a.steps,
        "higher_is_better": True,
        "dtype": "f32",
        "data": "synthetic, generated on the device around the shard's list centroids (seed 1234); queries "
                "datasets.synthetic_sift_like(seed 123, 200k centres)",
        "config": {"workload": f"C4 shard {lo}..{hi} of {a.shards}: IVF{nlist},PQ{M}x8, d={d}, "
                               f"{ix.ntotal} vectors ({ix.ntotal * M / 1e9:.2f} GB codes), nprobe={nprobe}, k={k}, "
                               f"batch={B}", "shards": a.shards},
        "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": ach / HBM_PEAK_GBPS, "traffic": None, "kernel": "k_scan_lists<48,1,1,4>",
                     "alg_bytes_per_launch": bpl, "avg_launch_ms": avg},
        "add": {"vectors_generated": added, "kept": int(ix.ntotal), "seconds": t_add,
                "vectors_per_s": added / t_add},
        "check": check,
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
