"""One-GPU emulation of bench.py's shard flow at N = 1, 2, 4, 8 (C2 index):
per-rank times of rank 0 (lists [lo_0, hi_0) of a balanced N-way cut) for a
global batch of 1024 x N queries.

  coarse   : coarse_device on the rank's own 1024-query slice (flat in N)
  preassigned: search_preassigned_device of the whole batch on the rank's lists
               (plan + scan + merge; T3 for the batch is computed on a side stream
               concurrently with the coarse step, as bench.py does), with the stage
               split of a run without the side stream (ms): tables (T3, grows with
               the batch), scan
  merge    : merge_topk_device of the rank's slice over N partials

  step_wall_ms: the whole per-rank step by wall clock, one batch at a time and with two
               batches in flight on two streams (as bench.py runs it)

Collectives are not run (one GPU): their per-rank bytes are printed instead
(all_gather of the probes: N x 1024 x nprobe x 12 B; all_to_all of partials:
N x 1024 x k x 12 B).  Usage: python3 profiles/shard_emulation.py [--nb 1000000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "chameleon-rag-acceleration_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nb", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch

    import faiss_amd as faiss
    from faiss_amd import datasets
    from faiss_amd.sharding import balanced_list_ranges

    k, B, npb = 10, 1024, 16
    xt = datasets.synthetic_sift_like(100_000, 128, seed=4321)
    xb = datasets.synthetic_sift_like(args.nb, 128, seed=1234)
    xq = datasets.synthetic_sift_like(8 * B, 128, seed=123)
    full = faiss.index_factory(128, "IVF1024,PQ16")
    full.train(xt)
    full.add(xb)
    full.nprobe = npb
    sizes = full.invlists.list_sizes()
    xd = torch.from_numpy(xq).cuda()
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    out = []
    for N in (1, 2, 4, 8):
        lo, hi = balanced_list_ranges(sizes, N, 16)[0]
        sh = faiss.IndexIVFPQ(None, 128, 1024, 16, 8, device=0)
        sh.set_trained(full.centroids(), full.codebook())
        sh.set_list_range(lo, hi)
        ls = [l for l in range(lo, hi) if sizes[l]]
        sh.add_preencoded(np.concatenate([np.full(sizes[l], l, np.int64) for l in ls]),
                          np.concatenate([full.invlists.get_codes(l).reshape(-1, 16) for l in ls]),
                          np.concatenate([full.invlists.get_ids(l) for l in ls]))
        sh.nprobe = npb
        xg = xd[:N * B]
        Dq_all, Iq_all = full.coarse_device(xg)  # stands in for the all-gathered probes
        t = {"coarse": 0.0, "preassigned": 0.0, "merge": 0.0}
        side = torch.cuda.Stream()
        for rep in range(args.reps + 2):
            e = [ev() for _ in range(4)]
            e[0].record()
            # T3 of the global batch on a side stream, concurrent with the coarse step (bench.py's shard flow)
            side.wait_stream(torch.cuda.current_stream())
            tok = sh.precompute_tables_device(xg, stream=side.cuda_stream)
            sh.coarse_device(xg[:B])
            e[1].record()
            Dp, Ip = sh.search_preassigned_device(xg, k, Iq_all, Dq_all, tables=tok)
            e[2].record()
            faiss.merge_topk_device(torch.stack([Dp[:B]] * N), torch.stack([Ip[:B]] * N))
            e[3].record()
            torch.cuda.synchronize()
            if rep >= 2:
                t["coarse"] += e[0].elapsed_time(e[1]) / args.reps
                t["preassigned"] += e[1].elapsed_time(e[2]) / args.reps
                t["merge"] += e[2].elapsed_time(e[3]) / args.reps
        # the whole per-rank step (T3 ahead on a side stream, coarse of the own slice,
        # preassigned search, merge), wall clock over reps steps: one stream, then
        # two batches in flight (step s on compute stream s % 2 with its own side stream)
        comp = [torch.cuda.Stream() for _ in range(2)]
        sides = [torch.cuda.Stream() for _ in range(2)]
        outs = [(torch.empty((N * B, k), device="cuda"), torch.empty((N * B, k), dtype=torch.int64, device="cuda"))
                for _ in range(2)]

        def rank_step(j):
            with torch.cuda.stream(comp[j]):
                sides[j].wait_stream(comp[j])
                tok = sh.precompute_tables_device(xg, stream=sides[j].cuda_stream)
                sh.coarse_device(xg[:B])
                Dp, Ip = sh.search_preassigned_device(xg, k, Iq_all, Dq_all, *outs[j], tables=tok)
                faiss.merge_topk_device(torch.stack([Dp[:B]] * N), torch.stack([Ip[:B]] * N))

        wall = {}
        for label, depth in (("serial", 1), ("inflight2", 2))[:2 if faiss.overlap_built() else 1]:
            sh.inflight = depth > 1
            for s in range(4):
                rank_step(s % depth)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for s in range(args.reps * 5):
                rank_step(s % depth)
            torch.cuda.synchronize()
            wall[label] = (time.perf_counter() - t0) * 1000.0 / (args.reps * 5)
        sh.set_timing(True)
        for _ in range(args.reps):
            sh.search_preassigned_device(xg, k, Iq_all, Dq_all)
        torch.cuda.synchronize()
        sh.set_timing(False)
        st = sh.get_timing()
        split = {s: v[0] / max(v[1], 1) for s, v in st.items()}
        row = {"N": N, "lists": [lo, hi], "batch": N * B, "ms": t, "step_wall_ms": wall,
               "preassigned_stages_ms": split,
               "allgather_bytes_per_rank": N * B * npb * 12, "alltoall_bytes_per_rank": N * B * k * 12}
        print(json.dumps(row), flush=True)
        out.append(row)


if __name__ == "__main__":
    main()
