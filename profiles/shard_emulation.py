"""One-GPU emulation of bench.py's shard flow at N = 1, 2, 4, 8 (C2 index): the
per-rank step of rank 0 (lists [lo_0, hi_0) of a balanced N-way cut) for a global
batch of 1024 x N queries, in bench.py's r06 stream topology, with the collectives in
the loop as real RCCL calls of the N-way payload on a one-rank nccl group:

  step (stream j of 3 in flight): coarse_tables_device (coarse of the own 1024-query
        slice + T3 of the global batch, one launch); one collective launch with the
        all_to_all of stream j's previous batch's N x 1024 x k partials and the
        all_gather of this batch's N x 1024 x nprobe probes; merge_topk_device of the
        previous batch's N partials; search_preassigned_device of the global batch on
        the rank's lists

At world 1 the collectives copy to self, so their kernels and payloads are those of
rank 0 of an N-way run but no xGMI transfer happens; the gathered probes are a stand-in
(the full index's coarse result for the global batch is fed to the scan), so results are
not checked here -- bench.py --shard-at-1 and the gloo / one-GPU shard tests check them.

Prints one JSON line per N: step_wall_ms (serial and 3 in flight), the stage split of
the preassigned search, and the per-rank collective bytes.
Usage: python3 profiles/shard_emulation.py [--nb 1000000] [--reps 10]
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
    ap.add_argument("--inflight", type=int, default=3)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist

    import faiss_amd as faiss
    from faiss_amd import datasets
    from faiss_amd.sharding import balanced_list_ranges, exchange_and_gather, exchange_partials

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    group = dist.group.WORLD

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
        streams = [torch.cuda.Stream() for _ in range(args.inflight)]
        outs = [(torch.empty((N * B, k), device="cuda"), torch.empty((N * B, k), dtype=torch.int64, device="cuda"))
                for _ in range(args.inflight)]
        pend = [None] * args.inflight

        def back(j):
            Dp, Ip = pend[j]
            pend[j] = None
            with torch.cuda.stream(streams[j]):
                Ds, Is = exchange_partials(Dp, Ip, 1, group, force=True)  # N x B x k payload
                faiss.merge_topk_device(Ds.view(N, B, k), Is.view(N, B, k))

        def step(j):
            # bench.py's shard step: one collective launch carries stream j's previous
            # batch's all_to_all (N x B x k) and this batch's all_gather (N x B x nprobe)
            prev = pend[j]
            pend[j] = None
            with torch.cuda.stream(streams[j]):
                _, _, tok = sh.coarse_tables_device(xg[:B], xg)
                Ds, Is, _, _ = exchange_and_gather(prev[0] if prev else None, prev[1] if prev else None,
                                                   Dq_all, Iq_all, 1, group, force=True)
                if prev is not None:
                    faiss.merge_topk_device(Ds.view(N, B, k), Is.view(N, B, k))
                pend[j] = sh.search_preassigned_device(xg, k, Iq_all, Dq_all, *outs[j], tables=tok)

        def drain():
            for j in range(args.inflight):
                if pend[j] is not None:
                    back(j)

        wall = {}
        for label, depth in (("serial", 1), (f"inflight{args.inflight}", args.inflight)):
            sh.inflight = depth > 1
            for s in range(2 * depth):
                step(s % depth)
            drain()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for s in range(args.reps * 5):
                step(s % depth)
                if depth == 1:
                    drain()
            drain()
            torch.cuda.synchronize()
            wall[label] = (time.perf_counter() - t0) * 1000.0 / (args.reps * 5)
        sh.inflight = False
        sh.set_timing(True)
        for _ in range(args.reps):
            sh.search_preassigned_device(xg, k, Iq_all, Dq_all)
        torch.cuda.synchronize()
        sh.set_timing(False)
        st = sh.get_timing()
        split = {s: v[0] / max(v[1], 1) for s, v in st.items()}
        row = {"N": N, "lists": [lo, hi], "batch": N * B, "step_wall_ms": wall, "preassigned_stages_ms": split,
               "allgather_bytes_per_rank": N * B * npb * 12, "alltoall_bytes_per_rank": N * B * k * 12,
               "collectives": "RCCL, one-rank nccl group (self-copies of the N-way payload)"}
        print(json.dumps(row), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
