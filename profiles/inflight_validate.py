#!/usr/bin/env python3
"""Validation of the batches-in-flight mode at scale: bench.py's C2
index, 40 query batches of 1024, their results one batch at a time on one stream
as the reference, then every batch again issued round robin on 2, 3, 4 and 5
streams with no synchronisation and the handle's inflight mode on (6 rounds per
stream count, k = 10 and k = 100: 1 920 overlapped batches), compared bit for bit,
and the merge kernels' index-check count.  Prints one JSON line."""
import json
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "chameleon-rag-acceleration_amd"))


def main():
    import numpy as np
    import torch

    import faiss_amd as faiss
    from faiss_amd import datasets

    nb, B, rounds = 40, 1024, 6
    gen = dict(n_centres=200_000)
    xt = datasets.synthetic_sift_like(100_000, 128, seed=4321, **gen)
    xb = datasets.synthetic_sift_like(1_000_000, 128, seed=1234, **gen)
    xq = datasets.synthetic_sift_like(nb * B, 128, seed=123, **gen)
    ix = faiss.index_factory(128, "IVF1024,PQ16", device=0)
    ix.train(xt)
    ix.add(xb)
    ix.nprobe = 16
    xd = torch.from_numpy(xq).cuda().view(nb, B, 128)
    out = {"batches_per_k": 0, "mismatched_batches": 0, "by_config": {}}
    t0 = time.time()
    for k in (10, 100):
        ref = []
        for b in range(nb):
            D, I = ix.search_device(xd[b], k)
            torch.cuda.synchronize()
            ref.append((D.cpu().numpy(), I.cpu().numpy()))
        for nst in (2, 3, 4, 5):
            streams = [torch.cuda.Stream() for _ in range(nst)]
            outs = [(torch.empty((B, k), device="cuda"), torch.empty((B, k), dtype=torch.int64, device="cuda"))
                    for _ in range(nb)]
            bad = 0
            ix.inflight = True
            for r in range(rounds):
                for o in outs:
                    o[0].fill_(-1.0)
                    o[1].fill_(-2)
                torch.cuda.synchronize()
                for b in range(nb):
                    ix.search_device(xd[b], k, outs[b][0], outs[b][1], stream=streams[b % nst].cuda_stream)
                torch.cuda.synchronize()
                for b in range(nb):
                    if not (np.array_equal(outs[b][1].cpu().numpy(), ref[b][1])
                            and np.array_equal(outs[b][0].cpu().numpy(), ref[b][0])):
                        bad += 1
            ix.inflight = False
            out["by_config"][f"k{k}_streams{nst}"] = {"batches": rounds * nb, "mismatched": bad}
            out["mismatched_batches"] += bad
            out["batches_per_k"] += rounds * nb
    out["index_check_errors"] = ix.error_count()
    out["seconds"] = time.time() - t0
    from faiss_amd import _lib

    out["lib"] = os.path.relpath(_lib.LIB_PATH, R)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
