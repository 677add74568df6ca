"""Coarse-step ablations (profiles/r06_gemm_ab.sh): an IVF1024,PQ16 index at C2's shape
(random centroids and codebook, 200k random codes added on the device) runs N rounds of
coarse_device (key-only k_coarse_gemm + k_coarse_select) and search_device (the search's
k_coarse_gemm with its T3 workgroups, select with planning, scan, merge) on 1024-query
batches.  Run it under rocprofv3 --kernel-trace --stats with IVFPQ_LIB pointing at a
-DGEMM_AB=<n> build: the kernel durations are the measurement (results are not checked;
the ablations compute wrong keys on purpose)."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "chameleon-rag-acceleration_amd"))


def main(rounds=200):
    import numpy as np
    import torch

    import faiss_amd as faiss

    d, nlist, M = 128, 1024, 16
    rng = np.random.default_rng(1)
    ix = faiss.IndexIVFPQ(None, d, nlist, M, 8, device=0)
    ix.set_trained((rng.random((nlist, d)) * 255).astype(np.float32),
                   (rng.standard_normal((M, 256, d // M)) * 16).astype(np.float32))
    dev = torch.device("cuda", 0)
    ix.add_device(torch.rand((200_000, d), device=dev) * 255)
    ix.nprobe = 16
    xq = torch.rand((4, 1024, d), device=dev) * 255
    Dq = torch.empty((1024, 10), dtype=torch.float32, device=dev)
    Iq = torch.empty((1024, 10), dtype=torch.int64, device=dev)
    for r in range(rounds):
        ix.coarse_device(xq[r % 4])
    torch.cuda.synchronize()
    for r in range(rounds):
        ix.search_device(xq[r % 4], 10, Dq, Iq)
    torch.cuda.synchronize()
    print("done", rounds)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 200)
