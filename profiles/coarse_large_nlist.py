#!/usr/bin/env python3
"""Coarse-quantizer time per 1024 queries at large nlist (SURVEY.md §8(f) row 3,
C4 shape: d = 96, nlist = 65536, nprobe = 32; and C2's nlist = 1024 for scale).

The coarse stage is k_coarse_gemm (key tiles on v_mfma_f32_16x16x4_f32, plus the
T3 workgroups when a search builds T3) followed by k_coarse_select (top-nprobe).
coarse_device runs the key tiles and the selection only.  Centroids and codebook
are random (timing does not depend on training).  Prints one JSON line per shape:
ms per 1024 queries from torch events on the launch stream, and the key-GEMM
rate (2 B nlist d flop).
"""
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "chameleon-rag-acceleration_amd"))


def main():
    import numpy as np
    import torch

    import faiss_amd as faiss

    rng = np.random.default_rng(0)
    for d, nlist, M, nprobe in ((128, 1024, 16, 16), (96, 65536, 48, 32), (768, 4096, 64, 32)):
        ix = faiss.IndexIVFPQ(None, d, nlist, M, 8, device=0)
        ix.set_trained(rng.standard_normal((nlist, d), dtype=np.float32),
                       rng.standard_normal((M, 256, d // M), dtype=np.float32))
        ix.nprobe = nprobe
        B = 1024
        x = torch.from_numpy(rng.standard_normal((B, d), dtype=np.float32)).cuda()
        for _ in range(3):
            ix.coarse_device(x)
        torch.cuda.synchronize()
        reps = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            ix.coarse_device(x)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(json.dumps({"d": d, "nlist": nlist, "nprobe": nprobe, "batch": B, "coarse_ms_per_batch": ms,
                          "key_gemm_tflops": 2.0 * B * nlist * d / (ms * 1e-3) / 1e12,
                          "key_matrix_bytes": B * nlist * 4}), flush=True)
        del ix


if __name__ == "__main__":
    main()
