"""Per-phase breakdown of k_scan_pipe from a -DDIAG_PSTAMPS build.

Slots per (workgroup, phase), lane 0: 0 phase start (wave 0, after the barrier),
1 wave 8 after taking the next record, 2 / 3 waves 8 / 9 after their LUT build
(stores drained), 4..11 scan wave w done, 12 codes | pairs << 32 | kind << 40,
13 wave 0 scan start (after the partner merge).

Usage (GPU box):
  bash profiles/build_variants.sh pdiag:"-DDIAG_PSTAMPS"      # here, before gpurun
  IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/pdiag/libivfpq.so python3 profiles/diag_pipe.py
Builds bench.py's C2 index (200k-centre data), runs warm-up searches and one stamped search.
"""
import ctypes
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "chameleon-rag-acceleration_amd"))
WG, ITEMS, SLOTS = 1024, 64, 16


def pct(v):
    v = np.asarray(v, np.float64)
    return f"mean {v.mean():8.0f} p50 {np.median(v):8.0f} p90 {np.percentile(v, 90):8.0f}"


def main():
    import torch

    import faiss_amd as faiss
    from faiss_amd import _lib, datasets

    gen = dict(n_centres=200_000)
    xt = datasets.synthetic_sift_like(100_000, 128, seed=4321, **gen)
    xb = datasets.synthetic_sift_like(1_000_000, 128, seed=1234, **gen)
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
    ix.search_device(xd, 10)
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    a = buf.reshape(WG, ITEMS, SLOTS).astype(np.int64)
    t0 = a[:, :, 0]
    valid = (t0 > 0) & (a[:, :, 13] > 0)
    nxt = np.roll(t0, -1, axis=1)
    has_next = valid & (nxt > 0)
    phase = (nxt - t0)[has_next]
    take = (a[:, :, 1] - t0)[valid & (a[:, :, 1] > 0)]
    b8 = (a[:, :, 2] - t0)[valid & (a[:, :, 2] > 0)]
    b9 = (a[:, :, 3] - t0)[valid & (a[:, :, 3] > 0)]
    merge0 = (a[:, :, 13] - t0)[valid]
    scan = [(a[:, :, 4 + w] - t0)[valid] for w in range(8)]
    scan_max = np.max(np.stack([a[:, :, 4 + w] for w in range(8)]), axis=0)
    scan_min = np.min(np.stack([a[:, :, 4 + w] for w in range(8)]), axis=0)
    n = a[:, :, 12] & 0xFFFFFFFF
    cnt = (a[:, :, 12] >> 32) & 0xFF
    kind = (a[:, :, 12] >> 40) & 1
    print(f"phases {valid.sum()} (kind0 {(valid & (kind == 0)).sum()}); codes/item {n[valid].mean():.0f}, "
          f"pairs/item {cnt[valid].mean():.2f}; phases per WG {valid.sum(1)[valid.any(1)].mean():.1f}")
    print("phase length (start -> next start)", pct(phase))
    print("wave 8 take done                  ", pct(take))
    print("wave 8 build done                 ", pct(b8))
    print("wave 9 build done                 ", pct(b9))
    print("wave 0 partner merge done         ", pct(merge0))
    for w in range(8):
        print(f"scan wave {w} done                 ", pct(scan[w]))
    print("slowest scan wave done            ", pct((scan_max - t0)[valid]))
    print("scan spread (slowest - fastest)   ", pct((scan_max - scan_min)[valid]))
    bound_by = np.where(np.maximum(a[:, :, 2], a[:, :, 3]) > scan_max, "loader", "scan")[has_next]
    print("phase bound by loaders:", float((bound_by == "loader").mean()))


if __name__ == "__main__":
    main()
