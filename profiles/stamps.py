"""Summarize phase-B in-kernel stamps (IVFPQ_STAMPS dump): per-item segment cycles."""
import sys

import numpy as np

GRID, ITEMS, SLOTS = int(sys.argv[2]) if len(sys.argv) > 2 else 512, 32, 6
a = np.fromfile(sys.argv[1], dtype=np.uint64)[:GRID * ITEMS * SLOTS].reshape(-1, ITEMS, SLOTS).astype(np.int64)
valid = a[:, :, 0] > 0
t0, t1, t2, t3, n, cnt = [a[:, :, i] for i in range(6)]
load = (t1 - t0)[valid]
scan = (t2 - t1)[valid]
merge = (t3 - t2)[valid]
ns = n[valid]
print(f"items {valid.sum()}  per-WG items mean {valid.sum(1).mean():.1f} max {valid.sum(1).max()}")
for name, v in (("load+LUT", load), ("scan", scan), ("merge", merge)):
    print(f"{name:9s} cycles: mean {v.mean():8.0f} p50 {np.median(v):8.0f} p90 {np.percentile(v,90):8.0f} max {v.max():8.0f}")
print(f"codes/item mean {ns.mean():.0f}; scan cycles per code {scan.sum()/ns.sum():.2f}")
# WG span and gaps
first = np.where(valid, t0, np.iinfo(np.int64).max).min(1)
last = np.where(valid, t3, 0).max(1)
span = (last - first)[valid.any(1)]
busy = ((t3 - t0) * valid).sum(1)[valid.any(1)]
g0 = first[valid.any(1)].min()
print(f"WG span cycles mean {span.mean():.0f} max {span.max():.0f}; busy frac {busy.sum()/span.sum():.3f}")
print(f"WG start offset (cycles) p50 {np.median(first[valid.any(1)]-g0):.0f} max {(first[valid.any(1)]-g0).max():.0f}")
