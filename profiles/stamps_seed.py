"""Summarize the seed-pass stamps appended after the phase-B stamps in an IVFPQ_STAMPS dump."""
import sys

import numpy as np

GRID, ITEMS, SLOTS = int(sys.argv[2]) if len(sys.argv) > 2 else 512, 32, 6
a = np.fromfile(sys.argv[1], dtype=np.uint64)
seed = a[GRID * ITEMS * SLOTS:].reshape(-1, 4).astype(np.int64)
ok = (seed[:, 0] > 0) & (seed[:, 3] > 0)
s = seed[ok]
for name, v in (("T3+LUT", s[:, 1] - s[:, 0]), ("scan+topk", s[:, 2] - s[:, 1]), ("write", s[:, 3] - s[:, 2]),
                ("total", s[:, 3] - s[:, 0])):
    print(f"{name:10s} cycles mean {v.mean():8.0f} p50 {np.median(v):8.0f} p90 {np.percentile(v, 90):8.0f} max {v.max():8.0f}")
print("queries stamped", ok.sum())
