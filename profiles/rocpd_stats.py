"""Per-kernel launch count / mean / total duration from a rocprofv3 rocpd database
(ROCm 7 writes run_results.db unless --output-format csv is given).
Usage: rocpd_stats.py <db or dir> [name regex] [grid_x filter]"""
import glob
import os
import re
import sqlite3
import sys


def stats(path, rx=".*"):
    db = path if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name, grid_x, workgroup_x, duration from kernels").fetchall()
    agg = {}
    for name, gx, wx, dur in rows:
        n = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "").replace("chivf::", "").replace("void ", ""))
        if not re.search(rx, n):
            continue
        key = (n, gx // max(wx, 1))
        a = agg.setdefault(key, [0, 0.0])
        a[0] += 1
        a[1] += dur
    out = []
    for (n, g), (cnt, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        out.append((n, g, cnt, tot / cnt / 1e3, tot / 1e3))
    return out


if __name__ == "__main__":
    print(f"{'kernel':60s} {'wgs':>7s} {'calls':>6s} {'mean_us':>9s} {'total_us':>10s}")
    for n, g, cnt, mean, tot in stats(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ".*"):
        print(f"{n[:60]:60s} {g:7d} {cnt:6d} {mean:9.2f} {tot:10.1f}")
