"""Summarize the search-phase kernels of a rocprofv3 kernel trace (last N steps)."""
import collections
import csv
import re
import sys


def short(name):
    name = re.sub(r"^void ", "", name)
    name = name.replace("(anonymous namespace)::", "")
    base = name.split("(")[0]
    return base.replace("chivf::(anonymous namespace)::", "")


def main(path, steps):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    enc = [i for i, r in enumerate(rows) if "pq_encode" in r["Kernel_Name"]]
    tail = rows[enc[-1] + 1:] if enc else rows
    agg = collections.OrderedDict()
    for r in tail:
        n = short(r["Kernel_Name"])
        agg.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    print(f"{'kernel':48s} {'calls':>6s} {'mean_us':>9s} {'min_us':>9s} {'total_us':>10s}")
    for n, v in agg.items():
        print(f"{n[:48]:48s} {len(v):6d} {sum(v)/len(v):9.2f} {min(v):9.2f} {sum(v):10.1f}")
    # one step's timeline (last scan_lists / scan_topk group)
    last = tail[-12:]
    t0 = int(last[0]["Start_Timestamp"])
    print("\nlast dispatches (start offset us, duration us):")
    for r in last:
        print(f"  {short(r['Kernel_Name'])[:44]:44s} +{(int(r['Start_Timestamp'])-t0)/1000:8.2f} "
              f"{(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000:8.2f} grid={r.get('Grid_Size_X','?')}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
