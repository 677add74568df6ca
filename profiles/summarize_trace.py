"""Summarize the search-phase kernels of a rocprofv3 kernel trace (last N steps).

With --passes W K (the bench's --warmup and --steps), the C2 list-scan kernel's
launches are also split by bench pass, in issue order: W warmup, K timed (the
pipelined region the bench's value and roofline come from), K serial (one
stream, reported as roofline.isolated), K stage split.  Usage:
  summarize_trace.py run_kernel_trace.csv [N] [--passes W K]
"""
import collections
import csv
import re
import sys


def short(name):
    name = re.sub(r"^void ", "", name)
    name = name.replace("(anonymous namespace)::", "")
    base = name.split("(")[0]
    return base.replace("chivf::(anonymous namespace)::", "")


def main(path, steps, passes=None):
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
    if passes:
        w, k = passes
        scans = [n for n in agg if "k_scan_lists<16, 4, 1" in n or "k_scan_lean<16" in n]
        if scans:
            name = scans[0]
            rs = [r for r in tail if short(r["Kernel_Name"]) == name]
            print(f"\n{name} by bench pass (mean us per launch; timed wall per step from the trace):")
            for label, a in (("warmup", 0), ("timed", w), ("serial", w + k), ("stages", w + 2 * k)):
                b = a + (w if label == "warmup" else k)
                seg = rs[a:b]
                if not seg:
                    continue
                d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0 for r in seg]
                span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1000.0
                print(f"  {label:7s} launches {len(seg):4d} mean {sum(d)/len(d):8.2f} us  "
                      f"first-start..last-end {span:9.1f} us ({span/max(len(seg)-1,1):7.2f} us per launch interval)")
    # one step's timeline (last scan_lists / scan_topk group)
    last = tail[-12:]
    t0 = int(last[0]["Start_Timestamp"])
    print("\nlast dispatches (start offset us, duration us):")
    for r in last:
        print(f"  {short(r['Kernel_Name'])[:44]:44s} +{(int(r['Start_Timestamp'])-t0)/1000:8.2f} "
              f"{(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000:8.2f} grid={r.get('Grid_Size_X','?')}")


if __name__ == "__main__":
    argv = sys.argv[1:]
    ps = None
    if "--passes" in argv:
        i = argv.index("--passes")
        ps = (int(argv[i + 1]), int(argv[i + 2]))
        argv = argv[:i] + argv[i + 3:]
    main(argv[0], int(argv[1]) if len(argv) > 1 else 20, ps)
