"""Counter traffic of the C4 shard's list-scan kernel (profiles/r06_c4.sh): per-launch
HBM bytes from separate rocprofv3 --pmc passes of profiles/c4_shard.py (FETCH_SIZE x 2 per
the gfx950 correction of MI355X_MICROARCH.md + WRITE_SIZE, the unit checked against
TCC_EA0_RDREQ_sum x 64 B as make_pmc_json.py does), written into the shard's JSON line.
Usage: c4_traffic.py <pmc dir with g*/run_counter_collection.csv> <c4 json> <out json>"""
import collections
import csv
import glob
import json
import os
import sys


def main(d, src, out):
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "g*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if "k_scan_lists" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    mean = {c: sum(v) / len(v) for c, v in agg.items()}
    f, w, rq = mean.get("FETCH_SIZE"), mean.get("WRITE_SIZE"), mean.get("TCC_EA0_RDREQ_sum")
    unit = 1024.0
    if f and rq:
        unit = 1024.0 if abs(f * 1024.0 / (rq * 64.0) - 1.0) < 0.25 else 1.0
    j = json.loads(open(src).read().strip().splitlines()[-1])
    j["roofline"]["traffic"] = 2.0 * f * unit + w * unit if f is not None and w is not None else None
    j["roofline"]["traffic_source"] = {"dir": os.path.relpath(d), "FETCH_SIZE": f, "WRITE_SIZE": w,
                                       "TCC_EA0_RDREQ_sum": rq, "unit_bytes": unit,
                                       "launches": len(agg.get("FETCH_SIZE", []))}
    json.dump(j, open(out, "w"))
    print(json.dumps(j["roofline"]))


if __name__ == "__main__":
    main(*sys.argv[1:4])
