"""C3 (profiles/r06_c3.sh): counter traffic of the list-scan kernels per launch, from
separate rocprofv3 --pmc passes of profiles/config_rates.py --only c3 (FETCH_SIZE x 2 per
the gfx950 correction of MI355X_MICROARCH.md + WRITE_SIZE; unit checked against
TCC_EA0_RDREQ_sum x 64 B), added to the k = 10 and k = 1000 lines of the rates file
(the scan kernel of each k is a different template instance; the first one dispatched
belongs to k = 10), plus the tiled key GEMM's TFLOP/s from the kernel trace.
Usage: c3_traffic.py <pmc dir with g*/run_counter_collection.csv> <trace csv> <rates jsonl> <out jsonl>"""
import collections
import csv
import glob
import json
import os
import re
import sys


def main(pmc, trace, src, out):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    first = {}
    for f in sorted(glob.glob(os.path.join(pmc, "g*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "k_scan_lists" not in n:
                continue
            n = re.search(r"k_\w+(<[^>]*>)?", n).group(0)
            first.setdefault(n, int(r.get("Dispatch_Id", 0) or 0))
            first[n] = min(first[n], int(r.get("Dispatch_Id", 0) or 0))
            per[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
    names = sorted(per, key=lambda n: first[n])
    traffic = {}
    for n in names:
        m = {c: sum(v) / len(v) for c, v in per[n].items()}
        f, w, rq = m.get("FETCH_SIZE"), m.get("WRITE_SIZE"), m.get("TCC_EA0_RDREQ_sum")
        unit = 1024.0 if not (f and rq) or abs(f * 1024.0 / (rq * 64.0) - 1.0) < 0.25 else 1.0
        traffic[n] = {"traffic": 2.0 * f * unit + w * unit if f is not None and w is not None else None,
                      "FETCH_SIZE": f, "WRITE_SIZE": w, "TCC_EA0_RDREQ_sum": rq, "unit_bytes": unit,
                      "launches": len(per[n].get("FETCH_SIZE", []))}
    gemm = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(trace))
            if "k_coarse_gemm_tiled" in r["Kernel_Name"] and r["Grid_Size_X"] == "131072"]
    lines = [json.loads(l) for l in open(src) if l.strip().startswith("{")]
    with open(out, "w") as o:
        for i, j in enumerate(lines):
            if i < len(names):
                t = traffic[names[i]]
                j["roofline"]["kernel"] = names[i]
                j["roofline"]["traffic"] = t["traffic"]
                j["roofline"]["traffic_source"] = {k: v for k, v in t.items() if k != "traffic"}
            if gemm:
                gemm.sort()
                us = gemm[len(gemm) // 2]
                flop = 2.0 * 1024 * 4096 * 768
                j["coarse_gemm"] = {"kernel": "k_coarse_gemm_tiled (1024 queries x 4096 centroids x 768)",
                                    "median_us": us, "tflops": flop / (us * 1e-6) / 1e12, "peak_tflops": 157.3,
                                    "frac": flop / (us * 1e-6) / 1e12 / 157.3, "launches": len(gemm)}
            o.write(json.dumps(j) + "\n")
            print(json.dumps({"k": j.get("k"), "roofline": j["roofline"], "coarse_gemm": j.get("coarse_gemm")}))


if __name__ == "__main__":
    main(*sys.argv[1:5])
