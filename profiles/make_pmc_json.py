"""Per-launch HBM traffic of the scan kernels from separate rocprofv3 --pmc passes
(profiles/pmc_kernel.sh output dir), corrected as MI355X_MICROARCH.md §HBM prescribes:
FETCH_SIZE reports 1/2 of the bytes of wide coalesced reads on gfx950 (doubled here);
WRITE_SIZE is taken as is.  The FETCH_SIZE unit is checked against TCC_EA0_RDREQ_sum x 64 B
rather than assumed.  Usage: make_pmc_json.py <pmc dir> <config_key> <out.json> [libivfpq.so]
The library's sha256 and the kernel sources' sha256 (faiss_amd._lib.kernel_source_sha256)
are recorded: bench.py uses the bytes only for the same kernel build."""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(n):
    n = re.sub(r"^void ", "", n).replace("(anonymous namespace)::", "")
    return n.split("(")[0].replace("chivf::", "")


def main(d, key, out, lib=None):
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "g*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    mean = {kc: sum(v) / len(v) for kc, v in agg.items()}
    kernels = sorted({k for k, _ in mean})
    res = {"config_key": key, "source": os.path.relpath(d), "kernels": {}}
    if lib:
        import hashlib

        res["lib_sha256"] = hashlib.sha256(open(lib, "rb").read()).hexdigest()
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "chameleon-rag-acceleration_amd"))
    from faiss_amd import _lib

    res["kernel_src_sha256"] = _lib.kernel_source_sha256()
    for k in kernels:
        f = mean.get((k, "FETCH_SIZE"))
        w = mean.get((k, "WRITE_SIZE"))
        rq = mean.get((k, "TCC_EA0_RDREQ_sum"))
        wq = mean.get((k, "TCC_EA0_WRREQ_sum"))
        unit = 1024.0  # rocprofv3 derived FETCH_SIZE / WRITE_SIZE are in KiB ...
        if f and rq:   # ... unless the raw request count says otherwise
            unit = 1024.0 if abs(f * 1024.0 / (rq * 64.0) - 1.0) < 0.25 else 1.0
        ent = {"FETCH_SIZE": f, "WRITE_SIZE": w, "TCC_EA0_RDREQ_sum": rq, "TCC_EA0_WRREQ_sum": wq,
               "unit_bytes": unit}
        if f is not None and w is not None:
            ent["hbm_bytes_per_launch"] = 2.0 * f * unit + w * unit
        res["kernels"][k] = ent
    # the bench's own scan kernel: of the list-scan instantiations, the most launched
    # (the bench's k = 100 extra runs another one a few times)
    nlaunch = {k: len(agg.get((k, "FETCH_SIZE"), [])) for k in kernels}
    lists = sorted((k for k in kernels if k.startswith(("k_scan_lean", "k_scan_pipe", "k_scan_lists"))), key=lambda k: -nlaunch[k])
    topk = [k for k in kernels if k.startswith("k_scan_topk") and "true" not in k]
    main_k = (lists or topk or [None])[0]
    res["kernel"] = main_k
    res["hbm_bytes_per_launch"] = res["kernels"].get(main_k, {}).get("hbm_bytes_per_launch")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
