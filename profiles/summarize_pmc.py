"""Average each PMC counter per kernel over the dispatches of a pmc_kernel.sh run."""
import collections
import csv
import glob
import os
import re
import sys


def short(n):
    n = re.sub(r"^void ", "", n).replace("(anonymous namespace)::", "")
    return n.split("(")[0].replace("chivf::", "")


def main(out):
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(out, "g*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(agg.items()):
        print(f"{k:36s} {c:28s} n={len(v):4d} mean={sum(v)/len(v):.6g}")


if __name__ == "__main__":
    main(sys.argv[1])
