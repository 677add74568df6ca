#!/bin/bash
# cold vs warm launches of the merge and coarse GEMM (a diagnostic build launches each twice)
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r06j
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
IVFPQ_LIB=$R/chameleon-rag-acceleration_amd/lib/var/twice/libivfpq.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-recall --no-extra --no-peak --inflight 1 > $R/$O/traced.json 2> $R/$O/traced.err || { echo traced failed; tail -5 $R/$O/traced.err; exit 1; }
python3 - $R/$O/trace/run_kernel_trace.csv <<'PY'
import csv, re, sys, statistics
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
def short(n): return re.sub(r"^void ", "", n).replace("(anonymous namespace)::", "").replace("chivf::", "").split("(")[0]
seq = [(short(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000) for r in rows]
for name in ("k_coarse_gemm", "k_merge_probes<1>"):
    first, second = [], []
    for i in range(len(seq) - 1):
        if seq[i][0] == name and seq[i + 1][0] == name:
            first.append(seq[i][1]); second.append(seq[i + 1][1])
    if first:
        print(f"{name}: pairs {len(first)}, first launch mean {statistics.mean(first):.2f} us, second (warm) {statistics.mean(second):.2f} us")
PY
