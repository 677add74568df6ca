#!/bin/bash
# SQ instruction-mix / wait counters for one kernel (regex $RX, default the list scan), one
# rocprofv3 --pmc pass per group (never combined with tracing).  Usage: sq_counters.sh <tag>
set -u
TAG=${1:-sq}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
RX=${RX:-k_scan_lists}
OUT=$R/gpurun_out/sq_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_IFETCH" \
           ${EXTRA_GROUP:+"$EXTRA_GROUP"}; do
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "$RX" --output-format csv -d "$OUT/g$i" -o run -- \
    python3 $R/bench.py --no-recall --no-cpu-baseline --steps 4 --warmup 1 "$@" > "$OUT/g$i.log" 2>&1 || { echo "pass $i failed"; tail -3 "$OUT/g$i.log"; }
  i=$((i+1))
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/g*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("chivf::", "")
        acc[(kn[:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k[0]:40s} {k[1]:28s} n={len(v):3d} mean={sum(v)/len(v):14.1f}")
PY
