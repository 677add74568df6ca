#!/bin/bash
# instruction-cache counters of the C2 kernels (the coarse kernels' fill phases take
# 12-20k cycles, far above a load round trip: profiles/coldload.hip)
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r06i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="--steps 10 --warmup 3 --no-cpu-baseline --no-recall --no-extra --no-peak --inflight 1"
i=0
for grp in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES SQ_IFETCH" "SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_coarse|k_scan|k_merge" --output-format csv -d $R/$O/g$i -o run -- python3 $R/bench.py $B > $R/$O/g$i.json 2> $R/$O/g$i.err || { echo "pass $i failed"; tail -5 $R/$O/g$i.err; exit 1; }
  i=$((i+1))
done
python3 $R/profiles/summarize_pmc.py $R/$O | tee $R/$O/summary.txt
