#!/bin/bash
# One rocprofv3 kernel-trace pass of the bench (no counters). Usage: trace_only.sh <tag> [bench args]
set -u
TAG=${1:-x}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/trace_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 $R/bench.py --no-recall --no-cpu-baseline --steps 20 --warmup 3 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
python3 $R/profiles/summarize_trace.py "$OUT/run_kernel_trace.csv" 20 > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
exit $rc
