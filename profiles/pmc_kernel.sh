#!/bin/bash
# PMC counter groups (one rocprofv3 pass each, no tracing) for kernels matching a regex.
# Usage: pmc_kernel.sh <tag> <kernel-regex> "<group1>" "<group2>" ... -- [bench args]
set -u
TAG=$1; RX=$2; shift 2
GRPS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do GRPS+=("$1"); shift; done
[ $# -gt 0 ] && shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "${GRPS[@]}"; do
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$RX" --output-format csv -d "$OUT/g$i" -o run -- \
    python3 $R/bench.py --no-recall --no-cpu-baseline --steps 6 --warmup 2 "$@" > "$OUT/g$i.json" 2> "$OUT/g$i.err" || exit $?
  i=$((i+1))
done
python3 $R/profiles/summarize_pmc.py "$OUT" | tee "$OUT/summary.txt"
