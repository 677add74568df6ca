#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box via gpurun).
# Pass 1: kernel trace + stats; passes 2-4: one PMC group each (never combined with tracing).
# Usage: bash profiles/run_profiles.sh <tag> [extra bench args]
set -u
TAG=${1:-r01}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --no-recall --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 $BENCH --steps 40 --warmup 5 > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err" || exit $?
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  name=$(echo "$grp" | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "k_scan|k_l2_dist|k_select|k_ip_table" \
    --output-format csv -d "$OUT/pmc_$name" -o run -- python3 $BENCH --steps 10 --warmup 2 \
    > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || exit $?
done
echo "profiles done: $OUT"
