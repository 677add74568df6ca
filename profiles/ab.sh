#!/bin/bash
# A/B of scan variants on the GPU box: GPU tests, then one short bench per variant
# (env assignments per variant), then a kernel trace of the default.  Usage: bash profiles/ab.sh <tag> [VAR=val,... ...]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
O=$R/gpurun_out/ab_$TAG; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest "$R/tests" -m gpu -x -q --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; tail -2 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
for v in default "$@"; do
  envs=""; [ "$v" != default ] && envs=$(echo "$v" | tr ',' ' ')
  env $envs timeout -k 10 300 python "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-recall > "$O/b_$v.json" 2> "$O/b_$v.err" || exit $?
  python3 -c "import json;j=json.load(open('$O/b_$v.json'));print('$v', round(j['value']), 'qps', {k: round(x*1000,1) for k,x in j['stages_ms_per_step'].items()}, 'us')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-recall > "$O/b_traced.json" 2> "$O/b_traced.err" || exit $?
python3 "$R/profiles/summarize_trace.py" "$O/trace/run_kernel_trace.csv" 20 > "$O/kernel_summary.txt" 2>&1; head -16 "$O/kernel_summary.txt"
