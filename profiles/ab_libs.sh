#!/bin/bash
# A/B of library builds on the GPU box: GPU tests on the default build (optional subset),
# then one short bench per build (default + lib/var/*), then a kernel trace of the default.
# Usage: bash profiles/ab_libs.sh <tag> [pytest -k expression | all | none]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; SEL=${2:-all}
O=$R/gpurun_out/ab_$TAG; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
if [ "$SEL" != none ]; then
  K=(); [ "$SEL" != all ] && K=(-k "$SEL")
  timeout -k 10 600 python -u -m pytest "$R/tests" -m gpu -x -q --timeout 120 --timeout-method thread "${K[@]}" > "$O/tests.log" 2>&1
  rc=$?; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
fi
B="--steps 30 --warmup 5 --no-cpu-baseline --no-recall --no-extra"
for lib in default $(ls -d "$R"/chameleon-rag-acceleration_amd/lib/var/*/ 2>/dev/null); do
  name=$(basename "$lib")
  if [ "$lib" = default ]; then envs=""; else envs="IVFPQ_LIB=${lib}libivfpq.so"; fi
  env $envs timeout -k 10 300 python "$R/bench.py" $B > "$O/b_$name.json" 2> "$O/b_$name.err" || { echo "bench $name failed"; tail -5 "$O/b_$name.err"; exit 1; }
  python3 -c "import json;j=json.load(open('$O/b_$name.json'));r=j['roofline'];print('$name', round(j['value']), 'qps step', round(j['ms_per_step']*1000,1), 'us scan', round(r['avg_launch_ms']*1000,1), 'us frac', round(r['frac'],3), {k: round(x*1000,1) for k,x in j['stages_ms_per_step'].items()})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python3 "$R/bench.py" $B > "$O/b_traced.json" 2> "$O/b_traced.err" || exit $?
python3 "$R/profiles/summarize_trace.py" "$O/trace/run_kernel_trace.csv" 20 > "$O/kernel_summary.txt" 2>&1; head -12 "$O/kernel_summary.txt"
