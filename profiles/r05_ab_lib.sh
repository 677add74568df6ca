#!/bin/bash
# r05: same-box A/B of the shipped library (new) vs lib/var/<name> builds (AB_VARIANTS, default base):
# quick C2 bench, alternating, twice each; optional parity tests first (AB_TESTS="...")
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -n "${AB_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $AB_TESTS -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_ab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05_ab_tests.log; exit 1; }
  tail -1 gpurun_out/r05_ab_tests.log
fi
for r in 1 2; do
  for v in ${AB_VARIANTS:-new base}; do
    L=""; [ $v != new ] && L=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so
    IVFPQ_LIB=$L timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-recall --mode replicas --steps 100 --warmup 20 > gpurun_out/r05_ab_$v$r.json 2> gpurun_out/r05_ab_$v$r.log || { echo "bench failed"; tail -5 gpurun_out/r05_ab_$v$r.log; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/r05_ab_$v$r.json').read().strip().split(chr(10))[-1]);e=d['extra'];print('$v', round(d['value']/1e6,3), round(d['ms_per_step']*1e3,1), round(d.get('ms_per_step_serial',0)*1e3,1), 'scan', round(d['roofline']['avg_launch_ms']*1e3,1), 'k100', round(e.get('k100_queries_per_s',0)/1e6,3), round(e.get('k100_queries_per_s_serial',0)/1e6,3), 'stages', {kk: round(vv*1e3,1) for kk, vv in d['stages_ms_per_step'].items()})"
  done
done
