#!/bin/bash
# r05: same-box A/B of T3 built on a side stream beside the coarse step
# (IVFPQ_SIDE_T3=1) vs inside the coarse key launch (0): parity tests with it on,
# then the quick C2 bench alternating, twice each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
IVFPQ_SIDE_T3=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_side_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05_side_tests.log; exit 1; }
tail -1 gpurun_out/r05_side_tests.log
for r in 1 2; do
  for v in 0 1; do
    IVFPQ_SIDE_T3=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-recall --mode replicas --steps 100 --warmup 20 > gpurun_out/r05_side_$v$r.json 2> gpurun_out/r05_side_$v$r.log || { echo "bench failed"; tail -5 gpurun_out/r05_side_$v$r.log; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/r05_side_$v$r.json').read().strip().split(chr(10))[-1]);e=d['extra'];print('side$v', round(d['value']/1e6,3), round(d['ms_per_step']*1e3,1), round(d.get('ms_per_step_serial',0)*1e3,1), 'scan', round(d['roofline']['avg_launch_ms']*1e3,1), 'k100', round(e.get('k100_queries_per_s',0)/1e6,3), round(e.get('k100_queries_per_s_serial',0)/1e6,3), 'stages', {kk: round(vv*1e3,1) for kk, vv in d['stages_ms_per_step'].items()})"
  done
done
