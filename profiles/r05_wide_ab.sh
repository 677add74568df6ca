#!/bin/bash
# r05: the 8-wave double-buffered scan (IVFPQ_SCAN_WIDE=1) -- parity tests with it on, then A/B vs the
# shipped 4-wave scan on the same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
IVFPQ_SCAN_WIDE=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_repair.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_wide_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r05_wide_tests.log; exit 1; }
tail -1 gpurun_out/r05_wide_tests.log
for r in 1 2; do
  for v in 1 0; do
    IVFPQ_SCAN_WIDE=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-recall --mode replicas --steps 100 --warmup 20 --no-extra > gpurun_out/r05_wide_$v$r.json 2> gpurun_out/r05_wide_$v$r.log || { echo "bench failed"; tail -5 gpurun_out/r05_wide_$v$r.log; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/r05_wide_$v$r.json').read().strip().split(chr(10))[-1]);print('wide=$v', round(d['value']/1e6,3), round(d['ms_per_step']*1e3,1), round(d.get('ms_per_step_serial',0)*1e3,1), 'scan', round(d['roofline']['avg_launch_ms']*1e3,1), d['recall'] if 'recall' in d else '')"
  done
done
