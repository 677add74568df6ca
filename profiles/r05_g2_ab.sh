#!/bin/bash
# r05: k <= 64 scan with 2 pairs per item (IVFPQ_SCAN_G2=1: 32 KB LUT, 3 workgroups per CU) vs 4 (default)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
IVFPQ_SCAN_G2=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_g2_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05_g2_tests.log; exit 1; }
tail -1 gpurun_out/r05_g2_tests.log
for r in 1 2; do
  for v in 1 0; do
    IVFPQ_SCAN_G2=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-recall --mode replicas --steps 100 --warmup 20 > gpurun_out/r05_g2_$v$r.json 2> gpurun_out/r05_g2_$v$r.log || { echo "bench failed"; tail -5 gpurun_out/r05_g2_$v$r.log; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/r05_g2_$v$r.json').read().strip().split(chr(10))[-1]);e=d['extra'];print('g2=$v', round(d['value']/1e6,3), round(d['ms_per_step']*1e3,1), round(d.get('ms_per_step_serial',0)*1e3,1), 'scan', round(d['roofline']['avg_launch_ms']*1e3,1), {kk: round(vv*1e3,1) for kk, vv in d['stages_ms_per_step'].items()})"
  done
done
