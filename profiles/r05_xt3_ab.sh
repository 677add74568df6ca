#!/bin/bash
# r05: in-scan T3 (ScanArgs::xt3) -- parity tests, then bench.py with it on (default) and off (IVFPQ_XT3=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_repair.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_xt3_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05_xt3_tests.log; exit 1; }
tail -1 gpurun_out/r05_xt3_tests.log
for v in 1 0; do
  IVFPQ_XT3=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-recall --mode replicas --steps 100 --warmup 20 > gpurun_out/r05_xt3_bench$v.json 2> gpurun_out/r05_xt3_bench$v.log || { echo "bench $v failed"; tail -5 gpurun_out/r05_xt3_bench$v.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r05_xt3_bench$v.json').read().strip().split(chr(10))[-1]);print('xt3=$v', d['value'], d['ms_per_step'], d.get('ms_per_step_serial'), d['roofline']['avg_launch_ms'], d['stages_ms_per_step'], d['extra'].get('k100_queries_per_s'))"
done
