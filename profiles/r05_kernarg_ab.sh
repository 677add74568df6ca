#!/bin/bash
# r05: kernel-argument placement A/B (HIP_FORCE_DEV_KERNARG) on bench.py, one batch at a time and in flight
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in 1 0; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-recall --mode replicas --steps 100 --warmup 20 > gpurun_out/r05_karg$v.json 2> gpurun_out/r05_karg$v.log || { echo "bench $v failed"; tail -5 gpurun_out/r05_karg$v.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r05_karg$v.json').read().strip().split(chr(10))[-1]);print('kernarg_dev=$v', d['value'], d['ms_per_step'], d.get('ms_per_step_serial'), d['roofline']['avg_launch_ms'], d['stages_ms_per_step'], d['extra'].get('k100_queries_per_s'))"
done
