#!/bin/bash
# r05: LDS-aggregated planning for large shard batches (k_plan_count_agg) -- tests, then the
# shard emulation with it on (default) and off (IVFPQ_PLAN_AGG=0), same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_bigshapes.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_agg_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05_agg_tests.log; exit 1; }
tail -1 gpurun_out/r05_agg_tests.log
for v in 1 0; do
  IVFPQ_PLAN_AGG=$v timeout -k 10 300 python3 -u profiles/shard_emulation.py > gpurun_out/r05_agg_emu$v.jsonl 2> gpurun_out/r05_agg_emu$v.log || { echo "emulation failed"; tail -5 gpurun_out/r05_agg_emu$v.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r05_agg_emu$v.jsonl'):
    d=json.loads(l); print('agg=$v', d['N'], {k:round(v,4) for k,v in d['step_wall_ms'].items()}, {k:round(v*1e3,1) for k,v in d['preassigned_stages_ms'].items()})"
done
