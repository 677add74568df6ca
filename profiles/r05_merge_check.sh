#!/bin/bash
# r05: merge fast-path changes -- parity/config/repair tests, then the shard emulation
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_repair.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_mc_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05_mc_tests.log; exit 1; }
tail -1 gpurun_out/r05_mc_tests.log
timeout -k 10 300 python3 -u profiles/shard_emulation.py > gpurun_out/r05_shard_emulation.jsonl 2> gpurun_out/r05_shard_emulation.log || { echo "emulation failed"; tail -5 gpurun_out/r05_shard_emulation.log; exit 1; }
