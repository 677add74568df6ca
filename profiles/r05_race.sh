#!/bin/bash
# r05: tagged partial lists -- the repair tests, then the r04 failure conditions
# (ordered searches beside a copy loop; batches in flight) with the stale-entry log.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
  tests/test_gpu_repair.py > gpurun_out/r05_repair_tests.log 2>&1 || exit 1
RACE_ROUNDS=3000 RACE_INFLIGHT=0 timeout -k 10 200 python -u profiles/race_diag.py 10,1,1 100,1,1 \
  > gpurun_out/r05_race_hog.jsonl 2> gpurun_out/r05_race_hog.log || exit 2
RACE_ROUNDS=1000 timeout -k 10 200 python -u profiles/race_diag.py 10,2 10,3 100,2 \
  > gpurun_out/r05_race_inflight.jsonl 2> gpurun_out/r05_race_inflight.log || exit 3
