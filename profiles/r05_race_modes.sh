#!/bin/bash
# r05: which stage fails under overlap -- coarse only, preassigned (plan + scan + merge) only,
# and the full search -- then the bound-sharing A/B (notau, nowb)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/base/libivfpq.so RACE_ROUNDS=400 \
  timeout -k 10 150 python -u profiles/race_diag.py 10,3,3 10,3,4 100,2,4 10,3 100,2 > gpurun_out/r05_modes.jsonl 2> gpurun_out/r05_modes.log || exit 1
bash profiles/r05_race_ab2.sh notau nowb
