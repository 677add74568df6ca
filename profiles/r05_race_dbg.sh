#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/dbg/libivfpq.so RACE_ROUNDS=300 \
  timeout -k 10 120 python -u profiles/race_diag.py 100,2 > gpurun_out/r05_dbg.jsonl 2> gpurun_out/r05_dbg.log || exit 1
IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/dbg/libivfpq.so RACE_ROUNDS=1000 RACE_INFLIGHT=0 \
  timeout -k 10 120 python -u profiles/race_diag.py 100,1,1 >> gpurun_out/r05_dbg.jsonl 2>> gpurun_out/r05_dbg.log || exit 2
