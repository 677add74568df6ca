#!/bin/bash
# r05 race A/B round 3: nops after / before the tau_q atomicMin, vs base and notau
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so RACE_ROUNDS=800 \
    timeout -k 10 150 python -u profiles/race_diag.py 10,3 100,2 > gpurun_out/r05_ab3_$v.jsonl 2> gpurun_out/r05_ab3_$v.log || exit 1
done
