#!/bin/bash
# r05 race A/B round 2: waits at the record hand-off, perturbations, no permlane swaps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so RACE_ROUNDS=400 \
    timeout -k 10 120 python -u profiles/race_diag.py 100,2 10,3 > gpurun_out/r05_ab2_$v.jsonl 2> gpurun_out/r05_ab2_$v.log || exit 1
done
