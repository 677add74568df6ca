#!/bin/bash
# r05 race A/B (profiles/race_variants.py): per variant, the three most sensitive r04/r05
# conditions -- k = 100 with two batches in flight, k = 10 with three, and ordered k = 100
# beside a 512 MB copy loop -- 1000 rounds x 24 batches each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so RACE_ROUNDS=1000 \
    timeout -k 10 120 python -u profiles/race_diag.py 100,2 10,3 > gpurun_out/r05_ab_$v.jsonl 2> gpurun_out/r05_ab_$v.log || exit 1
  IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so RACE_ROUNDS=1000 RACE_INFLIGHT=0 \
    timeout -k 10 120 python -u profiles/race_diag.py 100,1,1 >> gpurun_out/r05_ab_$v.jsonl 2>> gpurun_out/r05_ab_$v.log || exit 2
done
