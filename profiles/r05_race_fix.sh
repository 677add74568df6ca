#!/bin/bash
# r05: the wave-uniform bound fix (tau_get / s_wb readfirstlane) under the failing
# configurations -- shipped build, then the two perturbations that failed most before it
# (noswap: 321 bad k=10 batches in 19200; nowb: 86 bad, 963 index errors)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RACE_ROUNDS=800 timeout -k 10 200 python -u profiles/race_diag.py 10,3 100,2 100,3 10,2 > gpurun_out/r05_fix_shipped.jsonl 2> gpurun_out/r05_fix_shipped.log || exit 1
RACE_ROUNDS=300 timeout -k 10 200 python -u profiles/race_diag.py 100,1,1 10,1,1 > gpurun_out/r05_fix_hog.jsonl 2>> gpurun_out/r05_fix_shipped.log || exit 1
for v in noswap nowb; do
  IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so RACE_ROUNDS=800 \
    timeout -k 10 200 python -u profiles/race_diag.py 10,3 100,2 > gpurun_out/r05_fix_$v.jsonl 2> gpurun_out/r05_fix_$v.log || exit 1
done
