#!/bin/bash
# r05: cost of the cross-workgroup bound (tau_q): C2 bench with the shipped-source build vs
# the notau variant (profiles/race_variants.py), same box, alternating twice
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in base notau; do
    IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so timeout -k 10 240 python -u bench.py --steps 200 --warmup 20 \
      --no-cpu-baseline --no-recall --mode replicas > gpurun_out/r05_notau_$v$rep.json 2> gpurun_out/r05_notau_$v$rep.log || exit 1
  done
done
