#!/bin/bash
# r05: coarse launch with its loads hoisted ahead of the query staging (new) vs base,
# and each half alone (t3only: T3 centroid loads; gonly: the key GEMM's B rows):
# quick C2 bench A/B, then a serial kernel trace of new and base
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R"
AB_VARIANTS="new base t3only gonly" bash profiles/r05_ab_lib.sh || exit 1
cd /tmp && export TMPDIR=/tmp
for v in new base; do
  L=""; [ $v != new ] && L=$R/chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so
  IVFPQ_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05cp_$v -o run -- python3 $R/bench.py --no-recall --no-cpu-baseline --no-extra --inflight 1 --mode replicas --steps 50 --warmup 10 > $R/gpurun_out/r05cp_$v.json 2> $R/gpurun_out/r05cp_$v.log || { echo "trace $v failed"; tail -5 $R/gpurun_out/r05cp_$v.log; exit 1; }
done
echo traced
