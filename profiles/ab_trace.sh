#!/bin/bash
# Kernel-trace every variant in lib/var/ (optionally with IVFPQ_DEBUG=$DBG) and print the per-kernel means.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
RX=${RX:-scan_lists|plan_items|merge_probes|coarse}
for d in $R/chameleon-rag-acceleration_amd/lib/var/*/; do
  n=$(basename $d)
  IVFPQ_LIB=$d/libivfpq.so bash $R/profiles/trace_only.sh ab_$n "$@" > /dev/null || exit $?
  echo "== $n"; grep -E "$RX" $R/gpurun_out/trace_ab_$n/summary.txt | grep -v "^  " 
done
