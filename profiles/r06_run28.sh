#!/bin/bash
# shard flow at world 1: compute streams at normal vs high priority (RCCL normal), alternating, 3 runs each
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06p3
mkdir -p $O
for rep in 1 2 3; do
  for pr in normal high; do
    timeout -k 10 400 python -u bench.py --shard-at-1 --stream-priority $pr --no-cpu-baseline --no-recall --no-peak --no-extra > $O/shard1_${pr}_$rep.json 2> $O/shard1_${pr}_$rep.err || { echo "shard $pr failed"; tail -10 $O/shard1_${pr}_$rep.err; exit 1; }
    tail -1 $O/shard1_${pr}_$rep.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());print('shard $pr', round(j['value']), 'step', round(j['ms_per_step']*1e3,1), 'repairs', j['repairs'])"
  done
done
