#!/bin/bash
# shard flow at world 1, preassigned scans on every CU vs 16 CUs left free, alternating, 3 runs each
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06f2
mkdir -p $O
for rep in 1 2 3; do
  for f in 0 16; do
    IVFPQ_SCAN_FREE_CUS=$f timeout -k 10 400 python -u bench.py --shard-at-1 --no-cpu-baseline --no-recall --no-peak --no-extra > $O/shard1_f${f}_$rep.json 2> $O/shard1_f${f}_$rep.err || { echo "shard $f failed"; tail -10 $O/shard1_f${f}_$rep.err; exit 1; }
    tail -1 $O/shard1_f${f}_$rep.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());print('shard free $f', round(j['value']), 'step', round(j['ms_per_step']*1e3,1))"
  done
done
