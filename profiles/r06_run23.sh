#!/bin/bash
# shard flow at world 1: batches in flight 2 / 3 / 4 on the final library
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06z
mkdir -p $O
for rep in 1 2; do
  for n in 2 3 4; do
    timeout -k 10 400 python -u bench.py --shard-at-1 --inflight $n --no-cpu-baseline --no-recall --no-peak --no-extra > $O/shard_inf${n}_$rep.json 2> $O/shard_inf${n}_$rep.err || { echo "shard $n failed"; tail -10 $O/shard_inf${n}_$rep.err; exit 1; }
    tail -1 $O/shard_inf${n}_$rep.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());print('shard inflight $n', round(j['value']), 'step', round(j['ms_per_step']*1e3,1), 'repairs', j['repairs'])"
  done
done
