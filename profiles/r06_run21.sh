#!/bin/bash
# IVFPQ_SCAN_FREE_CUS finer sweep: plain C2 (two in flight) and the shard flow (three in flight)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06x
mkdir -p $O
for rep in 1 2 3; do
  for f in 0 12 16 20 24 32; do
    IVFPQ_SCAN_FREE_CUS=$f timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-recall --no-peak --no-extra > $O/plain_f${f}_$rep.json 2> $O/plain_f${f}_$rep.err || { echo "plain bench $f failed"; tail -10 $O/plain_f${f}_$rep.err; exit 1; }
    tail -1 $O/plain_f${f}_$rep.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());print('plain free $f', round(j['value']), 'step', round(j['ms_per_step']*1e3,1), 'scan', round(j['roofline']['avg_launch_ms']*1e3,1))"
  done
done
for rep in 1 2; do
  for f in 0 4 8 12; do
    IVFPQ_SCAN_FREE_CUS=$f timeout -k 10 400 python -u bench.py --shard-at-1 --no-cpu-baseline --no-recall --no-peak --no-extra > $O/shard1_f${f}_$rep.json 2> $O/shard1_f${f}_$rep.err || { echo "shard bench $f failed"; tail -10 $O/shard1_f${f}_$rep.err; exit 1; }
    tail -1 $O/shard1_f${f}_$rep.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());print('shard free $f', round(j['value']), 'step', round(j['ms_per_step']*1e3,1))"
  done
done
