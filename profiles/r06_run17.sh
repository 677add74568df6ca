#!/bin/bash
# shard flow with one fused collective launch per step (all_to_all of the previous batch +
# all_gather of this one): bench --shard-at-1 (twice, and with per-stream communicators),
# then the one-GPU emulation at N = 1..8 in the same topology
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06t
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 400 python -u bench.py --shard-at-1 --no-cpu-baseline --no-recall --no-peak > $O/shard1_$rep.json 2> $O/shard1_$rep.err || { echo "shard bench failed"; tail -10 $O/shard1_$rep.err; exit 1; }
  tail -1 $O/shard1_$rep.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());e=j['extra'];print('shard1', round(j['value']), 'step', round(j['ms_per_step']*1e3,1), 'serial', round(j['ms_per_step_serial']*1e3,1), 'replicas', round(e['replicas']['ms_per_step']*1e3,1), e['shard_vs_replica_rows_identical'], 'repairs', j['repairs'])"
done
timeout -k 10 400 python -u bench.py --shard-at-1 --comms per-stream --no-cpu-baseline --no-recall --no-peak --no-extra > $O/shard1_per.json 2> $O/shard1_per.err || { echo "shard bench failed"; tail -10 $O/shard1_per.err; exit 1; }
tail -1 $O/shard1_per.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());print('shard1 per-stream', round(j['value']), 'step', round(j['ms_per_step']*1e3,1))"
timeout -k 10 600 python -u profiles/shard_emulation.py > $O/shard_emulation.jsonl 2> $O/shard_emulation.err || { echo "emulation failed"; tail -10 $O/shard_emulation.err; exit 1; }
grep "^{" $O/shard_emulation.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    j=json.loads(l); print('N', j['N'], {k: round(v,4) for k,v in j['step_wall_ms'].items()})"
