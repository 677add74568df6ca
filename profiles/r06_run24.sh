#!/bin/bash
# final shard-flow numbers with two batches in flight (the new default): bench --shard-at-1
# (with the replicas beside it) twice, then the one-GPU emulation
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06final2
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 400 python -u bench.py --shard-at-1 --no-cpu-baseline --no-recall > $O/shard1_$rep.json 2> $O/shard1_$rep.err || { echo "shard bench failed"; tail -10 $O/shard1_$rep.err; exit 1; }
  tail -1 $O/shard1_$rep.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());e=j['extra'];print('shard1', round(j['value']), 'step', round(j['ms_per_step']*1e3,1), 'serial', round(j['ms_per_step_serial']*1e3,1), 'replicas', round(e['replicas']['ms_per_step']*1e3,1), e['shard_vs_replica_rows_identical'], 'repairs', j['repairs'])"
done
timeout -k 10 600 python -u profiles/shard_emulation.py > $O/shard_emulation.jsonl 2> $O/shard_emulation.err || { echo "emulation failed"; tail -10 $O/shard_emulation.err; exit 1; }
grep "^{" $O/shard_emulation.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    j=json.loads(l); print('N', j['N'], {k: round(v,4) for k,v in j['step_wall_ms'].items()})"
