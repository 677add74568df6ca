#!/bin/bash
# hardware queues per process: HIP's default 4 vs 8 (every stream of the shard flow -- null,
# index, three compute, RCCL's -- on its own queue), shard flow at world 1 and plain C2, alternating
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06q2
mkdir -p $O
for rep in 1 2 3; do
  for qn in 4 8; do
    GPU_MAX_HW_QUEUES=$qn timeout -k 10 400 python -u bench.py --shard-at-1 --no-cpu-baseline --no-recall --no-peak --no-extra > $O/shard1_q${qn}_$rep.json 2> $O/shard1_q${qn}_$rep.err || { echo "shard q$qn failed"; tail -10 $O/shard1_q${qn}_$rep.err; exit 1; }
    tail -1 $O/shard1_q${qn}_$rep.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());print('shard queues $qn', round(j['value']), 'step', round(j['ms_per_step']*1e3,1), 'repairs', j['repairs'])"
  done
done
for rep in 1 2; do
  for qn in 4 8; do
    GPU_MAX_HW_QUEUES=$qn timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-recall --no-peak --no-extra > $O/plain_q${qn}_$rep.json 2> $O/plain_q${qn}_$rep.err || { echo "plain q$qn failed"; tail -10 $O/plain_q${qn}_$rep.err; exit 1; }
    tail -1 $O/plain_q${qn}_$rep.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());print('plain queues $qn', round(j['value']), 'step', round(j['ms_per_step']*1e3,1))"
  done
done
