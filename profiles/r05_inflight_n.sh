#!/bin/bash
# r05: batches in flight 1, 2, 3 on the C2 bench (quick, replicas)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for n in 2 3 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-recall --mode replicas --steps 120 --warmup 20 --inflight $n --no-extra > gpurun_out/r05_if$n.json 2> gpurun_out/r05_if$n.log || { echo "bench failed"; tail -5 gpurun_out/r05_if$n.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r05_if$n.json').read().strip().split(chr(10))[-1]);print('inflight $n', round(d['value']/1e6,3), round(d['ms_per_step']*1e3,1))"
done
