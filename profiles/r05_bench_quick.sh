#!/bin/bash
# r05: quick C2 bench (replicas, no CPU baseline / recall), twice
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-recall --mode replicas --steps 100 --warmup 20 > gpurun_out/r05_q$r.json 2> gpurun_out/r05_q$r.log || { echo "bench failed"; tail -5 gpurun_out/r05_q$r.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r05_q$r.json').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'], d.get('ms_per_step_serial'), d['roofline']['avg_launch_ms'], d['stages_ms_per_step'], d['extra'].get('k100_queries_per_s'), d['extra'].get('k100_queries_per_s_serial'))"
done
