#!/bin/bash
# batches in flight 2 / 3 / 4 on the final library (coarse GEMM beside the scan, scan on 16 CUs fewer)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06y
mkdir -p $O
for rep in 1 2; do
  for n in 2 3 4; do
    timeout -k 10 300 python -u bench.py --inflight $n --steps 40 --warmup 5 --no-cpu-baseline --no-recall --no-peak --no-extra > $O/inf${n}_$rep.json 2> $O/inf${n}_$rep.err || { echo "bench $n failed"; tail -10 $O/inf${n}_$rep.err; exit 1; }
    tail -1 $O/inf${n}_$rep.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());print('inflight $n', round(j['value']), 'step', round(j['ms_per_step']*1e3,1), 'scan', round(j['roofline']['avg_launch_ms']*1e3,1), 'repairs', j['repairs'])"
  done
done
