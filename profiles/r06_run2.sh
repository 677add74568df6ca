#!/bin/bash
# r06 second GPU pass: gpu suite on the lean-scan library, smoke, A/B of the lean
# scan against the queue-based scan (lib/var/queue), the default bench, and the
# shard flow at world size 1 with real RCCL collectives.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 400 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gputest.log; exit 1; }
tail -3 $O/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
B="--steps 30 --warmup 5 --no-cpu-baseline --no-recall --no-extra --no-peak"
for rep in 1 2; do
  for v in default queue; do
    if [ $v = default ]; then envs=""; else envs="IVFPQ_LIB=$R/chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so"; fi
    env $envs timeout -k 10 300 python bench.py $B > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/ab_${v}_$rep.err; exit 1; }
    python3 -c "import json;j=json.load(open('$O/ab_${v}_$rep.json'));r=j['roofline'];print('$v', round(j['value']), 'step', round(j['ms_per_step']*1000,1), 'serial', round(j['ms_per_step_serial']*1000,1), 'scan', round(r['avg_launch_ms']*1000,1), 'frac', round(r['frac'],3), {k: round(x*1000,1) for k,x in j['stages_ms_per_step'].items()})"
  done
done
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
timeout -k 10 240 python -u bench.py --shard-at-1 --no-cpu-baseline --no-recall > $O/shard1_one.json 2> $O/shard1_one.err || { echo shard1 failed; tail -20 $O/shard1_one.err; exit 1; }
timeout -k 10 240 python -u bench.py --shard-at-1 --comms per-stream --no-cpu-baseline --no-recall > $O/shard1_per.json 2> $O/shard1_per.err || { echo shard1 per failed; tail -20 $O/shard1_per.err; exit 1; }
echo done
