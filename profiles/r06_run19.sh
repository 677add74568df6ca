#!/bin/bash
# shard flow at world 1: RCCL channel count (fewer workgroups per collective kernel, so it
# finds room beside the scans) -- default vs NCCL_MAX_NCHANNELS=1 / 2
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06v
mkdir -p $O
for rep in 1 2; do
  for v in default ch1 ch2; do
    case $v in default) envs="";; ch1) envs="NCCL_MAX_NCHANNELS=1";; ch2) envs="NCCL_MAX_NCHANNELS=2";; esac
    env $envs timeout -k 10 400 python -u bench.py --shard-at-1 --no-cpu-baseline --no-recall --no-peak --no-extra > $O/shard1_${v}_$rep.json 2> $O/shard1_${v}_$rep.err || { echo "shard bench $v failed"; tail -10 $O/shard1_${v}_$rep.err; exit 1; }
    tail -1 $O/shard1_${v}_$rep.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());print('$v', round(j['value']), 'step', round(j['ms_per_step']*1e3,1), 'serial', round(j['ms_per_step_serial']*1e3,1), 'repairs', j['repairs'])"
  done
done
