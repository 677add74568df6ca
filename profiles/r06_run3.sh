#!/bin/bash
# r06 third GPU pass: parity of the prefetching lean scan, A/B against its variants,
# and the world-1 shard flow with coalesced RCCL collectives (2 and 3 in flight),
# plus a kernel trace of the shard flow.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_repair.py tests/test_gpu_ip.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
B="--steps 30 --warmup 5 --no-cpu-baseline --no-recall --no-extra --no-peak"
for rep in 1 2; do
  for v in default nopf nopf6 queue; do
    if [ $v = default ]; then envs=""; else envs="IVFPQ_LIB=$R/chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so"; fi
    env $envs timeout -k 10 300 python bench.py $B > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/ab_${v}_$rep.err; exit 1; }
    tail -1 $O/ab_${v}_$rep.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());r=j['roofline'];print('$v', round(j['value']), 'step', round(j['ms_per_step']*1000,1), 'serial', round(j['ms_per_step_serial']*1000,1), 'scan', round(r['avg_launch_ms']*1000,1), 'frac', round(r['frac'],3), {k: round(x*1000,1) for k,x in j['stages_ms_per_step'].items()})"
  done
done
for inf in 2 3; do
  timeout -k 10 240 python -u bench.py --shard-at-1 --inflight $inf --no-cpu-baseline --no-recall > $O/shard1_inf$inf.json 2> $O/shard1_inf$inf.err || { echo shard1 failed; tail -20 $O/shard1_inf$inf.err; exit 1; }
  tail -1 $O/shard1_inf$inf.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());print('shard1 inflight $inf', round(j['value']), 'step', round(j['ms_per_step']*1000,1), 'serial', round(j['ms_per_step_serial']*1000,1), j['extra'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- python3 $R/bench.py --shard-at-1 --steps 20 --warmup 5 --no-cpu-baseline --no-recall --no-extra --no-peak > $R/$O/shard_traced.json 2> $R/$O/shard_traced.err || { echo traced failed; tail -5 $R/$O/shard_traced.err; exit 1; }
python3 $R/profiles/summarize_trace.py $R/$O/trace/run_kernel_trace.csv 25 > $R/$O/shard_kernel_summary.txt 2>&1; head -30 $R/$O/shard_kernel_summary.txt
echo done
