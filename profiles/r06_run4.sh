#!/bin/bash
# r06 fourth GPU pass: parity of the lean scan (JB 6, no prefetch), its phase stamps,
# batches in flight 2 / 3 / 4 on the plain path, and a kernel trace of the bench.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_repair.py tests/test_gpu_ip.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
IVFPQ_LIB=$R/chameleon-rag-acceleration_amd/lib/var/diag/libivfpq.so timeout -k 10 300 python -u profiles/diag_stamps.py > $O/stamps.txt 2>&1 || { echo stamps failed; tail -20 $O/stamps.txt; exit 1; }
cat $O/stamps.txt
B="--steps 40 --warmup 5 --no-cpu-baseline --no-recall --no-extra --no-peak"
for rep in 1 2; do
  for inf in 2 3 4; do
    timeout -k 10 300 python bench.py $B --inflight $inf > $O/inf${inf}_$rep.json 2> $O/inf${inf}_$rep.err || { echo "bench failed"; tail -5 $O/inf${inf}_$rep.err; exit 1; }
    tail -1 $O/inf${inf}_$rep.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());r=j['roofline'];print('inflight $inf', round(j['value']), 'step', round(j['ms_per_step']*1000,1), 'serial', round(j['ms_per_step_serial']*1000,1), 'scan', round(r['avg_launch_ms']*1000,1), 'frac', round(r['frac'],3))"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-recall --no-extra --no-peak --inflight 1 > $R/$O/traced.json 2> $R/$O/traced.err || { echo traced failed; tail -5 $R/$O/traced.err; exit 1; }
python3 $R/profiles/summarize_trace.py $R/$O/trace/run_kernel_trace.csv 20 > $R/$O/kernel_summary.txt 2>&1; head -40 $R/$O/kernel_summary.txt
echo done
