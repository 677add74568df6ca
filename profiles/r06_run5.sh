#!/bin/bash
# r06 fifth GPU pass: parity of the lean scan (cheaper insertion) with and without the
# T3 prefetch, phase stamps of both, bench A/B against the queue-based scan.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r06f
mkdir -p $O
V=$R/chameleon-rag-acceleration_amd/lib/var
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_repair.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
IVFPQ_LIB=$V/pf/libivfpq.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_repair.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/gputest_pf.log 2>&1 || { echo "gpu tests (pf) failed rc=$?"; tail -30 $O/gputest_pf.log; exit 1; }
tail -1 $O/gputest_pf.log
for v in diag diagpf; do
  IVFPQ_LIB=$V/$v/libivfpq.so timeout -k 10 300 python -u profiles/diag_stamps.py > $O/stamps_$v.txt 2>&1 || { echo stamps failed; tail -20 $O/stamps_$v.txt; exit 1; }
  echo "== $v"; sed -n 7,12p $O/stamps_$v.txt
done
B="--steps 40 --warmup 5 --no-cpu-baseline --no-recall --no-extra --no-peak"
for rep in 1 2; do
  for v in default pf queue; do
    if [ $v = default ]; then envs=""; else envs="IVFPQ_LIB=$V/$v/libivfpq.so"; fi
    env $envs timeout -k 10 300 python bench.py $B > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/ab_${v}_$rep.err; exit 1; }
    tail -1 $O/ab_${v}_$rep.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());r=j['roofline'];print('$v', round(j['value']), 'step', round(j['ms_per_step']*1000,1), 'serial', round(j['ms_per_step_serial']*1000,1), 'scan', round(r['avg_launch_ms']*1000,1), 'frac', round(r['frac'],3))"
  done
done
echo done
