#!/bin/bash
# paired centroid loads (coarse GEMM) parity + kernel times; scan grid 2 / 1.75 / 1.5 WGs per CU A/B
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r06l
mkdir -p $O
V=$R/chameleon-rag-acceleration_amd/lib/var
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_add.py tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
B="--steps 40 --warmup 5 --no-cpu-baseline --no-recall --no-extra --no-peak"
for rep in 1 2; do
  for v in default g7 g6; do
    if [ $v = default ]; then envs=""; else envs="IVFPQ_LIB=$V/$v/libivfpq.so"; fi
    env $envs timeout -k 10 300 python bench.py $B > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/ab_${v}_$rep.err; exit 1; }
    tail -1 $O/ab_${v}_$rep.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());r=j['roofline'];print('$v', round(j['value']), 'step', round(j['ms_per_step']*1000,1), 'serial', round(j['ms_per_step_serial']*1000,1), 'scan', round(r['avg_launch_ms']*1000,1), 'frac', round(r['frac'],3), {k: round(x*1000,1) for k,x in j['stages_ms_per_step'].items()})"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_serial -o run -- python3 $R/bench.py --no-recall --no-cpu-baseline --no-extra --no-peak --inflight 1 --steps 30 --warmup 5 > $R/$O/prof_serial.json 2> $R/$O/prof_serial.log || { echo "serial trace failed"; exit 1; }
python3 $R/profiles/summarize_trace.py $R/$O/prof_serial/run_kernel_trace.csv 12 > $R/$O/kernel_summary.txt 2>&1; grep -E "k_coarse|k_scan|k_merge" $R/$O/kernel_summary.txt | head -8
