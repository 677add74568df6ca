#!/bin/bash
# unconditional (clamped) query-tile loads in the coarse GEMMs: parity, then bench A/B
# against the previous library (lib/var/prev), then a one-at-a-time kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r06o
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_bigshapes.py tests/test_gpu_repair.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
B="--steps 40 --warmup 5 --no-cpu-baseline --no-recall --no-extra --no-peak"
for rep in 1 2; do
  for v in new prev; do
    if [ $v = new ]; then envs=""; else envs="IVFPQ_LIB=$R/chameleon-rag-acceleration_amd/lib/var/prev/libivfpq.so"; fi
    env $envs timeout -k 10 300 python bench.py $B > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/ab_${v}_$rep.err; exit 1; }
  done
done
python3 profiles/ab_table.py "r06o: clamped query-tile loads (new) vs previous library" $O/ab_*.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_serial -o run -- python3 $R/bench.py --no-recall --no-cpu-baseline --no-extra --no-peak --inflight 1 --steps 30 --warmup 5 > $R/$O/prof_serial.json 2> $R/$O/prof_serial.log || { echo "serial trace failed"; exit 1; }
python3 $R/profiles/summarize_trace.py $R/$O/prof_serial/run_kernel_trace.csv 12 > $R/$O/kernel_summary.txt 2>&1; grep -E "k_coarse|k_scan|k_merge" $R/$O/kernel_summary.txt | head -8
