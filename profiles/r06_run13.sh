#!/bin/bash
# r06 load-issue fixes (coarse query tiles, tiled-GEMM norms, k_merge_big, LUT-build
# fence in k_scan_lists): parity first, then C2 bench A/B and C3 rates A/B against the
# previous library (lib/var/prev), then a one-at-a-time C2 kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_repair.py tests/test_gpu_fullsize.py tests/test_gpu_bigshapes.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
B="--steps 40 --warmup 5 --no-cpu-baseline --no-recall --no-extra --no-peak"
P=$R/chameleon-rag-acceleration_amd/lib/var/prev/libivfpq.so
for rep in 1 2; do
  for v in new prev; do
    if [ $v = new ]; then envs=""; else envs="IVFPQ_LIB=$P"; fi
    env $envs timeout -k 10 300 python bench.py $B > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/ab_${v}_$rep.err; exit 1; }
  done
done
python3 profiles/ab_table.py "r06p: r06 load-issue fixes (new) vs previous library" $O/ab_*.json
for v in new prev; do
  if [ $v = new ]; then envs=""; else envs="IVFPQ_LIB=$P"; fi
  env $envs timeout -k 10 400 python -u profiles/config_rates.py --only c3 > $O/c3_$v.jsonl 2> $O/c3_$v.err || { echo "c3 $v failed"; tail -5 $O/c3_$v.err; exit 1; }
  python3 -c "
import json
for l in open('$O/c3_$v.jsonl'):
    j=json.loads(l); r=j['roofline']; print('$v', 'k', j['k'], 'ms', round(j['ms_per_batch'],4), 'inflight2', round(j.get('ms_per_batch_inflight2',0),4), 'scan us', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],3), {k: round(x*1e3,1) for k,x in j['stages_ms'].items()})"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_serial -o run -- python3 $R/bench.py --no-recall --no-cpu-baseline --no-extra --no-peak --inflight 1 --steps 30 --warmup 5 > $R/$O/prof_serial.json 2> $R/$O/prof_serial.log || { echo "serial trace failed"; exit 1; }
python3 $R/profiles/summarize_trace.py $R/$O/prof_serial/run_kernel_trace.csv 12 > $R/$O/kernel_summary.txt 2>&1; grep -E "k_coarse|k_scan|k_merge" $R/$O/kernel_summary.txt | head -8
