#!/bin/bash
# coarse GEMM register footprint vs the scan's: paired up-front B loads (default, 148 + 16 AGPR)
# vs chunked B loads (np: 74 + 16) vs chunked with waves_per_eu 5 (npw5: 74 + 0), C2 A/B
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r06s
mkdir -p $O
V=$R/chameleon-rag-acceleration_amd/lib/var
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
IVFPQ_LIB=$V/np/libivfpq.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/gputest_np.log 2>&1 || { echo "np gpu tests failed rc=$?"; tail -30 $O/gputest_np.log; exit 1; }
tail -1 $O/gputest_np.log
B="--steps 40 --warmup 5 --no-cpu-baseline --no-recall --no-extra --no-peak"
for rep in 1 2 3; do
  for v in new np npw5; do
    if [ $v = new ]; then envs=""; else envs="IVFPQ_LIB=$V/$v/libivfpq.so"; fi
    env $envs timeout -k 10 300 python bench.py $B > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/ab_${v}_$rep.err; exit 1; }
  done
done
python3 profiles/ab_table.py "r06s: coarse GEMM paired up-front B loads (new) vs chunked B loads (np) vs chunked + waves_per_eu 5 (npw5)" $O/ab_*.json
cd /tmp && export TMPDIR=/tmp
for v in new np; do
  if [ $v = new ]; then L=$R/chameleon-rag-acceleration_amd/lib/libivfpq.so; else L=$V/$v/libivfpq.so; fi
  IVFPQ_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --no-recall --no-cpu-baseline --no-extra --no-peak --steps 30 --warmup 5 > $R/$O/prof_$v.json 2> $R/$O/prof_$v.log || { echo "trace failed"; exit 1; }
  python3 $R/profiles/summarize_trace.py $R/$O/prof_$v/run_kernel_trace.csv 12 > $R/$O/kernel_summary_$v.txt 2>&1; echo "== $v (two in flight)"; grep -E "k_coarse|k_scan|k_merge" $R/$O/kernel_summary_$v.txt | head -5
done
