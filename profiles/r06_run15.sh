#!/bin/bash
# register-staged query tile + shuffle-folded norms in the coarse GEMMs (default) vs the
# LDS staging with clamped loads (-DSTAGE_LDS_NORM) vs the previous library: parity, C2 A/B, trace
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r06r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_bigshapes.py tests/test_gpu_add.py tests/test_gpu_transform.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
B="--steps 40 --warmup 5 --no-cpu-baseline --no-recall --no-extra --no-peak"
V=$R/chameleon-rag-acceleration_amd/lib/var
for rep in 1 2 3 4; do
  for v in new prev; do
    if [ $v = new ]; then envs=""; else envs="IVFPQ_LIB=$V/$v/libivfpq.so"; fi
    env $envs timeout -k 10 300 python bench.py $B > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/ab_${v}_$rep.err; exit 1; }
  done
done
python3 profiles/ab_table.py "r06r: query rows loaded ahead of the centroid rows, non-divergent (new) vs previous library" $O/ab_*.json
cd /tmp && export TMPDIR=/tmp
for v in new prev; do
  if [ $v = new ]; then L=$R/chameleon-rag-acceleration_amd/lib/libivfpq.so; else L=$V/$v/libivfpq.so; fi
  IVFPQ_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$v -o run -- python3 $R/bench.py --no-recall --no-cpu-baseline --no-extra --no-peak --inflight 1 --steps 30 --warmup 5 > $R/$O/prof_$v.json 2> $R/$O/prof_$v.log || { echo "trace failed"; exit 1; }
  python3 $R/profiles/summarize_trace.py $R/$O/prof_$v/run_kernel_trace.csv 12 > $R/$O/kernel_summary_$v.txt 2>&1; echo "== $v (one at a time)"; grep -E "k_coarse|k_scan|k_merge" $R/$O/kernel_summary_$v.txt | head -5
done
