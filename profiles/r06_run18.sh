#!/bin/bash
# k_coarse_gemm<HOIST>: up-front centroid loads for searches whose scan is k_scan_lists (k > 16),
# chunked for k_scan_lean searches.  Parity, then the bench's k = 100 extra and C2 value A/B
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r06u
mkdir -p $O
V=$R/chameleon-rag-acceleration_amd/lib/var
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
B="--steps 40 --warmup 5 --no-cpu-baseline --no-recall --no-peak"
for rep in 1 2 3; do
  for v in new nohoist; do
    if [ $v = new ]; then envs=""; else envs="IVFPQ_LIB=$V/$v/libivfpq.so"; fi
    env $envs timeout -k 10 300 python bench.py $B > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/ab_${v}_$rep.err; exit 1; }
    tail -1 $O/ab_${v}_$rep.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());e=j['extra'];print('$v', round(j['value']), 'step', round(j['ms_per_step']*1e3,1), 'k100', round(e['k100_queries_per_s']), 'k100 serial', round(e['k100_queries_per_s_serial']))"
  done
done
