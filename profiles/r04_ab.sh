#!/bin/bash
# r04 A/B on the GPU box: parity subset on the shipped library and the no-pipe
# variant, bench.py C2 for both, phase stamps for both (build_variants.sh first).
set -u
O=gpurun_out
V=chameleon-rag-acceleration_amd/lib/var
T="-k golden or sweep or c1_c2 or k100 or round_robin or two_streams or shards_c2"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider "$T" > $O/ab_test_pipe.log 2>&1 || { echo "pipe tests failed"; tail -20 $O/ab_test_pipe.log; exit 1; }
IVFPQ_LIB=$V/nopipe/libivfpq.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider "$T" > $O/ab_test_nopipe.log 2>&1 || { echo "nopipe tests failed"; tail -20 $O/ab_test_nopipe.log; exit 1; }
for v in pipe nopipe; do
  if [ $v = pipe ]; then L=""; else L=$V/$v/libivfpq.so; fi
  IVFPQ_LIB=$L timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-recall > $O/ab_bench_$v.json 2> $O/ab_bench_$v.log || { echo "bench $v failed"; exit 1; }
done
IVFPQ_LIB=$V/pdiag/libivfpq.so timeout -k 10 300 python -u profiles/diag_pipe.py > $O/ab_stamps_pipe.txt 2>&1 || exit 1
IVFPQ_LIB=$V/sdiag/libivfpq.so timeout -k 10 300 python -u profiles/diag_stamps.py > $O/ab_stamps_lists.txt 2>&1 || exit 1
tail -1 $O/ab_test_pipe.log; tail -1 $O/ab_test_nopipe.log
