#!/bin/bash
# r04 A/B on the GPU box: parity subset on the shipped library and each variant,
# bench.py C2 for all, list-scan phase stamps (profiles/build_variants.sh first:
# pipe = -DSCAN_PIPE=1, nofc = -DFUSED_COARSE=0, notc = -DTILED_COARSE=0, sdiag = -DDIAG_STAMPS).
set -u
O=gpurun_out
V=chameleon-rag-acceleration_amd/lib/var
T="-k golden or sweep or c1_c2 or k100 or round_robin or two_streams or shards_c2 or tiled_coarse"
for v in default pipe nofc; do
  if [ $v = default ]; then L=""; else L=$V/$v/libivfpq.so; fi
  IVFPQ_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider "$T" > $O/ab_test_$v.log 2>&1 || { echo "$v tests failed"; tail -20 $O/ab_test_$v.log; exit 1; }
  tail -1 $O/ab_test_$v.log
  IVFPQ_LIB=$L timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-recall > $O/ab_bench_$v.json 2> $O/ab_bench_$v.log || { echo "bench $v failed"; exit 1; }
done
IVFPQ_LIB=$V/sdiag/libivfpq.so timeout -k 10 300 python -u profiles/diag_stamps.py > $O/ab_stamps_lists.txt 2>&1 || exit 1
# coarse step alone (C3 shape: the tiled key GEMM vs the 16-query tiles), kernel stats per variant
for v in default notc; do
  if [ $v = default ]; then L=""; else L=$V/$v/libivfpq.so; fi
  IVFPQ_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ab_coarse_$v -o run -- python3 -u profiles/coarse_large_nlist.py > $O/ab_coarse_$v.jsonl 2> $O/ab_coarse_$v.log || { echo "coarse $v failed"; exit 1; }
done
