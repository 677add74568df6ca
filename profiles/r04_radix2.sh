#!/bin/bash
# k_merge_radix with the 16-bit early exit and the register sort: parity (k sweep, ties,
# C2 k = 100, padding) and the C2 k = 10 / 100 rates under a kernel trace
set -u
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "sweep or ties or k100 or padding or golden or round_robin or c3_shape" > $O/radix2_test.log 2>&1 || { echo "tests failed"; tail -30 $O/radix2_test.log; exit 1; }
tail -1 $O/radix2_test.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/radix2_prof -o run -- python3 -u profiles/config_rates.py --only c2 --reps 10 > $O/radix2_rates.jsonl 2> $O/radix2_rates.log || { echo "rates failed"; exit 1; }
cat $O/radix2_rates.jsonl
