#!/bin/bash
# r04 full GPU pass: every gpu test, the batches-in-flight validation, the default
# bench line (with the CPU baseline) and the coarse step alone under rocprofv3.
set -u
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r04b_gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/r04b_gputest.log; exit 1; }
tail -2 $O/r04b_gputest.log
timeout -k 10 400 python -u profiles/inflight_validate.py > $O/r04_inflight_validate.json 2> $O/r04_inflight_validate.log || { echo "inflight validate failed"; tail -20 $O/r04_inflight_validate.log; exit 1; }
cat $O/r04_inflight_validate.json
timeout -k 10 400 python -u bench.py > $O/r04b_bench.json 2> $O/r04b_bench.log || { echo "bench failed"; tail -20 $O/r04b_bench.log; exit 1; }
cat $O/r04b_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r04b_coarse -o run -- python3 -u profiles/coarse_large_nlist.py > $O/r04b_coarse.jsonl 2> $O/r04b_coarse.log || { echo "coarse failed"; exit 1; }
cat $O/r04b_coarse.jsonl
