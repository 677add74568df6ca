#!/bin/bash
# r04 second full pass: every gpu test, then C3 rates with the roofline block under a
# kernel trace (coarse-step split), then the default bench line
set -u
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r04c_gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/r04c_gputest.log; exit 1; }
tail -2 $O/r04c_gputest.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r04c_c3prof -o run -- python3 -u profiles/config_rates.py --only c3 --reps 10 > $O/r04c_rates_c3.jsonl 2> $O/r04c_rates_c3.log || { echo "c3 failed"; tail -20 $O/r04c_rates_c3.log; exit 1; }
cat $O/r04c_rates_c3.jsonl
timeout -k 10 400 python -u bench.py > $O/r04c_bench.json 2> $O/r04c_bench.log || { echo "bench failed"; tail -20 $O/r04c_bench.log; exit 1; }
cat $O/r04c_bench.json
