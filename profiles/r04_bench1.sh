#!/bin/bash
# bench.py with its defaults (one batch at a time on one stream) and the full output
set -u
O=gpurun_out
timeout -k 10 500 python3 -u bench.py > $O/bench1.json 2> $O/bench1.log || { echo "bench failed"; tail -30 $O/bench1.log; exit 1; }
cat $O/bench1.json
