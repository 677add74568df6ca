#!/bin/bash
# batches in flight with the scans ordered (INFLIGHT_SCAN_ORDER=1: only a batch's coarse
# step overlaps the search in flight): k = 10 mismatch rate at 2 / 3 / 5 streams x 1000
# rounds, then bench.py with two in flight
set -u
O=gpurun_out
RACE_ROUNDS=1000 timeout -k 10 400 python3 -u profiles/race_diag.py 10,2 10,3 10,5,2 > $O/race_order.jsonl 2> $O/race_order.log || { echo "race diag failed"; tail -20 $O/race_order.log; exit 1; }
cut -c1-400 $O/race_order.jsonl
timeout -k 10 400 python3 -u bench.py --inflight 2 --no-cpu-baseline --no-recall > $O/bench_order2.json 2> $O/bench_order2.log || { echo "bench failed"; tail -20 $O/bench_order2.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_order2.json')); print(d['value'], d['ms_per_step'], d['ms_per_step_serial'])"
