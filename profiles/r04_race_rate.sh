#!/bin/bash
# mismatch rate of k = 10 batches in flight by stream count (profiles/race_diag.py):
# 2 and 3 streams x 1000 rounds (24000 batches each), and 3 streams ordered
# (inflight off) x 500 rounds as the control
set -u
O=gpurun_out
RACE_ROUNDS=1000 timeout -k 10 300 python3 -u profiles/race_diag.py 10,2 10,3 > $O/race_rate.jsonl 2> $O/race_rate.log || { echo "race diag failed"; tail -20 $O/race_rate.log; exit 1; }
RACE_INFLIGHT=0 RACE_ROUNDS=500 timeout -k 10 300 python3 -u profiles/race_diag.py 10,3 10,5 >> $O/race_rate.jsonl 2>> $O/race_rate.log || { echo "race diag (ordered) failed"; tail -20 $O/race_rate.log; exit 1; }
cut -c1-600 $O/race_rate.jsonl
