#!/bin/bash
# k = 10 batches in flight with the round-robin test's coarse_device + preassigned mix
# (profiles/race_diag.py hog = 2), 150 rounds per stream count
set -u
O=gpurun_out
RACE_ROUNDS=150 timeout -k 10 500 python3 -u profiles/race_diag.py 10,5,2 10,4,2 10,3,2 10,2,2 10,5 > $O/race_mix.jsonl 2> $O/race_mix.log || { echo "race diag failed"; tail -20 $O/race_mix.log; exit 1; }
cat $O/race_mix.jsonl
