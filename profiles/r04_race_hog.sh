#!/bin/bash
# one stream, no overlap of batches (inflight off), with and without an unrelated copy
# loop on a side stream (profiles/race_diag.py hog = 1), 1000 rounds x 24 k = 10 batches
set -u
O=gpurun_out
RACE_ROUNDS=1000 timeout -k 10 500 python3 -u profiles/race_diag.py 10,1,1 10,1 > $O/race_hog.jsonl 2> $O/race_hog.log || { echo "race diag failed"; tail -20 $O/race_hog.log; exit 1; }
cut -c1-600 $O/race_hog.jsonl
