#!/bin/bash
# k = 10 batches in flight on 2..5 round-robin streams (profiles/race_diag.py), 20 rounds
# each, after the round-robin test's one-row mismatch at k = 10 / 5 streams; then the
# k_merge_radix parity subset and C2 rates (profiles/r04_radix2.sh)
set -u
O=gpurun_out
RACE_ROUNDS=20 timeout -k 10 400 python3 -u profiles/race_diag.py 10,2 10,3 10,4 10,5 100,5 > $O/race_k10.jsonl 2> $O/race_k10.log || { echo "race diag failed"; tail -20 $O/race_k10.log; exit 1; }
cat $O/race_k10.jsonl
bash profiles/r04_radix2.sh
