#!/bin/bash
# batches-in-flight mismatch hunt: profiles/race_diag.py on the shipped library and on
# the k_merge_big variant (noradix), 8 rounds of 24 batches per configuration
set -u
O=gpurun_out
timeout -k 10 300 python -u profiles/race_diag.py > $O/race_default.jsonl 2> $O/race_default.log || { echo "default failed"; tail -20 $O/race_default.log; exit 1; }
cat $O/race_default.jsonl
IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/noradix/libivfpq.so timeout -k 10 300 python -u profiles/race_diag.py > $O/race_noradix.jsonl 2> $O/race_noradix.log || { echo "noradix failed"; tail -20 $O/race_noradix.log; exit 1; }
cat $O/race_noradix.jsonl
