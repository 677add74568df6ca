#!/bin/bash
# forcezero build (every memory result waited for at once, lib/var/wz) under the
# conditions that fail with the shipped build: one stream + an unrelated copy loop on a
# side stream, and two streams in flight, 1000 rounds x 24 k = 10 batches each; then the
# bench rate of that build (one at a time)
set -u
O=gpurun_out
L=chameleon-rag-acceleration_amd/lib/var/wz/libivfpq.so
IVFPQ_LIB=$L RACE_ROUNDS=1000 timeout -k 10 500 python3 -u profiles/race_diag.py 10,1,1 10,2 > $O/race_wz.jsonl 2> $O/race_wz.log || { echo "race diag failed"; tail -20 $O/race_wz.log; exit 1; }
cut -c1-300 $O/race_wz.jsonl
IVFPQ_LIB=$L timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --no-recall --no-extra > $O/bench_wz.json 2> $O/bench_wz.log || { echo "bench failed"; tail -20 $O/bench_wz.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_wz.json')); print('wz bench', d['value'], d['ms_per_step'], d['stages_ms_per_step'])"
