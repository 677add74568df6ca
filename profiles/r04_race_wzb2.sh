#!/bin/bash
# larger sample of the per-stage forcezero bisection (profiles/r04_race_wzb.sh): 3000 rounds
# x 24 batches per stage beside the copy loop, then the bench rate with the merges from the
# forcezero copy
set -u
O=gpurun_out
L=chameleon-rag-acceleration_amd/lib/var/wzb/libivfpq.so
for m in merge none scan; do
  IVFPQ_WZ=$m IVFPQ_LIB=$L RACE_ROUNDS=3000 timeout -k 10 300 python3 -u profiles/race_diag.py 10,1,1 > $O/race_wzb2_$m.jsonl 2> $O/race_wzb2_$m.log || { echo "$m failed"; tail -20 $O/race_wzb2_$m.log; exit 1; }
  echo "== $m: $(cut -c1-120 $O/race_wzb2_$m.jsonl)"
done
for m in merge none; do
  IVFPQ_WZ=$m IVFPQ_LIB=$L timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-recall --no-extra > $O/bench_wzb_$m.json 2> $O/bench_wzb_$m.log || { echo "bench $m failed"; tail -20 $O/bench_wzb_$m.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_wzb_$m.json')); print('bench $m', d['value'], d['ms_per_step'], d['stages_ms_per_step'])"
done
