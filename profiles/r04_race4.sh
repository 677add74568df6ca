#!/bin/bash
# false-sharing experiment: every device buffer at least 64 KB (pad) against the shipped
# library, k = 100 round robin on 2 and 3 streams, 16 rounds each
set -u
O=gpurun_out
export RACE_ROUNDS=16
for v in pad default; do
  if [ $v = default ]; then L=""; else L=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so; fi
  IVFPQ_LIB=$L timeout -k 10 300 python -u profiles/race_diag.py 100,3 100,2 > $O/race4_$v.jsonl 2> $O/race4_$v.log || { echo "$v failed"; tail -20 $O/race4_$v.log; exit 1; }
  echo "== $v"; python -c "
import json
for l in open('$O/race4_$v.jsonl'):
    d=json.loads(l); print(d['k'], d['streams'], sum(r['bad_batches'] for r in d['per_round']), sum(r['err'] for r in d['per_round']))"
done
