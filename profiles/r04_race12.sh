#!/bin/bash
# bisection of the waitcnt effect (r04_race.txt item 7): a full s_waitcnt at one point of the
# k > 64 scan per variant -- w1 before the partial writes, w2 after them, w3 after every
# queue drain; every variant built with -DINFLIGHT_MAXK=1024 (k = 100 batches overlap)
set -u
O=gpurun_out
export RACE_ROUNDS=12
for v in base w1 w2 w3; do
  L=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so
  IVFPQ_LIB=$L timeout -k 10 300 python -u profiles/race_diag.py 100,3 100,2 > $O/race12_$v.jsonl 2> $O/race12_$v.log || { echo "$v failed"; tail -20 $O/race12_$v.log; exit 1; }
  echo "== $v"; python -c "
import json
for l in open('$O/race12_$v.jsonl'):
    d=json.loads(l); print(d['k'], d['streams'], sum(r['bad_batches'] for r in d['per_round']), [r['err'] for r in d['per_round'] if r['err']])"
done
