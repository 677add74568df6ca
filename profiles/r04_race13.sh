#!/bin/bash
# write-through partial lists (wt: agent-scope stores, the line is not kept dirty in the
# writer's L2) against the same build with plain stores (base); k = 100 overlapping
set -u
O=gpurun_out
export RACE_ROUNDS=16
for v in base wt base wt; do
  L=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so
  IVFPQ_LIB=$L timeout -k 10 300 python -u profiles/race_diag.py 100,3 100,2 > $O/race13_$v.jsonl 2> $O/race13_$v.log || { echo "$v failed"; tail -20 $O/race13_$v.log; exit 1; }
  echo "== $v"; python -c "
import json
for l in open('$O/race13_$v.jsonl'):
    d=json.loads(l); print(d['k'], d['streams'], sum(r['bad_batches'] for r in d['per_round']), [r['err'] for r in d['per_round'] if r['err']])"
done
