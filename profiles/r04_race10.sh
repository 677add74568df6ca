#!/bin/bash
# out-of-bounds hypothesis: every device buffer followed by a 64 KB 0xA5 guard (guard
# variant, checked at every error_count; +1e9 per overwritten guard, stderr names the
# buffer), k = 100 and 10 round robin, 12 rounds; the shipped library on the same box
set -u
O=gpurun_out
export RACE_ROUNDS=12
for v in guard default; do
  if [ $v = default ]; then L=""; else L=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so; fi
  IVFPQ_LIB=$L timeout -k 10 400 python -u profiles/race_diag.py 100,3 100,2 10,3 > $O/race10_$v.jsonl 2> $O/race10_$v.log || { echo "$v failed"; tail -20 $O/race10_$v.log; exit 1; }
  echo "== $v"; python -c "
import json
for l in open('$O/race10_$v.jsonl'):
    d=json.loads(l); print(d['k'], d['streams'], sum(r['bad_batches'] for r in d['per_round']), [r['err'] for r in d['per_round'] if r['err']])"
  grep -c guard $O/race10_$v.log || true
  grep guard $O/race10_$v.log | sort | uniq -c | head
done
