#!/bin/bash
# waitcnt hypothesis: every s_waitcnt forced to zero (wz = -mllvm -amdgpu-waitcnt-forcezero,
# every memory result waited for right after its instruction) against the shipped library,
# same box, k = 100 round robin on 3 and 2 streams, 12 rounds each, twice
set -u
O=gpurun_out
export RACE_ROUNDS=12
for pass in 1 2; do for v in wz default; do
  if [ $v = default ]; then L=""; else L=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so; fi
  IVFPQ_LIB=$L timeout -k 10 400 python -u profiles/race_diag.py 100,3 100,2 > $O/race11_${v}_$pass.jsonl 2> $O/race11_${v}_$pass.log || { echo "$v failed"; tail -20 $O/race11_${v}_$pass.log; exit 1; }
  echo "== $v pass $pass"; python -c "
import json
for l in open('$O/race11_${v}_$pass.jsonl'):
    d=json.loads(l); print(d['k'], d['streams'], sum(r['bad_batches'] for r in d['per_round']), [r['err'] for r in d['per_round'] if r['err']], d['s'])"
done; done
