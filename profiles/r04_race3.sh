#!/bin/bash
# stream-order canary: every list-scan workgroup counts its exit; the radix merge that
# follows on the same stream checks the count (a violation adds 1000 to the error word)
set -u
O=gpurun_out
IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/canary/libivfpq.so RACE_ROUNDS=12 timeout -k 10 300 python -u profiles/race_diag.py 100,3 100,2 100,4 > $O/race3_canary.jsonl 2> $O/race3_canary.log || { echo "canary failed"; tail -20 $O/race3_canary.log; exit 1; }
python -c "
import json
for l in open('$O/race3_canary.jsonl'):
    d=json.loads(l); print(d['k'], d['streams'], [(r['bad_batches'], r['sentinels'], r['err']) for r in d['per_round']])"
