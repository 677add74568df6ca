#!/bin/bash
# partial-list checksum experiment (chk = -DPART_CHECK): the scan records (count, hash) of
# every partial list it writes; the radix merge recomputes both from what it reads.
# error word: +1000000 per count mismatch, +1000 per content mismatch (+100000 if an agent-scope
# re-read still differs, +10000000 if a system-scope one does), +1 per bad position,
# +100000000 per bucket pair that is not a probe of its item's list
set -u
O=gpurun_out
IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/chk/libivfpq.so RACE_ROUNDS=16 timeout -k 10 300 python -u profiles/race_diag.py 100,3 100,2 > $O/race5_chk.jsonl 2> $O/race5_chk.log || { echo "chk failed"; tail -20 $O/race5_chk.log; exit 1; }
python -c "
import json
for l in open('$O/race5_chk.jsonl'):
    d=json.loads(l); print(d['k'], d['streams'], [(r['bad_batches'], r['err']) for r in d['per_round'] if r['bad_batches'] or r['err']])"
