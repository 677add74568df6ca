#!/bin/bash
# checksum experiment, second form (chk): error word += 1 per bad position, +100 per partial
# list whose stores read back differently right after the scan wrote them, +1000 per list
# the merge reads differently (+100000 / +10000000: agent / system re-read also differs),
# +10000 per partial list with a hole (an empty entry below its count), +1000000 per count
# mismatch or per list written by no item or by several
set -u
O=gpurun_out
IVFPQ_LIB=chameleon-rag-acceleration_amd/lib/var/chk/libivfpq.so RACE_ROUNDS=16 timeout -k 10 300 python -u profiles/race_diag.py 100,3 100,2 > $O/race7_chk.jsonl 2> $O/race7_chk.log || { echo "chk failed"; tail -20 $O/race7_chk.log; exit 1; }
python -c "
import json
for l in open('$O/race7_chk.jsonl'):
    d=json.loads(l); print(d['k'], d['streams'], [(r['bad_batches'], r['err']) for r in d['per_round'] if r['bad_batches'] or r['err']])"
