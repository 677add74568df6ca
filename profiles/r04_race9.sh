#!/bin/bash
# latency hypothesis: k = 100 batches on ONE stream (no batch overlap, inflight off) while a
# device-copy loop keeps HBM busy on a side stream, against 3 streams in flight; the shipped
# library, 12 rounds each
set -u
O=gpurun_out
RACE_ROUNDS=12 timeout -k 10 400 python -u profiles/race_diag.py 100,1,1 100,1,0 100,3,0 100,1,1 > $O/race9.jsonl 2> $O/race9.log || { echo "race9 failed"; tail -20 $O/race9.log; exit 1; }
python -c "
import json
for l in open('$O/race9.jsonl'):
    d=json.loads(l); print(d['k'], d['streams'], d['hog'], sum(r['bad_batches'] for r in d['per_round']), [r['err'] for r in d['per_round'] if r['err']])"
