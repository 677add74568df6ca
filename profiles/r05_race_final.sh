#!/bin/bash
# r05 final: the concurrent-kernel stress on the final library -- 4000 rounds x 24 batches per configuration
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RACE_ROUNDS=4000 timeout -k 10 400 python -u profiles/race_diag.py 10,3 100,2 10,2 100,3 > gpurun_out/r05_race_final.jsonl 2> gpurun_out/r05_race_final.log || { echo "failed"; tail -5 gpurun_out/r05_race_final.log; exit 1; }
RACE_ROUNDS=1500 timeout -k 10 300 python -u profiles/race_diag.py 100,1,1 10,1,1 >> gpurun_out/r05_race_final.jsonl 2>> gpurun_out/r05_race_final.log || { echo "failed"; tail -5 gpurun_out/r05_race_final.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r05_race_final.jsonl'):
    d=json.loads(l); print(d['k'], d['streams'], 'hog' if d['hog'] else '', d['rounds']*24, 'batches: bad', d['bad_batches'], 'err', sum(r['err'] for r in d['bad_rounds']), 'stale', d['stale_reads_total'], 'repairs', d['repairs_total'], d['s'], 's')"
