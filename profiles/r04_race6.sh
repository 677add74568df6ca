#!/bin/bash
# partial lists padded to whole 128-B lines for k > 64 (default) against the unpadded
# layout (nopad), and the padded layout with the checksum checks (chk); k = 100 round
# robin on 3 and 2 streams, 16 rounds each; then the round-robin parity test
set -u
O=gpurun_out
export RACE_ROUNDS=16
for v in default chk nopad; do
  if [ $v = default ]; then L=""; else L=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so; fi
  IVFPQ_LIB=$L timeout -k 10 300 python -u profiles/race_diag.py 100,3 100,2 > $O/race6_$v.jsonl 2> $O/race6_$v.log || { echo "$v failed"; tail -20 $O/race6_$v.log; exit 1; }
  echo "== $v"; python -c "
import json
for l in open('$O/race6_$v.jsonl'):
    d=json.loads(l); print(d['k'], d['streams'], sum(r['bad_batches'] for r in d['per_round']), [r['err'] for r in d['per_round'] if r['err']])"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "round_robin or sweep or ties or padding" > $O/race6_test.log 2>&1; tail -2 $O/race6_test.log
