#!/bin/bash
# coherence experiment: the k = 100 in-flight mismatch with an agent-scope acquire at the
# radix merge's start (acq) and with an agent-scope release at the list scan's end (rel)
set -u
O=gpurun_out
export RACE_ROUNDS=12
for v in acq rel default; do
  if [ $v = default ]; then L=""; else L=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so; fi
  IVFPQ_LIB=$L timeout -k 10 300 python -u profiles/race_diag.py 100,3 100,2 100,4 > $O/race2_$v.jsonl 2> $O/race2_$v.log || { echo "$v failed"; tail -20 $O/race2_$v.log; exit 1; }
  echo "== $v"; python -c "
import json
for l in open('$O/race2_$v.jsonl'):
    d=json.loads(l); print(d['k'], d['streams'], sum(r['bad_batches'] for r in d['per_round']), sum(r['err'] for r in d['per_round']))"
done
# kernel trace of the failing pattern (per-stream ordering of scan -> merges)
RACE_ROUNDS=4 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/race2_trace -o run -- python3 -u profiles/race_diag.py 100,3 > $O/race2_trace.jsonl 2> $O/race2_trace.log || { echo "trace failed"; exit 1; }
cat $O/race2_trace.jsonl
