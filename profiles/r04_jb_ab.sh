#!/bin/bash
# JB (code chunks held in registers per item) at M > 32: shipped 2 vs 4 (jb4), C3 and C4 rates
set -u
O=gpurun_out
for v in default jb4; do
  if [ $v = default ]; then L=""; else L=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so; fi
  IVFPQ_LIB=$L timeout -k 10 500 python -u profiles/config_rates.py --only c3,c4 --reps 10 > $O/jbab_$v.jsonl 2> $O/jbab_$v.log || { echo "$v failed"; tail -5 $O/jbab_$v.log; exit 1; }
  echo "== $v"; python -c "
import json
for l in open('$O/jbab_$v.jsonl'):
    d=json.loads(l); print(d['config'][:12], d['k'], round(d['ms_per_batch'],4), round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],3))"
done
