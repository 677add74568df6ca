#!/bin/bash
# where k_coarse_segtop's time goes (C4: nlist 65536, d 96, 1024 queries): shipped vs without
# the key tiles (nomma) vs without the selection (nosel) -- timing-only builds, wrong results
set -u
O=gpurun_out
for v in default nomma nosel; do
  if [ $v = default ]; then L=""; else L=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so; fi
  IVFPQ_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/segab_$v -o run -- python3 -u profiles/coarse_large_nlist.py > $O/segab_$v.jsonl 2> $O/segab_$v.log || { echo "$v failed"; exit 1; }
done
