#!/bin/bash
# where k_merge_radix's time goes (C2, k = 100): timing-only builds that stop after the key
# loads (rs1), the radix select (rs2), the compaction (rs3), the labels (rs4); shipped = full
set -u
O=gpurun_out
for v in default rs1 rs2 rs3 rs4; do
  if [ $v = default ]; then L=""; else L=chameleon-rag-acceleration_amd/lib/var/$v/libivfpq.so; fi
  IVFPQ_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/rsplit_$v -o run -- python3 -u profiles/config_rates.py --only c2 --reps 10 > $O/rsplit_$v.jsonl 2> $O/rsplit_$v.log || { echo "$v failed"; exit 1; }
done
