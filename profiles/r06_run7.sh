#!/bin/bash
# coarse-kernel stamps: in a search vs the coarse step run twice back to back
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r06h
mkdir -p $O
V=$R/chameleon-rag-acceleration_amd/lib/var
for m in search coarse2; do
  MODE=$m NGEMM=512 IVFPQ_LIB=$V/cdiag/libivfpq.so timeout -k 10 300 python -u profiles/diag_coarse.py > $O/cstamps_$m.txt 2>&1 || { echo cstamps failed; tail -20 $O/cstamps_$m.txt; exit 1; }
  echo "== $m"; grep -v "start\|end " $O/cstamps_$m.txt
done
timeout -k 10 60 ./profiles/coldload | tee $O/coldload.txt
