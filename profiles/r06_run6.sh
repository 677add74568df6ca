#!/bin/bash
# r06 sixth GPU pass: coarse-kernel phase stamps and an in-flight kernel trace of the bench.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r06g
mkdir -p $O
V=$R/chameleon-rag-acceleration_amd/lib/var
NGEMM=512 IVFPQ_LIB=$V/cdiag/libivfpq.so timeout -k 10 300 python -u profiles/diag_coarse.py > $O/cstamps.txt 2>&1 || { echo cstamps failed; tail -20 $O/cstamps.txt; exit 1; }
cat $O/cstamps.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace -o run -- python3 $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-recall --no-extra --no-peak > $R/$O/traced.json 2> $R/$O/traced.err || { echo traced failed; tail -5 $R/$O/traced.err; exit 1; }
ls $R/$O/trace
echo done
