#!/bin/bash
# r05 final profiles: kernel traces (one batch at a time / two in flight), PMC passes of the
# search kernels (one group per run), the counter file for bench.py, and bench.py with it
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=r05f
bash $R/profiles/r05_prof.sh $T > $O/${T}_prof.log 2>&1 || { echo "profiles failed"; tail -20 $O/${T}_prof.log; exit 1; }
python3 $R/profiles/make_pmc_json.py $O/pmc_$T "nb1000000-d128-IVF1024-PQ16-np16-k10-B1024-w1-single-c200000" $O/r05_scan_pmc.json $R/chameleon-rag-acceleration_amd/lib/libivfpq.so > $O/${T}_pmcjson.log 2>&1 || { echo "pmc json failed"; tail -5 $O/${T}_pmcjson.log; exit 1; }
cd $R
timeout -k 10 400 python3 -u bench.py --pmc-json $O/r05_scan_pmc.json > $O/r05f_bench.json 2> $O/r05f_bench.log || { echo "bench failed"; tail -20 $O/r05f_bench.log; exit 1; }
tail -c 1500 $O/r05f_bench.json
