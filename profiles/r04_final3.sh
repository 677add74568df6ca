#!/bin/bash
# r04 closing pass on the final library: every gpu test, the kernel trace + stats of bench.py
# (defaults: one batch at a time), then the scan kernel's PMC passes -> r04_scan_pmc.json
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r04f_gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/r04f_gputest.log; exit 1; }
tail -1 $O/r04f_gputest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r04fprof -o run -- python3 $R/bench.py --no-recall --no-cpu-baseline --no-extra --steps 50 --warmup 10 > $O/r04fprof.json 2> $O/r04fprof.log || { echo "trace failed"; tail -5 $O/r04fprof.log; exit 1; }
bash $R/profiles/pmc_kernel.sh r04f "k_scan_lists" "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU" > $O/r04f_pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/r04f_pmc.log; exit 1; }
tail -12 $O/r04f_pmc.log
