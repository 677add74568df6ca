#!/bin/bash
# r04 profiles: kernel trace + stats of bench.py one batch at a time and with two in
# flight, then the scan kernel's PMC passes (one group per run) -> r04_scan_pmc.json
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r04prof_serial -o run -- python3 $R/bench.py --no-recall --no-cpu-baseline --no-extra --inflight 1 --steps 50 --warmup 10 > $O/r04prof_serial.json 2> $O/r04prof_serial.log || { echo "serial trace failed"; tail -5 $O/r04prof_serial.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r04prof_inflight -o run -- python3 $R/bench.py --no-recall --no-cpu-baseline --no-extra --steps 50 --warmup 10 > $O/r04prof_inflight.json 2> $O/r04prof_inflight.log || { echo "inflight trace failed"; tail -5 $O/r04prof_inflight.log; exit 1; }
bash $R/profiles/pmc_kernel.sh r04 "k_scan_lists" "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU" -- --inflight 1 > $O/r04_pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/r04_pmc.log; exit 1; }
tail -30 $O/r04_pmc.log
