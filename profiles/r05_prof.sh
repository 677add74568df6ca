#!/bin/bash
# r05 profiles: kernel trace + stats of bench.py one batch at a time and with two in
# flight (the default), then PMC passes (one counter group per run, no tracing) of the
# search kernels, one batch at a time
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=${1:-r05}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}prof_serial -o run -- python3 $R/bench.py --no-recall --no-cpu-baseline --no-extra --inflight 1 --steps 50 --warmup 10 > $O/${T}prof_serial.json 2> $O/${T}prof_serial.log || { echo "serial trace failed"; tail -5 $O/${T}prof_serial.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}prof_inflight -o run -- python3 $R/bench.py --no-recall --no-cpu-baseline --no-extra --steps 50 --warmup 10 > $O/${T}prof_inflight.json 2> $O/${T}prof_inflight.log || { echo "inflight trace failed"; tail -5 $O/${T}prof_inflight.log; exit 1; }
[ "${NO_PMC:-0}" = 1 ] && exit 0
bash $R/profiles/pmc_kernel.sh $T "k_scan_lists|k_coarse|k_merge" "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM" \
  -- --inflight 1 --mode replicas > $O/${T}_pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/${T}_pmc.log; exit 1; }
tail -40 $O/${T}_pmc.log
