#!/bin/bash
# r06 profiles: kernel trace + stats of bench.py one batch at a time and with two in
# flight (the default), then PMC passes (one counter group per run, no tracing) of the
# search kernels one batch at a time, and the counter file bench.py reads (traffic).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06}
T=${1:-r06}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_serial -o run -- python3 $R/bench.py --no-recall --no-cpu-baseline --no-extra --no-peak --inflight 1 --steps 50 --warmup 10 > $O/prof_serial.json 2> $O/prof_serial.log || { echo "serial trace failed"; tail -5 $O/prof_serial.log; exit 1; }
python3 $R/profiles/summarize_trace.py $O/prof_serial/run_kernel_trace.csv 12 > $O/kernel_summary.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_inflight -o run -- python3 $R/bench.py --no-recall --no-cpu-baseline --no-extra --no-peak --steps 50 --warmup 10 > $O/prof_inflight.json 2> $O/prof_inflight.log || { echo "inflight trace failed"; tail -5 $O/prof_inflight.log; exit 1; }
python3 $R/profiles/summarize_trace.py $O/prof_inflight/run_kernel_trace.csv 12 > $O/kernel_summary_inflight.txt 2>&1
head -30 $O/kernel_summary.txt
[ "${NO_PMC:-0}" = 1 ] && exit 0
bash $R/profiles/pmc_kernel.sh $T "k_scan_lean|k_scan_lists|k_coarse|k_merge" "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM" \
  -- --inflight 1 --no-peak > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
cp -r $R/gpurun_out/pmc_$T $O/pmc
python3 $R/profiles/make_pmc_json.py $O/pmc "nb1000000-d128-IVF1024-PQ16-np16-k10-B1024-w1-single-c200000" $O/scan_pmc.json $R/chameleon-rag-acceleration_amd/lib/libivfpq.so > $O/pmcjson.log 2>&1 || { echo "pmc json failed"; tail -5 $O/pmcjson.log; exit 1; }
grep -E "k_scan_lean|k_coarse_gemm |k_merge_probes<1>" $O/pmc/summary.txt | head -60
python3 -c "import json;j=json.load(open('$O/scan_pmc.json'));print('scan kernel', j['kernel'], 'hbm bytes per launch', j['hbm_bytes_per_launch'])"
