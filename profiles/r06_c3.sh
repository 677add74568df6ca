#!/bin/bash
# C3 (d 768, 2.68 M vectors, IVF4096,PQ64, IP, nprobe 32): rates + roofline under a kernel
# trace, then counter passes of its list-scan kernels -> gpurun_out/r06c3/c3_rates.jsonl
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=$R/gpurun_out/r06c3
mkdir -p $O/pmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/profiles/config_rates.py --only c3 > $O/rates.jsonl 2> $O/rates.log || { echo "c3 rates failed"; tail -5 $O/rates.log; exit 1; }
cut -c1-300 $O/rates.jsonl
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum"; do
  timeout -k 10 600 rocprofv3 --pmc $grp --kernel-include-regex "k_scan_lists" --output-format csv -d $O/pmc/g$i -o run -- python3 $R/profiles/config_rates.py --only c3 --reps 6 > $O/pmc/g$i.jsonl 2> $O/pmc/g$i.err || { echo "pmc pass $i failed"; tail -5 $O/pmc/g$i.err; exit 1; }
  i=$((i+1))
done
python3 $R/profiles/c3_traffic.py $O/pmc $O/trace/run_kernel_trace.csv $O/rates.jsonl $O/c3_rates.jsonl
