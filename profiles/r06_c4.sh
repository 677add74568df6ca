#!/bin/bash
# C4 per-GPU shard (rank 0 of 8: 125 M vectors, 6 GB of codes) on the r06 library:
# rate + roofline, a 64-query oracle check, then counter traffic of its scan kernel.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r06c4
mkdir -p $O/pmc
timeout -k 10 400 python -u profiles/c4_shard.py --check > $O/c4.json 2> $O/c4.err || { echo c4 failed; tail -10 $O/c4.err; exit 1; }
tail -1 $O/c4.json
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  timeout -k 10 400 rocprofv3 --pmc $grp --kernel-include-regex "k_scan_lists" --output-format csv -d $R/$O/pmc/g$i -o run -- python3 $R/profiles/c4_shard.py --steps 6 > $R/$O/pmc/g$i.json 2> $R/$O/pmc/g$i.err || { echo "pmc pass $i failed"; tail -5 $R/$O/pmc/g$i.err; exit 1; }
  i=$((i+1))
done
python3 $R/profiles/c4_traffic.py $R/$O/pmc $R/$O/c4.json $R/$O/c4_traffic.json
