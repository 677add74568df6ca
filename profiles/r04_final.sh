#!/bin/bash
# r04 final measurement pass (after the last kernel change): C3 rates + coarse split under a
# kernel trace, then profiles/r04_prof.sh (bench traces one batch at a time / two in flight,
# scan PMC passes), then the default bench line
set -u
O=gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r04d_c3prof -o run -- python3 -u profiles/config_rates.py --only c3 --reps 10 > $O/r04d_rates_c3.jsonl 2> $O/r04d_rates_c3.log || { echo "c3 failed"; tail -20 $O/r04d_rates_c3.log; exit 1; }
cat $O/r04d_rates_c3.jsonl
bash profiles/r04_prof.sh || exit 1
