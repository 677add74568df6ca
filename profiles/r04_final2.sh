#!/bin/bash
# r04 closing pass (library at HEAD): every gpu test, C4 shard from 1 M slices, C1/C3/C4
# rates, then profiles/r04_prof.sh (traces + scan PMC) -- the counter file must come from
# the final kernels
set -u
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r04e_gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/r04e_gputest.log; exit 1; }
tail -1 $O/r04e_gputest.log
timeout -k 10 600 python -u profiles/c4_shard.py --slice 1000000 --check > $O/r04e_c4_shard.json 2> $O/r04e_c4_shard.log || { echo "c4 failed"; tail -20 $O/r04e_c4_shard.log; exit 1; }
cat $O/r04e_c4_shard.json
timeout -k 10 600 python -u profiles/config_rates.py > $O/r04e_config_rates.jsonl 2> $O/r04e_config_rates.log || { echo "rates failed"; tail -20 $O/r04e_config_rates.log; exit 1; }
cat $O/r04e_config_rates.jsonl
bash profiles/r04_prof.sh > $O/r04e_prof.log 2>&1 || { echo "prof failed"; tail -20 $O/r04e_prof.log; exit 1; }
tail -3 $O/r04e_prof.log
