#!/bin/bash
# r05: the other BASELINE configs on one GPU (profiles/config_rates.py), C1 + C3 under a kernel trace
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05_cfgprof -o run -- python3 $R/profiles/config_rates.py --only c1,c3 > $O/r05_config_rates.jsonl 2> $O/r05_config_rates.log || { echo "c1/c3 failed"; tail -5 $O/r05_config_rates.log; exit 1; }
cat $O/r05_config_rates.jsonl | cut -c1-400
cd $R
timeout -k 10 400 python3 -u profiles/config_rates.py --only c4 > $O/r05_config_rates_c4.jsonl 2> $O/r05_config_rates_c4.log || { echo "c4 failed"; tail -5 $O/r05_config_rates_c4.log; exit 1; }
cat $O/r05_config_rates_c4.jsonl | cut -c1-400
