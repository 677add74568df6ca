#!/bin/bash
# r04 config runs: C4 per-GPU shard built from 1 M-vector slices (125 M vectors) with the
# oracle check; C1 / C3 / C4 rates; the one-GPU shard emulation
set -u
O=gpurun_out
timeout -k 10 600 python -u profiles/c4_shard.py --slice 1000000 --check > $O/r04_c4_shard.json 2> $O/r04_c4_shard.log || { echo "c4 failed"; tail -20 $O/r04_c4_shard.log; exit 1; }
cat $O/r04_c4_shard.json
timeout -k 10 600 python -u profiles/config_rates.py > $O/r04_config_rates.jsonl 2> $O/r04_config_rates.log || { echo "rates failed"; tail -20 $O/r04_config_rates.log; exit 1; }
cat $O/r04_config_rates.jsonl
timeout -k 10 400 python -u profiles/shard_emulation.py > $O/r04_shard_emulation.jsonl 2> $O/r04_shard_emulation.log || { echo "shard emulation failed"; tail -20 $O/r04_shard_emulation.log; exit 1; }
cat $O/r04_shard_emulation.jsonl
