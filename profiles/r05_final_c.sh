#!/bin/bash
# r05 final: profiles + counter file + bench (r05_final_b.sh), then the shard emulation
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/profiles/r05_final_b.sh || exit 1
cd $R
timeout -k 10 300 python3 -u profiles/shard_emulation.py > gpurun_out/r05_shard_emulation.jsonl 2> gpurun_out/r05_shard_emulation.log || { echo "emulation failed"; tail -5 gpurun_out/r05_shard_emulation.log; exit 1; }
cat gpurun_out/r05_shard_emulation.jsonl | cut -c1-200
