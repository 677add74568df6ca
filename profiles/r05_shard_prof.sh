#!/bin/bash
# r05: shard emulation (N = 1..8) plain, then under a kernel trace (per-kernel times per N)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd "$R"
timeout -k 10 300 python3 -u profiles/shard_emulation.py > $O/r05_shard_emulation.jsonl 2> $O/r05_shard_emulation.log || { echo "emulation failed"; tail -5 $O/r05_shard_emulation.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/r05_shardprof -o run -- python3 $R/profiles/shard_emulation.py --reps 5 > $O/r05_shardprof.jsonl 2> $O/r05_shardprof.log || { echo "trace failed"; tail -5 $O/r05_shardprof.log; exit 1; }
