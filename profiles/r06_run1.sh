#!/bin/bash
# r06 first GPU pass: the gpu suite, smoke, the default bench, and the shard flow at
# world size 1 with real RCCL collectives (one communicator, then one per stream).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 400 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gputest.log; exit 1; }
tail -3 $O/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
timeout -k 10 240 python -u bench.py --shard-at-1 --no-cpu-baseline --no-recall > $O/shard1_one.json 2> $O/shard1_one.err || { echo shard1 failed; tail -20 $O/shard1_one.err; exit 1; }
timeout -k 10 240 python -u bench.py --shard-at-1 --comms per-stream --no-cpu-baseline --no-recall > $O/shard1_per.json 2> $O/shard1_per.err || { echo shard1 per failed; tail -20 $O/shard1_per.err; exit 1; }
echo done
