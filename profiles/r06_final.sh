#!/bin/bash
# r06 final measurements on the shipped library.
#   bash profiles/r06_final.sh measure  -> traces + PMC (profiles/r06_prof.sh), the counter
#        file copied to profiles/r06_scan_pmc.json (on the box's copy), then the default
#        bench line (picks up that traffic), and the shard flow at world 1 over RCCL
#   bash profiles/r06_final.sh tests    -> the whole -m gpu suite and smoke()
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r06final
mkdir -p $O
case "${1:-measure}" in
measure)
  bash profiles/r06_prof.sh r06final > $O/prof_call.log 2>&1 || { echo "profiles failed"; tail -20 $O/prof_call.log; exit 1; }
  tail -5 $O/prof_call.log
  cp $O/scan_pmc.json profiles/r06_scan_pmc.json
  timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -10 $O/bench.err; exit 1; }
  tail -1 $O/bench.json
  timeout -k 10 400 python -u bench.py --shard-at-1 --no-cpu-baseline --no-recall > $O/shard1.json 2> $O/shard1.err || { echo "shard bench failed"; tail -10 $O/shard1.err; exit 1; }
  tail -1 $O/shard1.json
  ;;
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gputest.log; exit 1; }
  tail -1 $O/gputest.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -10 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  timeout -k 10 600 python -u profiles/shard_emulation.py > $O/shard_emulation.jsonl 2> $O/shard_emulation.err || { echo "emulation failed"; tail -10 $O/shard_emulation.err; exit 1; }
  cut -c1-200 $O/shard_emulation.jsonl
  ;;
esac
