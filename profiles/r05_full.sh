#!/bin/bash
# r05: every gpu test (incl. the in-flight stress and caller replays), smoke(), bench.py defaults
set -u
O=gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r05_gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/r05_gputest.log; exit 1; }
tail -1 $O/r05_gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r05_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/r05_smoke.log; exit 1; }
tail -1 $O/r05_smoke.log
timeout -k 10 400 python3 -u bench.py > $O/r05_bench.json 2> $O/r05_bench.log || { echo "bench failed"; tail -20 $O/r05_bench.log; exit 1; }
cat $O/r05_bench.json
