#!/bin/bash
# final library (overlap compiled out): every gpu test, smoke(), and bench.py with defaults
set -u
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r04g_gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/r04g_gputest.log; exit 1; }
tail -1 $O/r04g_gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r04g_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/r04g_smoke.log; exit 1; }
tail -1 $O/r04g_smoke.log
timeout -k 10 400 python3 -u bench.py > $O/r04g_bench.json 2> $O/r04g_bench.log || { echo "bench failed"; tail -20 $O/r04g_bench.log; exit 1; }
cat $O/r04g_bench.json
