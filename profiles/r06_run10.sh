#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_add.py tests/test_gpu_ip.py tests/test_gpu_repair.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
bash profiles/r06_prof.sh r06k
