#!/bin/bash
# segmented coarse with per-query candidate queues + no zero-padded k-chunks: parity tests
# that take the segmented path, then the coarse step alone under a kernel trace
set -u
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_bigshapes.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "segmented or c4 or ralm or tiled or golden or sweep" > $O/segq_test.log 2>&1 || { echo "tests failed"; tail -30 $O/segq_test.log; exit 1; }
tail -1 $O/segq_test.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/segq_prof -o run -- python3 -u profiles/coarse_large_nlist.py > $O/segq.jsonl 2> $O/segq.log || { echo "prof failed"; exit 1; }
cat $O/segq.jsonl
