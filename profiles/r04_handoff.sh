#!/bin/bash
# kernel-boundary hand-off micro (profiles/handoff_streams.hip), mode 6: readers pinned by
# XCD (a stale line kept in a reader XCD's L2 across the kernel boundary would be read),
# 1 and 3 streams, whole- and partial-line writes
set -u
O=gpurun_out
for s in 1 3; do for p in 0 1; do
  timeout -k 10 100 ./profiles/handoff_streams $s 2000 6 $p >> $O/handoff3.jsonl || { echo "handoff $s $p failed"; exit 1; }
done; done
cat $O/handoff3.jsonl
