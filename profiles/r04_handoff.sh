#!/bin/bash
# kernel-boundary hand-off micro (profiles/handoff_streams.hip): long-lived writer
# (dirty lines held ~50 us) with plain and write-through stores, 1 and 3 streams
set -u
O=gpurun_out
for s in 1 3; do for p in 0 1; do for m in 4 5; do
  timeout -k 10 100 ./profiles/handoff_streams $s 1000 $m $p >> $O/handoff2.jsonl || { echo "handoff $s $m $p failed"; exit 1; }
done; done; done
cat $O/handoff2.jsonl
