#!/bin/bash
# forcezero bisection (profiles/build_wz_bisect.sh): one stream + the side-stream copy loop
# (the condition that fails, profiles/r04_race_hog.sh), 1000 rounds x 24 k = 10 batches,
# with the coarse / scan / merge launches taken from the forcezero copy, and neither;
# then the closing pass (profiles/r04_final3.sh)
set -u
O=gpurun_out
L=chameleon-rag-acceleration_amd/lib/var/wzb/libivfpq.so
for m in scan merge coarse none; do
  IVFPQ_WZ=$m IVFPQ_LIB=$L RACE_ROUNDS=1000 timeout -k 10 300 python3 -u profiles/race_diag.py 10,1,1 > $O/race_wzb_$m.jsonl 2> $O/race_wzb_$m.log || { echo "$m failed"; tail -20 $O/race_wzb_$m.log; exit 1; }
  echo "== $m: $(cut -c1-200 $O/race_wzb_$m.jsonl)"
done
bash profiles/r04_final3.sh
