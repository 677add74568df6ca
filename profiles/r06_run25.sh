#!/bin/bash
# shard emulation (N = 1..8, three in flight) with the preassigned scans on every CU vs 16 CUs left free
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06e2
mkdir -p $O
for f in 0 16; do
  IVFPQ_SCAN_FREE_CUS=$f timeout -k 10 500 python -u profiles/shard_emulation.py > $O/emul_f$f.jsonl 2> $O/emul_f$f.err || { echo "emulation $f failed"; tail -10 $O/emul_f$f.err; exit 1; }
  grep "^{" $O/emul_f$f.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    j=json.loads(l); print('free $f N', j['N'], {k: round(v,4) for k,v in j['step_wall_ms'].items()})"
done
