#!/bin/bash
# The round's measurement recipe (run on the GPU box via gpurun).  Usage: bash profiles/run_profiles.sh <tag> [bench args]
#  1. PMC passes (one counter group per rocprofv3 run, never combined with tracing) over the
#     scan kernels -> scan_pmc.json (per-launch HBM bytes, gfx950 FETCH_SIZE correction)
#  2. bench.py (the driver's command) with roofline.traffic taken from (1) -> bench.json
#  3. rocprofv3 --kernel-trace --stats of that same bench command -> trace/ + kernel_summary.txt
set -u
TAG=${1:-r01}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT/pmc"
cd /tmp && export TMPDIR=/tmp
PB="$R/bench.py --no-recall --no-cpu-baseline --no-extra --steps 10 --warmup 2 $*"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "k_scan|k_merge_probes|k_coarse|k_plan" \
    --output-format csv -d "$OUT/pmc/g$i" -o run -- python3 $PB > "$OUT/pmc/g$i.json" 2> "$OUT/pmc/g$i.err" || exit $?
  i=$((i+1))
done
KEY=$(python3 -c "import json,sys; j=json.load(open('$OUT/pmc/g0.json')); c=j['config']; print(c['key'])")
LIB=$(python3 -c "import sys; sys.path.insert(0, '$R/chameleon-rag-acceleration_amd'); from faiss_amd import _lib; print(_lib.LIB_PATH)")
python3 $R/profiles/make_pmc_json.py "$OUT/pmc" "$KEY" "$OUT/scan_pmc.json" "$LIB" > /dev/null || exit $?
timeout -k 10 400 python3 $R/bench.py --pmc-json "$OUT/scan_pmc.json" "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 $R/bench.py --pmc-json "$OUT/scan_pmc.json" "$@" > "$OUT/bench_traced.json" 2> "$OUT/bench_traced.err" || exit $?
WK=$(python3 -c "import json; j=json.loads(open('$OUT/bench_traced.json').read().strip().splitlines()[-1]); print(j['warmup'], j['steps'])")
python3 $R/profiles/summarize_trace.py "$OUT/trace/run_kernel_trace.csv" 20 --passes $WK > "$OUT/kernel_summary.txt" 2>&1
cat "$OUT/bench.json"; head -24 "$OUT/kernel_summary.txt"
echo "profiles done: $OUT"
