#!/bin/bash
# coarse GEMM ablations (-DGEMM_AB=1..5: no key stores / no centroid loads / no query
# staging / neither load / key workgroups exit at once): kernel durations by rocprofv3.
# The switches lived in the paired-load path of commit 48d3133, removed after r06s.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=$R/gpurun_out/r06n
mkdir -p $O
V=$R/chameleon-rag-acceleration_amd/lib/var
cd /tmp && export TMPDIR=/tmp
for v in ab0 ab1 ab2 ab3 ab4 ab5; do
  if [ $v = ab0 ]; then L=$R/chameleon-rag-acceleration_amd/lib/libivfpq.so; else L=$V/$v/libivfpq.so; fi
  IVFPQ_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $R/profiles/gemm_ab.py 200 > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  python3 - $O/$v/run_kernel_trace.csv $v <<'PY'
import csv, sys, collections, re
g = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Kernel_Name']
    if 'k_coarse' in n or 'k_scan' in n or 'k_merge_probes' in n:
        nm = re.search(r'k_\w+(<[^>]*>)?', n).group(0) + ' grid ' + r['Grid_Size_X']
        g[nm].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
for k, v in sorted(g.items()):
    v = sorted(v)
    print(f"{sys.argv[2]:4} {k:<44} n {len(v):4d} median {v[len(v)//2]:7.2f} us  min {v[0]:7.2f}")
PY
done
