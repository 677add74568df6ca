#!/bin/bash
# Bisection library for the forcezero effect (profiles/r04_race.txt item 12): the kernels
# built twice, normally and with -mllvm -amdgpu-waitcnt-forcezero; the second copy's
# launchers renamed *_wz and every other symbol of it made local; index built with
# -DWZ_BISECT so IVFPQ_WZ = coarse | scan | merge picks that stage's launches from the
# forcezero copy.  Output: lib/var/wzb/libivfpq.so
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/chameleon-rag-acceleration_amd/csrc
O=$R/chameleon-rag-acceleration_amd/lib/var/wzb
mkdir -p "$O"
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -I$R/include -I$C -DWZ_BISECT"
K="-mllvm -amdgpu-atomic-optimizer-strategy=None"
/opt/rocm/bin/hipcc $F $K -c -o "$O/k.o" "$C/ivfpq_kernels.hip" &
/opt/rocm/bin/hipcc $F $K -mllvm -amdgpu-waitcnt-forcezero -c -o "$O/kz.o" "$C/ivfpq_kernels.hip" &
/opt/rocm/bin/hipcc $F -x hip -c -o "$O/i.o" "$C/ivfpq_index.cpp" &
/opt/rocm/bin/hipcc $F -c -o "$O/b.o" "$C/ivfpq_build.hip" &
wait
ren=""
keep=""
for f in set_launch_parts launch_scan_lists launch_coarse_keys launch_coarse_select; do
  sym=$(nm "$O/kz.o" | awk -v f="$f" '$2 == "T" && $3 ~ ("^_ZN5chivf" length(f) f) {print $3}' | head -1)
  [ -n "$sym" ] || { echo "no symbol for $f"; exit 1; }
  new=$(echo "$sym" | sed "s/_ZN5chivf${#f}${f}/_ZN5chivf$((${#f} + 3))${f}_wz/")
  ren="$ren --redefine-sym $sym=$new"
  keep="$keep --keep-global-symbol=$new"
done
objcopy $ren "$O/kz.o" "$O/kz2.o"
objcopy $keep "$O/kz2.o" "$O/kz3.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$O/libivfpq.so" "$O/k.o" "$O/kz3.o" "$O/b.o" "$O/i.o"
rm -f "$O"/*.o
nm -D "$O/libivfpq.so" | grep -c "_wz" 
echo "built $O/libivfpq.so"
