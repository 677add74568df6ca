#!/bin/bash
# Build A/B variants of libivfpq.so (compile-time experiment switches) into lib/var/<name>/.
# Usage: build_variants.sh name:"-DFOO=1 -DBAR=2" ...   ; select one at run time with IVFPQ_LIB=<path>.
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/chameleon-rag-acceleration_amd/csrc
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -I$R/include -I$C"
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  O=$R/chameleon-rag-acceleration_amd/lib/var/$name
  mkdir -p "$O"
  /opt/rocm/bin/hipcc $F -mllvm -amdgpu-atomic-optimizer-strategy=None $defs -c -o "$O/k.o" "$C/ivfpq_kernels.hip" &
  /opt/rocm/bin/hipcc $F $defs -x hip -c -o "$O/i.o" "$C/ivfpq_index.cpp" &
  /opt/rocm/bin/hipcc $F $defs -c -o "$O/b.o" "$C/ivfpq_build.hip" &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$O/libivfpq.so" "$O/k.o" "$O/b.o" "$O/i.o"
  rm -f "$O/k.o" "$O/i.o" "$O/b.o"
  echo "built $name ($defs)"
done
