#!/bin/bash
# Dump the gfx950 assembly of one kernel of ivfpq_kernels.hip (mangled-name regex) to /tmp/kernel.s
# and print its lines matching a pattern.  Usage: bash profiles/isa.sh <symbol-regex> [grep-regex] [max lines]
R=$(cd "$(dirname "$0")/.." && pwd)
SYM=${1:-k_scan_sysILi1ELb0E}
PAT=${2:-"ds_read_b128|lgkmcnt"}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I"$R/include" \
  -I"$R/chameleon-rag-acceleration_amd/csrc" --cuda-device-only -S -o /tmp/all.s \
  "$R/chameleon-rag-acceleration_amd/csrc/ivfpq_kernels.hip" 2>/dev/null || exit 1
L=$(grep -n "^_ZN.*${SYM}.*:" /tmp/all.s | head -1 | cut -d: -f1)
E=$(awk -v s="$L" 'NR>s && /^\.Lfunc_end/ {print NR; exit}' /tmp/all.s)
sed -n "${L},${E}p" /tmp/all.s > /tmp/kernel.s
echo "lines $L-$E -> /tmp/kernel.s ($(wc -l < /tmp/kernel.s) lines)"
grep -nE "$PAT" /tmp/kernel.s | head -${3:-80}
