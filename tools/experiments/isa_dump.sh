#!/bin/bash
# Dump the gfx950 ISA of one kernel of kh_kernels.hip: tools/isa_dump.sh <symbol-substring> [out]
set -e
D=/tmp/kh_isa; mkdir -p $D
HERE=$(cd "$(dirname "$0")/.." && pwd)
( cd $D && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c "$HERE/cs267_hw3_amd/csrc/kh_kernels.hip" -save-temps -o k.o 2>/dev/null )
S=$D/kh_kernels-hip-amdgcn-amd-amdhsa-gfx950.s
SYM=$(grep -o "^_ZN2kh[A-Za-z0-9_]*$1[A-Za-z0-9_]*:" $S | head -1 | tr -d :)
awk -v s="$SYM" 'index($0, s":")==1 {p=1} p {print} p && /s_endpgm/ {exit}' $S > ${2:-$D/$1.s}
echo "$SYM -> ${2:-$D/$1.s} ($(wc -l < ${2:-$D/$1.s}) lines)"
