#!/bin/bash
# Build the C-ABI library with extra compile flags into .ab/<name>/libkmerhash_amd.so (A/B runs:
# KH_LIB=.ab/<name>/libkmerhash_amd.so, tools/ab_libs.sh). Run here (CPU), not on the GPU box.
#   tools/build_variant.sh q0 -DKH_QMODE=0
set -e
NAME=$1; shift
D=$(dirname "$0")/../.ab/$NAME
rm -rf $D
mkdir -p $D/obj
cd $(dirname "$0")/../cs267_hw3_amd/csrc
PIDS=()
for f in kh_kernels.hip kh_build.hip kh_mwalk.hip kh_mseg.hip kh_gen.hip kh_capi.cpp kh_host.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function "$@" -c $f -o ../../.ab/$NAME/obj/$f.o &
  PIDS+=($!)
done
for p in "${PIDS[@]}"; do wait $p || { echo "compile failed"; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../.ab/$NAME/libkmerhash_amd.so ../../.ab/$NAME/obj/*.o -lpthread
echo built .ab/$NAME/libkmerhash_amd.so
