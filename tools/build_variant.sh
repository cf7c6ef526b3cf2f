#!/bin/bash
# Build the C-ABI library with extra compile flags into .ab/<name>/libkmerhash_amd.so (A/B runs:
# KH_LIB=.ab/<name>/libkmerhash_amd.so, tools/ab_libs.sh). Run here (CPU), not on the GPU box.
#   tools/build_variant.sh q0 -DKH_QMODE=0
#   SRC_REV=HEAD tools/build_variant.sh prev      (the committed sources, not the working tree)
set -e
NAME=$1; shift
R=$(cd $(dirname "$0")/.. && pwd)
D=$R/.ab/$NAME
rm -rf $D
mkdir -p $D/obj
if [ -n "$SRC_REV" ]; then
  mkdir -p $D/src && git -C $R archive $SRC_REV cs267_hw3_amd/csrc include | tar -x -C $D/src
  cd $D/src/cs267_hw3_amd/csrc
else
  cd $R/cs267_hw3_amd/csrc
fi
PIDS=()
for f in kh_kernels.hip kh_build.hip kh_mwalk.hip kh_mseg.hip kh_gen.hip kh_capi.cpp kh_host.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function "$@" -c $f -o $D/obj/$f.o &
  PIDS+=($!)
done
for p in "${PIDS[@]}"; do wait $p || { echo "compile failed"; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libkmerhash_amd.so $D/obj/*.o -lpthread
rm -rf $D/src
echo built .ab/$NAME/libkmerhash_amd.so
