#!/bin/bash
# A/B: splitter-walker target 2^18 / 2^19 / 2^21 vs 2^20 on C2 (twice). ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  AB_ARGS="--workload c2" timeout -k 10 300 bash tools/ab_libs.sh .ab/sw18/libkmerhash_amd.so .ab/sw19/libkmerhash_amd.so \
    .ab/sw21/libkmerhash_amd.so >> gpurun_out/ab_seg.txt 2>&1
done
