#!/bin/bash
# A/B: line writer 4 blocks in flight (u4); segment chains 32 / 64 serial hops (ss32 / ss64) on C5 / C2 / C3.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in c5 c2 c3; do
  AB_ARGS="--workload $w" timeout -k 10 300 bash tools/ab_libs.sh .ab/u4/libkmerhash_amd.so .ab/ss32/libkmerhash_amd.so \
    .ab/ss64/libkmerhash_amd.so >> gpurun_out/ab_misc.txt 2>&1
done
