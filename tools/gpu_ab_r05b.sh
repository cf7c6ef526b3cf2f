#!/bin/bash
# A/B of chunk-writer threads per chunk (1 / 2 vs 4) and walker batches per atomic (2 / 32 vs 8)
# on C3, C5 and C5F, then the round-5 profile. ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
for w in c3 c5 c5f; do
  AB_ARGS="--workload $w" timeout -k 10 900 bash tools/ab_libs.sh .ab/tpc1/libkmerhash_amd.so .ab/tpc2/libkmerhash_amd.so \
    .ab/wb2/libkmerhash_amd.so .ab/wb32/libkmerhash_amd.so >> gpurun_out/ab_r05b.txt 2>&1
done
bash tools/profile_r05.sh
