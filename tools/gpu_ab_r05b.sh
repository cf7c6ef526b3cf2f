#!/bin/bash
# Parity tests of the text path, then A/B on C3 / C5 / C5F: the round-4 heads + chunks writers
# (oldtext) vs the line writer, one thread per chunk in the chunk writer (tpc1), 32 walker batches
# per atomic (wb32). ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/t_parity.log 2>&1
for w in c3 c5 c5f; do
  AB_ARGS="--workload $w" timeout -k 10 600 bash tools/ab_libs.sh .ab/oldtext/libkmerhash_amd.so \
    .ab/tpc1/libkmerhash_amd.so .ab/wb32/libkmerhash_amd.so >> gpurun_out/ab_r05b.txt 2>&1
done
