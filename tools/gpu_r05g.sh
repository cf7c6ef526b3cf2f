#!/bin/bash
# Walker with one place() site: parity, then A/B against the previous library on C3 / C5 / C5H.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/t_parity.log 2>&1
for w in c3 c5 c5h c3; do
  AB_ARGS="--workload $w" timeout -k 10 300 bash tools/ab_libs.sh .ab/prev/libkmerhash_amd.so >> gpurun_out/ab_r05g.txt 2>&1
done
