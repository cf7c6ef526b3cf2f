#!/bin/bash
# Full GPU suite, then the bench on C3 / C5 / C5F / C5H. ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=8 --timeout 600 --timeout-method thread \
  > gpurun_out/t_gpu.log 2>&1
for w in c3 c5 c5f c5h; do
  AB_ARGS="--workload $w" timeout -k 10 300 bash tools/ab_libs.sh >> gpurun_out/ab_r05d.txt 2>&1
done
