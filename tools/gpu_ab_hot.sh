#!/bin/bash
# Hot-family tests + A/B (KH_LIB .ab/prev vs the tree) on C5H / C5F / C3. ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -k "(hot or flank) and not 1b" \
  --timeout 600 --timeout-method thread > gpurun_out/t_hot.log 2>&1
for w in c5h c5f c3; do
  AB_ARGS="--workload $w" timeout -k 10 300 bash tools/ab_libs.sh .ab/prev/libkmerhash_amd.so >> gpurun_out/ab_hot.txt 2>&1
done
