#!/bin/bash
# Parity of the text path and the hot families, then C3 / C5 / C5F / C5H benches with the line
# writer v1 (per-byte) vs v2 (v_perm) A/B. ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/t_parity.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -x -q -k "(hot or flank) and not 1b" --timeout 600 --timeout-method thread \
  > gpurun_out/t_hot.log 2>&1
for w in c3 c5 c5f c5h; do
  AB_ARGS="--workload $w" timeout -k 10 600 bash tools/ab_libs.sh .ab/lines1/libkmerhash_amd.so >> gpurun_out/ab_r05c.txt 2>&1
done
