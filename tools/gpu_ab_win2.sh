#!/bin/bash
# A/B: k_win2 with 1024 threads (8 words each) vs 512 (16 each), C3 twice and C5H. ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "golden or generated or build_kernels" > gpurun_out/t_parity.log 2>&1 || true
for w in c3 c5h c3; do
  AB_ARGS="--workload $w" timeout -k 10 300 bash tools/ab_libs.sh .ab/w2tb1024/libkmerhash_amd.so >> gpurun_out/ab_win2.txt 2>&1
done
