#!/bin/bash
# Walker-resolved splitter links: splitter parity tests, then A/B vs .ab/prev on C3 / C5 / C2. ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/t_parity.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 500 --timeout-method thread \
  -k "c2_10m or skewed" > gpurun_out/t_cfg.log 2>&1
for w in c3 c5 c2; do
  AB_ARGS="--workload $w" timeout -k 10 300 bash tools/ab_libs.sh .ab/prev/libkmerhash_amd.so >> gpurun_out/ab_link.txt 2>&1
done
