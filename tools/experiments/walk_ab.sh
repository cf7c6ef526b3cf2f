#!/bin/bash
# Walker shapes on the C3 bench (KH_WALK_G = lanes per contig), after the walk parity tests. ON the GPU box.
set -eo pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "walk_group or golden or generated_vs_oracle or c3_shape" > gpurun_out/t_walk.log 2>&1
for G in ${GS:-1 4 8}; do
  KH_WALK_G=$G timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-verify > gpurun_out/walk_G$G.log 2>&1
done
