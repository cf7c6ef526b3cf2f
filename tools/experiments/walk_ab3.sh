#!/bin/bash
set -eo pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "walk_group or multi_walker or golden" > gpurun_out/t_walk.log 2>&1
for v in ${WV:-4:1 4:2 4:3 2:2 8:4 1:1}; do
  KH_WALK_G=${v%:*} KH_WALK_NS=${v#*:} timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-verify > gpurun_out/walk_${v/:/_}.log 2>&1
done
