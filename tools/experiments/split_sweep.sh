#!/bin/bash
# C3 / C2 bench: default splitter policy vs off. Run ON the GPU box.
set -eo pipefail
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t_gpu.log 2>&1
for w in c3 c2; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/split_${w}_def.log 2>&1
  KH_SPLIT_BITS=0 timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/split_${w}_0.log 2>&1
done
