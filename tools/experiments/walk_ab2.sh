#!/bin/bash
# Walker group sizes on C3 and C2 (KH_WALK_G). ON the GPU box.
set -eo pipefail
for G in ${GS3:-2 4}; do
  KH_WALK_G=$G timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-verify > gpurun_out/walk_G$G.log 2>&1
done
for G in ${GS2:-1 4 8 16}; do
  KH_WALK_G=$G timeout -k 10 300 python bench.py --workload c2 --steps 10 --warmup 2 --cpu-sample 0 --no-verify > gpurun_out/walkc2_G$G.log 2>&1
done
