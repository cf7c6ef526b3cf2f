#!/bin/bash
# A/B the C3 bench: old tree in .ab/ vs the working tree, interleaved, same box. Run ON the GPU box.
set -eo pipefail
for i in 1 2; do
  (cd .ab && timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample 0 ${ABARGS:-} > ../gpurun_out/ab_old_$i.log 2>&1)
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample 0 ${ABARGS:-} > gpurun_out/ab_new_$i.log 2>&1
done
