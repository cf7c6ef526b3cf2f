#!/bin/bash
# A/B the C3 bench: old tree in .ab/ vs the working tree, interleaved, same box (+ GPU tests of
# the working tree first when ABTEST=1). Run ON the GPU box.
set -eo pipefail
if [ "${ABTEST:-0}" = 1 ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t_gpu.log 2>&1
fi
for i in 1 2; do
  (cd .ab && timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample 0 ${ABARGS:-} > ../gpurun_out/ab_old_$i.log 2>&1)
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample 0 ${ABARGS:-} > gpurun_out/ab_new_$i.log 2>&1
done
