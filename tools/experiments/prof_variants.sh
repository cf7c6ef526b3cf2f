#!/bin/bash
# Kernel traces of the C3 bench under env variants: VARIANTS="name:ENV=V,ENV2=V2 ..." (ON the GPU box)
set -eo pipefail
export TMPDIR=/tmp
for v in $VARIANTS; do
  name=${v%%:*}; envs=${v#*:}
  OUT=gpurun_out/pv_$name; rm -rf $OUT; mkdir -p $OUT
  ( export $(echo $envs | tr ',' ' '); timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/trace -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify ${BARGS:-} > $OUT/log 2>&1 )
  python3 tools/kstats.py $OUT/trace > $OUT/kernel_stats.txt
done
