#!/bin/bash
# Kernel trace of the default single-GPU bench. Run ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof_${1:-c3}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/trace -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify ${2:-} > $OUT/trace.log 2>&1
python3 tools/kstats.py $OUT/trace > $OUT/kernel_stats.txt
