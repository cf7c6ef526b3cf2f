#!/bin/bash
# Kernel trace of a short bench run: tools/trace_quick.sh <tag> [bench args...]. Run ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/tq_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/trace -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu --e2e-steps 0 --no-verify "$@" > $OUT/trace.log 2>&1
python3 tools/kstats.py $OUT/trace > $OUT/kernel_stats.txt
cat $OUT/kernel_stats.txt
