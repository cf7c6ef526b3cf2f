#!/bin/bash
# Kernel trace of the sharded path forced at one rank (run ON the GPU box).
set -eo pipefail
export TMPDIR=/tmp
TAG=${1:-dist1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export KH_BENCH_FORCE_DIST=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/trace -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-verify > $OUT/trace.log 2>&1
python3 tools/kstats.py $OUT/trace > $OUT/kernel_stats.txt
echo done
