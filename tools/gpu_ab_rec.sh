#!/bin/bash
# A/B: records pass 1 with 640 threads (3840-record tiles, 20 waves per CU) vs 512 (3584, 16). ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in c3 c5h c3; do
  AB_ARGS="--workload $w" timeout -k 10 300 bash tools/ab_libs.sh .ab/rec640/libkmerhash_amd.so >> gpurun_out/ab_rec.txt 2>&1
done
