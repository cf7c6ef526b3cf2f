#!/bin/bash
# Default bench (C3: HBM-resident value, reference-boundary figure, CPU baselines) + the
# kernel-trace/PMC profile of the same build. Run ON the GPU box:  tools/gpu_bench_prof.sh <tag>
set -eo pipefail
export TMPDIR=/tmp
TAG=${1:-head}
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.log 2>&1
bash tools/profile_round.sh $TAG
