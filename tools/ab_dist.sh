#!/bin/bash
# A/B environment settings on the forced one-rank sharded bench (ON the GPU box):
#   tools/ab_dist.sh <tag> "<ENV=..>" ...   (AB_ARGS: extra bench args, e.g. --workload c5)
set -eo pipefail
TAG=$1; shift
mkdir -p gpurun_out/abd_$TAG
i=0
for e in "$@"; do
  env $e KH_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port $((29600 + i)) bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu \
    --e2e-steps 0 ${AB_ARGS:-} > gpurun_out/abd_$TAG/b$i.log 2>&1
  echo "$e: $(grep 'step ms' gpurun_out/abd_$TAG/b$i.log) $(grep -o '"walk_rounds": [0-9]*' gpurun_out/abd_$TAG/b$i.log) $(grep -o '"verified_vs_truth": [a-z]*' gpurun_out/abd_$TAG/b$i.log)"
  i=$((i+1))
done
