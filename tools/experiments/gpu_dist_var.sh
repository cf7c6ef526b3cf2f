#!/bin/bash
# Sharded 1-rank bench repeated (variance hunt), with per-phase timings. ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp KH_BENCH_FORCE_DIST=1 KH_BENCH_PHASES=1
for i in 1 2 3; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2955$i bench.py --gpus 1 --steps 4 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/bdv_$i.log 2>&1
done
