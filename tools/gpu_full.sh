#!/bin/bash
# Full GPU suite (incl. the config-size tests) + default bench (C3) + C2 bench + forced 1-rank
# sharded bench. Run ON the GPU box. A heartbeat line per minute keeps the run visibly alive.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 600 \
  --timeout-method thread > gpurun_out/t_gpu.log 2>&1
timeout -k 10 400 python bench.py --steps 7 --warmup 2 > gpurun_out/bench.log 2>&1
timeout -k 10 300 python bench.py --workload c2 --steps 7 --warmup 2 --cpu-sample 0 > gpurun_out/bench_c2.log 2>&1
KH_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 --steps 3 --warmup 1 --cpu-sample 0 \
  > gpurun_out/b_dist_migrate.log 2>&1
