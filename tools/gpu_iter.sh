#!/bin/bash
# Iteration run: GPU suite (stop at first failure), then C3 / C2 / C5 benches without the CPU
# legs, then the forced one-rank sharded bench. Run ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=10 --timeout 600 \
  --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/t_gpu.log 2>&1
B="--no-cpu --e2e-steps 0 --steps 7 --warmup 2"
timeout -k 10 300 python bench.py $B > gpurun_out/bench_c3.log 2>&1
timeout -k 10 300 python bench.py --workload c2 $B > gpurun_out/bench_c2.log 2>&1
timeout -k 10 300 python bench.py --workload c5 $B > gpurun_out/bench_c5.log 2>&1
KH_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu --e2e-steps 0 \
  > gpurun_out/b_dist.log 2>&1
