#!/bin/bash
# Round-5 iteration: GPU suite (stop at first failure), then C3 / C5H / C5F / C5 benches without the
# CPU legs, then the forced one-rank sharded bench, direct and routed. Run ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=10 --timeout 600 \
  --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/t_gpu.log 2>&1
B="--no-cpu --e2e-steps 0 --steps 7 --warmup 2"
for w in c3 c5h c5f c5; do
  timeout -k 10 300 python bench.py --workload $w $B > gpurun_out/bench_$w.log 2>&1
done
for w in c3 c5h c5f; do
  timeout -k 10 300 python bench.py --workload $w --load 0.85 $B > gpurun_out/bench_${w}_85.log 2>&1
done
KH_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu --e2e-steps 0 \
  > gpurun_out/b_dist.log 2>&1
KH_BENCH_FORCE_DIST=1 KH_DIST_ROUTE_ONE_RANK=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29545 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu \
  --e2e-steps 0 > gpurun_out/b_dist_routed.log 2>&1
