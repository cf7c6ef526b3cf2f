#!/bin/bash
# Text-path parity, C3 / C5 / C5F bench, the forced one-rank sharded line (direct + routed). ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/t_parity.log 2>&1
for w in c3 c5 c5f; do
  AB_ARGS="--workload $w" timeout -k 10 300 bash tools/ab_libs.sh >> gpurun_out/ab_r05e.txt 2>&1
done
KH_BENCH_FORCE_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 --no-cpu --e2e-steps 0 --steps 5 --warmup 2 \
  > gpurun_out/b_dist.log 2>&1
