#!/bin/bash
# GPU suite, then A/B of the contig text writer (lanes per contig 32 default / 16 / 64, and the
# round-4 head + chunk writers) on C3 and C5, then the one-rank sharded benches. ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=5 --timeout 600 \
  --timeout-method thread > gpurun_out/t_gpu.log 2>&1
for w in c3 c5; do
  AB_ARGS="--workload $w" timeout -k 10 900 bash tools/ab_libs.sh .ab/g16/libkmerhash_amd.so .ab/g64/libkmerhash_amd.so .ab/wb1/libkmerhash_amd.so \
    .ab/oldw/libkmerhash_amd.so >> gpurun_out/ab_text.txt 2>&1
done
B="--no-cpu --e2e-steps 0 --steps 5 --warmup 2"
KH_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 $B > gpurun_out/b_dist.log 2>&1
KH_BENCH_FORCE_DIST=1 KH_DIST_ROUTE_ONE_RANK=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29545 bench.py --gpus 1 $B > gpurun_out/b_dist_routed.log 2>&1
