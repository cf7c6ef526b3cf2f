#!/bin/bash
# Forced 1-rank sharded bench (graph on/off) + kernel trace. Run ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
KH_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/b_dist_graph.log 2>&1
KH_DIST_GRAPH=0 KH_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29545 bench.py --gpus 1 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/b_dist_nograph.log 2>&1
bash tools/profile_dist1.sh dist1
