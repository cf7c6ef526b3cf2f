#!/bin/bash
# Sharded path on the GPU box: its tests, then the forced 1-rank bench plain and with the
# self-exchange pipelined insert (route -> RCCL all-to-all -> staged build).
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_dist.log 2>&1
export KH_BENCH_FORCE_DIST=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bd_plain.log 2>&1
KH_DIST_SELF_EXCHANGE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29545 bench.py --gpus 1 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bd_self.log 2>&1
