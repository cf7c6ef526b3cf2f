#!/bin/bash
# Sharded path on one GPU: threaded-rank parity tests, forced 1-rank dist bench (both
# protocols) and a kernel trace of the fixed protocol. Run ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests/test_gpu_dist.py -x -q > gpurun_out/t_dist.log 2>&1
KH_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/b_dist_fixed.log 2>&1
KH_DIST_PROTOCOL=variable KH_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29545 bench.py --gpus 1 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/b_dist_var.log 2>&1
bash tools/profile_dist1.sh dist1
