#!/bin/bash
# Full GPU suite + default bench (C3) + C2 bench + forced 1-rank sharded bench. Run ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t_gpu.log 2>&1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
timeout -k 10 300 python bench.py --workload c2 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/bench_c2.log 2>&1
KH_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/b_dist_migrate.log 2>&1
