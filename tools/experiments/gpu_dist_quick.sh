#!/bin/bash
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_driver.py tests/test_gpu_dist.py -x -q > gpurun_out/t_dq.log 2>&1
KH_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/b_dist_migrate.log 2>&1
