#!/bin/bash
# C5 (skewed) checks on the GPU box: tests, single-GPU bench, forced one-rank sharded bench.
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread -k "c5" > gpurun_out/t_c5.log 2>&1
timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 > gpurun_out/bench_c5.log 2>&1
KH_BENCH_FORCE_DIST=1 KH_BENCH_PHASES=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29547 bench.py --workload c5 --gpus 1 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c5_dist1.log 2>&1
