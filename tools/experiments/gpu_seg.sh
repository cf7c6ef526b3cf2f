#!/bin/bash
# Sharded walk with splitter segments: tests, then forced one-rank benches (C3, C5). ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_seg.log 2>&1
export KH_BENCH_FORCE_DIST=1 KH_BENCH_PHASES=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29548 bench.py --gpus 1 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bseg_c3.log 2>&1
KH_MW_SEGMENTS=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29549 bench.py --gpus 1 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bseg_c3_off.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29550 bench.py --workload c5 --gpus 1 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bseg_c5.log 2>&1
