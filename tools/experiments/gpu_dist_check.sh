#!/bin/bash
# Sharded path on one GPU: threaded-rank parity tests, then the forced 1-rank dist bench for the
# given protocols, rank-count simulation, and a kernel trace. Run ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_dist.py -x -q > gpurun_out/t_dist.log 2>&1
for proto in ${PROTOS:-migrate}; do
  KH_DIST_PROTOCOL=$proto KH_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/b_dist_$proto.log 2>&1
done
timeout -k 10 200 python tools/dist_sim.py 51 20000000 8 > gpurun_out/sim.log 2>&1
bash tools/profile_dist1.sh dist1
