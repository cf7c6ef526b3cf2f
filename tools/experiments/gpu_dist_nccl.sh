#!/bin/bash
# RCCL code paths at one rank: exchanges forced (self all-to-all), chunked per-peer-list
# all-to-all (64 MiB chunks), both walk protocols; ground truth checked by bench_main.
set -eo pipefail
export TMPDIR=/tmp
for proto in migrate fixed; do
  KH_DIST_SELF_EXCHANGE=1 KH_A2A_CHUNK_MB=64 KH_DIST_PROTOCOL=$proto KH_BENCH_FORCE_DIST=1 timeout -k 10 300 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29546 \
    bench.py --gpus 1 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/nccl_$proto.log 2>&1
done
timeout -k 10 600 python -m pytest tests/test_gpu_dist.py -x -q -k "hash_owner or golden" > gpurun_out/t_dist2.log 2>&1
