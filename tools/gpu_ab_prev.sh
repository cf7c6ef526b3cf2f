#!/bin/bash
# Working tree vs the committed library (.ab/prev: SRC_REV=HEAD tools/build_variant.sh prev): full
# GPU suite, then A/B on C3 / C5 / C2 and
# the forced one-rank sharded line. ON the GPU box. SUITE=0 skips the suite; AB_WORKLOADS picks the lines.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
[ "${SUITE:-1}" = 0 ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=5 --timeout 600 --timeout-method thread \
  > gpurun_out/t_gpu.log 2>&1
for w in ${AB_WORKLOADS:-c3 c5 c2 c3}; do
  AB_ARGS="--workload $w" timeout -k 10 300 bash tools/ab_libs.sh .ab/prev/libkmerhash_amd.so >> gpurun_out/ab_prev.txt 2>&1
done
for L in default .ab/prev/libkmerhash_amd.so; do
  if [ "$L" = default ]; then unset KH_LIB; else export KH_LIB=$PWD/$L; fi
  KH_BENCH_FORCE_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 --no-cpu --e2e-steps 0 --steps 5 --warmup 2 \
    > gpurun_out/b_dist.log 2>&1
  tail -n1 gpurun_out/b_dist.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('dist $L', round(d['ms_per_step'],3), d['phases_ms'], d.get('routed_one_rank'), d['verified_vs_truth'])" >> gpurun_out/ab_prev.txt
done
