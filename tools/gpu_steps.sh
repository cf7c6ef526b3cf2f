#!/bin/bash
# Run named GPU steps in order on the GPU box, each under its own time limit, logs in gpurun_out/;
# stops at the first failure. Steps: tests[:<pytest -k expr>] | bench:<name>:<bench.py args> |
# dist:<name>:<bench.py args> (forced one-rank sharded bench).
#   tools/gpu_steps.sh "tests:hot" "bench:c3:" "bench:c5h:--workload c5h"
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
B="--no-cpu --e2e-steps 0 --steps 5 --warmup 2"
for step in "$@"; do
  kind=${step%%:*}; rest=${step#*:}
  case $kind in
    tests)
      K=()
      [ -n "$rest" ] && [ "$rest" != "tests" ] && K=(-k "$rest")
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 300 \
        --timeout-method thread "${K[@]}" > gpurun_out/t_gpu.log 2>&1 ;;
    bench)
      name=${rest%%:*}; args=${rest#*:}
      timeout -k 10 400 python bench.py $B $args > gpurun_out/bench_$name.log 2>&1 ;;
    dist)
      name=${rest%%:*}; args=${rest#*:}
      KH_BENCH_FORCE_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 $B $args > gpurun_out/dist_$name.log 2>&1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $step ok" >> gpurun_out/steps.log
done
