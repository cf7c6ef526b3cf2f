#!/bin/bash
# Round-end rehearsal ON the GPU box: smoke(), the full GPU suite, the default bench line.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=5 --timeout 600 --timeout-method thread \
  > gpurun_out/t_gpu.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1
