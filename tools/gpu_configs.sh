#!/bin/bash
# Config-size GPU tests (C3 200M, C3-shape vs oracle, C4 1B / C5 200M at 8 logical ranks) plus
# the C++ sharded-table tests; a heartbeat line per minute keeps the run visibly alive.
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_cpp_api.py -x -v --durations=0 \
  --timeout 600 --timeout-method thread > gpurun_out/r2_configs.log 2>&1
rc=$?
kill $HB
exit $rc
