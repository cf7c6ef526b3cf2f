#!/bin/bash
# Round-6 closing run ON the GPU box: smoke(), C5 and C3 kernel traces, the default bench line.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
bash tools/trace_quick.sh c5 --workload c5
bash tools/trace_quick.sh c3
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1
tail -1 gpurun_out/bench_default.log
