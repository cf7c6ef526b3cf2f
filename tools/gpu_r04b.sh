#!/bin/bash
# round-4 validation batch (ON the GPU box): protocol tests, benches, A/Bs
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_steps.sh "tests:dist or driver or cpp or 8_ranks or configs or sharded or load or 0.85" "dist:c3:"
timeout -k 10 300 ./tools/kh_bench_cpp --ranks 1 --steps 5 --warmup 2 > gpurun_out/cpp_c3.log 2>&1
tools/ab_libs.sh .ab/sortil/libkmerhash_amd.so > gpurun_out/ab2.txt 2>&1
AB_ARGS="--load 0.85" tools/ab_env.sh l85 "X=1" "KH_DEBUG=probe_build" > gpurun_out/ab_85.txt 2>&1
timeout -k 10 300 python bench.py --workload c5h --no-cpu --e2e-steps 0 --steps 5 --warmup 2 > gpurun_out/bench_c5h.log 2>&1
