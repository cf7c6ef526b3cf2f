#!/bin/bash
# round-4 bench batch (ON the GPU box): both hosts' one-rank lines, library and env A/Bs, C5H
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 ./tools/kh_bench_cpp --ranks 1 --steps 5 --warmup 2 > gpurun_out/cpp_c3.log 2>&1
tools/ab_libs.sh .ab/sortil/libkmerhash_amd.so .ab/nt/libkmerhash_amd.so > gpurun_out/ab_libs.txt 2>&1
tools/ab_env.sh l50 "X=1" "KH_BALANCED=1" "KH_BALANCED=1 KH_DEBUG=probe_build" > gpurun_out/ab_50.txt 2>&1
AB_ARGS="--load 0.85" tools/ab_env.sh l85 "X=1" "KH_DEBUG=probe_build" > gpurun_out/ab_85.txt 2>&1
timeout -k 10 300 python bench.py --workload c5h --no-cpu --e2e-steps 0 --steps 5 --warmup 2 > gpurun_out/bench_c5h.log 2>&1
