#!/bin/bash
# Kernel-trace + PMC profile of the default bench workload (run ON the GPU box):
#   tools/profile_round.sh <tag>   -> gpurun_out/prof_<tag>/{kernel_stats.txt,pmc_traffic.json,...}
# One counter per rocprofv3 pass (FETCH_SIZE / WRITE_SIZE do not fit one pass on gfx950);
# --pmc is never combined with sys/runtime tracing.
set -eo pipefail
export TMPDIR=/tmp
TAG=${1:-run}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/trace -- $B > $OUT/trace.log 2>&1
python3 tools/kstats.py $OUT/trace > $OUT/kernel_stats.txt
for c in FETCH_SIZE WRITE_SIZE TCC_EA0_ATOMIC_sum; do
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $PWD/$OUT/pmc_$c -- $B > $OUT/pmc_$c.log 2>&1
done
python3 tools/pmc_traffic.py c3 200000000 $OUT/pmc_ $OUT/pmc_traffic.json > /dev/null
grep '"metric"' $OUT/trace.log > $OUT/bench_under_trace.json || true
echo "profile $TAG done"
