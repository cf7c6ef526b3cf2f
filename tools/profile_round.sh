#!/bin/bash
# Kernel-trace + PMC profile of the default bench workload (run ON the GPU box):
#   tools/profile_round.sh <tag>   -> gpurun_out/prof_<tag>/{kernel_stats.txt,pmc_traffic.json,...}
# One counter group per rocprofv3 pass (FETCH_SIZE / WRITE_SIZE do not fit one pass on gfx950);
# --pmc is never combined with sys/runtime tracing. The membench pass calibrates the request
# size of random 16-B loads (known load counts) against the same counters.
set -eo pipefail
export TMPDIR=/tmp
TAG=${1:-run}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --e2e-steps 0 --no-verify ${BARGS:-}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/trace -- $B > $OUT/trace.log 2>&1
python3 tools/kstats.py $OUT/trace > $OUT/kernel_stats.txt
for c in FETCH_SIZE WRITE_SIZE TCC_EA0_ATOMIC_sum; do
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $PWD/$OUT/pmc_$c -- $B > $OUT/pmc_$c.log 2>&1
done
timeout -k 10 400 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum --output-format csv -d $PWD/$OUT/pmc_RDREQ -- $B > $OUT/pmc_RDREQ.log 2>&1
python3 tools/pmc_traffic.py c3 200000000 $OUT/pmc_ $OUT/pmc_traffic.json > /dev/null
# one pass of the 8 SQ counters behind DESIGN's bound statements (wave parking, VALU, LDS conflicts)
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
timeout -k 10 400 rocprofv3 --kernel-trace --pmc $SQ --output-format csv -d $PWD/$OUT/pmc_SQ -- $B > $OUT/pmc_SQ.log 2>&1
python3 tools/sq_summary.py $OUT/pmc_SQ > $OUT/sq_counters.json
grep '"metric"' $OUT/trace.log > $OUT/bench_under_trace.json || true
if [ -x tools/membench ]; then
  for c in FETCH_SIZE; do
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $PWD/$OUT/cal_$c -- tools/membench calib > $OUT/cal_$c.log 2>&1
  done
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum --output-format csv -d $PWD/$OUT/cal_RDREQ -- tools/membench calib > $OUT/cal_RDREQ.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $PWD/$OUT/cal_WRITE_SIZE -- tools/membench calib > $OUT/cal_WRITE_SIZE.log 2>&1
  python3 tools/pmc_traffic.py membench 0 $OUT/cal_ $OUT/pmc_traffic.json > /dev/null
fi
# the sharded path at one rank (KH_BENCH_FORCE_DIST: route, routed-word build, migrating walk):
# its PMC traffic goes in as workload "c3_dist" (the N > 1 bench line reads it). The env makes
# rank 0 of a one-rank process group without the torchrun launcher (the profiler runs python).
if [ -z "${NO_DIST:-}" ]; then
  D="python3 bench.py --steps 3 --warmup 1 --no-cpu --e2e-steps 0 --no-verify --no-routed ${BARGS:-}"
  export KH_BENCH_FORCE_DIST=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/dtrace -- $D > $OUT/dtrace.log 2>&1
  python3 tools/kstats.py $OUT/dtrace > $OUT/kernel_stats_dist.txt
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $PWD/$OUT/dpmc_$c -- $D > $OUT/dpmc_$c.log 2>&1
  done
  python3 tools/pmc_traffic.py c3_dist 200000000 $OUT/dpmc_ $OUT/pmc_traffic.json > /dev/null
  grep '"metric"' $OUT/dtrace.log > $OUT/bench_dist_under_trace.json || true
  unset KH_BENCH_FORCE_DIST RANK WORLD_SIZE LOCAL_RANK MASTER_ADDR MASTER_PORT
fi
echo "profile $TAG done"
