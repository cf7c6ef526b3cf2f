#!/bin/bash
# Round-5 profile (ON the GPU box): the C3 kernel trace + PMC + SQ passes of profile_round.sh, then
# kernel traces of C5 (walker skew) and C5F (hot flank) for their walk / text phases.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
bash tools/profile_round.sh r05
for w in c5 c5f c5h; do
  OUT=gpurun_out/prof_r05/$w
  mkdir -p $OUT
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/trace -- \
    python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu --e2e-steps 0 --no-verify > $OUT/trace.log 2>&1
  python3 tools/kstats.py $OUT/trace > $OUT/kernel_stats.txt
done
# walker requests at C5H / C5F (random 64-B read requests of k_walk_q + k_rec_succ)
for w in c5h c5f; do
  OUT=gpurun_out/prof_r05/$w
  mkdir -p $OUT
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum --output-format csv \
    -d $PWD/$OUT/pmc_RDREQ -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu --e2e-steps 0 --no-verify \
    > $OUT/pmc_RDREQ.log 2>&1
done
echo "profile r05 done"
