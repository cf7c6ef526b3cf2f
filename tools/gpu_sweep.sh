#!/bin/bash
# Bench sweep of the committed tree (ON the GPU box): every workload line, verified, into
# gpurun_out/sweep/ (copied to profiles/rNN/bench_sweep afterwards)
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/sweep
mkdir -p $O
B="--steps 5 --warmup 2 --e2e-steps 0"
( while true; do sleep 50; date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > $O/bench_c3.json.log 2>&1
timeout -k 10 300 python bench.py $B --no-cpu --load 0.85 > $O/bench_c3_l085.json.log 2>&1
timeout -k 10 300 python bench.py $B --no-cpu --workload c2 > $O/bench_c2.json.log 2>&1
timeout -k 10 300 python bench.py $B --no-cpu --workload c5 > $O/bench_c5.json.log 2>&1
timeout -k 10 300 python bench.py $B --no-cpu --workload c5h > $O/bench_c5h.json.log 2>&1
timeout -k 10 300 python bench.py $B --no-cpu --workload c5h --load 0.85 > $O/bench_c5h_l085.json.log 2>&1
timeout -k 10 300 python bench.py $B --no-cpu --workload c5f > $O/bench_c5f.json.log 2>&1
timeout -k 10 300 python bench.py $B --no-cpu --workload c5f --load 0.85 > $O/bench_c5f_l085.json.log 2>&1
KH_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 $B --no-cpu > $O/dist_c3_one_rank.json.log 2>&1
timeout -k 10 300 ./tools/kh_bench_cpp --ranks 1 --steps 5 --warmup 2 > $O/cpp_c3_one_rank.json.log 2>&1
for f in $O/*.log; do grep -h '^{' $f | tail -1 > ${f%.log}; done
echo sweep done
