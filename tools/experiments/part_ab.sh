#!/bin/bash
# Partitioned-build pass variants on C3 (KH_P1 x KH_P2), after their parity tests. ON the GPU box.
set -eo pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "part_pass or both_insert or golden or c3_shape or duplicate or walk_group" > gpurun_out/t_part.log 2>&1
for v in ${VARIANTS:-fused:res convert:res}; do
  KH_P1=${v%:*} KH_P2=${v#*:} timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/part_${v/:/_}.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/prof_part/trace -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/prof_part.log 2>&1
python3 tools/kstats.py gpurun_out/prof_part/trace > gpurun_out/prof_part/kernel_stats.txt
