#!/bin/bash
# Iteration loop on the GPU box: selected parity tests, kernel trace of the C3 bench, forced 1-rank
# sharded bench (+ its trace). TESTK selects tests.
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread -k "${TESTK:-part_pass or both_insert or golden or c3_shape or duplicate or walk_group or dist}" > gpurun_out/t_iter.log 2>&1
VARIANTS="${VARIANTS:-def:KH_DUMMY=1}" bash tools/prof_variants.sh
bash tools/profile_dist1.sh dist1
