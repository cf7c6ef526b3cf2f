#!/bin/bash
# A/B on C5H twice (KH_LIB .ab/prev = before the LDS-aggregated sample counts), then walker blocks
# per CU 4 / 5 vs 3 on C3 / C5 / C5H. ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ab() {  # ab <workload> <lib>...
  local w=$1; shift
  for L in default "$@"; do
    if [ "$L" = default ]; then unset KH_LIB; else export KH_LIB=$PWD/$L; fi
    timeout -k 10 200 python bench.py --workload $w --steps 7 --warmup 2 --no-cpu --e2e-steps 0 --no-verify > gpurun_out/ab_one.log 2>&1
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/ab_one.log') if l.startswith('{')][0])
print('$w $L', round(d['ms_per_step'],3), [round(x,2) for x in d['step_ms']], {k: round(v,3) for k,v in d['phases_ms'].items()})" >> gpurun_out/ab_c5h.txt
  done
}
ab c5h .ab/prev/libkmerhash_amd.so
ab c5h .ab/prev/libkmerhash_amd.so
for w in c3 c5 c5h; do ab $w .ab/bpc4/libkmerhash_amd.so .ab/bpc5/libkmerhash_amd.so; done
