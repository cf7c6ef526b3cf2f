#!/bin/bash
# A/B of variant libraries (KH_LIB) on the bench: tools/ab_libs.sh <lib.so>... (ON the GPU box)
# AB_ARGS: extra bench args (e.g. "--workload c5"); default workload C3.
set -e
mkdir -p gpurun_out
for L in default "$@"; do
  if [ "$L" = default ]; then unset KH_LIB; else export KH_LIB=$PWD/$L; fi
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --e2e-steps 0 --no-verify ${AB_ARGS:-} > gpurun_out/ab_$(basename $L).log 2>&1
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/ab_$(basename $L).log') if l.startswith('{')][0])
print('$L ${AB_ARGS:-}', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms'].items()})"
done
