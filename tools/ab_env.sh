#!/bin/bash
# A/B environment settings on the C3 bench: tools/ab_env.sh <tag> "<ENV=.. ENV=..>" ... (ON the GPU box).
# One bench per setting (7 steps); prints ms/step and phase times.
set -eo pipefail
TAG=$1; shift
mkdir -p gpurun_out/ab_$TAG
i=0
for e in "$@"; do
  env $e timeout -k 10 200 python bench.py --steps 7 --warmup 2 --no-cpu --e2e-steps 0 ${AB_ARGS:-} > gpurun_out/ab_$TAG/b$i.log 2>&1
  python3 - "$e" gpurun_out/ab_$TAG/b$i.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:40s} {d['ms_per_step']:.3f} ms", {k: round(v, 3) for k, v in d['phases_ms'].items()}, d['verified_vs_truth'])
PY
  i=$((i+1))
done
