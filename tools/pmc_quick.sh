#!/bin/bash
# One PMC pass over a short bench run: tools/pmc_quick.sh <tag> "<counters>" [bench args]. ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
TAG=$1; CTRS=$2; shift 2
OUT=gpurun_out/pq_$TAG
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $PWD/$OUT/pmc -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu --e2e-steps 0 --no-verify "$@" > $OUT/pmc.log 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/pmc/**/*_counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    if any(x in k for x in ("k_walk", "k_part_build", "k_win1", "k_win2", "k_part1_convert", "k_route")):
        print(k, {c: "%.4g" % (sum(v) / len(v)) for c, v in d.items()})
PY
