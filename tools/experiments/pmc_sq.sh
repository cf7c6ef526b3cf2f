#!/bin/bash
# SQ stall counters of the C3 bench kernels (one pass of 8 SQ counters). ON the GPU box.
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/sq_${1:-run}; rm -rf $OUT; mkdir -p $OUT
CTRS=${CTRS:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM}
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $PWD/$OUT/p -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-verify > $OUT/log 2>&1
python3 - $OUT <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/p/**/*_counter_collection.csv", recursive=True)[0]
v = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:34]
    v[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in v.items():
    a = {c: sum(x) / len(x) for c, x in d.items()}
    wc = a.get("SQ_WAVE_CYCLES", 1) or 1
    if "SQ_WAVE_CYCLES" not in a: wc = 1
    print(f"{k:34s} " + " ".join(f"{c.replace('SQ_','')}={a[c]/wc:.4g}" for c in sorted(a) if c != "SQ_WAVE_CYCLES") + f" wave_cyc={wc:.3g}")
PY
