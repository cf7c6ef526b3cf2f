"""Per-round timing of the sharded walk from a rocprofv3 kernel trace (last step's rounds)."""
import csv
import glob
import sys

import os
f = max(glob.glob(f"{sys.argv[1]}/**/*_kernel_trace.csv", recursive=True), key=os.path.getmtime)
rows = list(csv.DictReader(open(f)))
nr = int(sys.argv[2]) if len(sys.argv) > 2 else 200


def spans(pat):
    return [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if pat in r["Kernel_Name"]]


em = spans("k_rw_step_fixed")[-nr:]
for pat in ["k_rw_step_fixed", "k_find_ext_fixed", "rcclGenericKernel"]:
    sp = spans(pat)
    sp = [x for x in sp if x[0] >= em[0][0]]
    d = [(e - s) / 1e3 for s, e in sp]
    print(f"{pat:20s} n={len(d)} first={d[:3]} mid={d[len(d)//2:len(d)//2+3]} last={d[-3:]}")
print("round wall us", [round((em[i + 1][0] - em[i][0]) / 1e3, 1) for i in range(0, len(em) - 1, 20)])
allk = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
t0, t1 = em[0][0], em[-1][1]
busy = sum(min(e, t1) - max(s, t0) for s, e in allk if e > t0 and s < t1)
print("walk span ms", (t1 - t0) / 1e6, "gpu busy ms", busy / 1e6)
