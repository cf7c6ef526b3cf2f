"""Per-step operation counts of a rocprofv3 kernel trace: the dispatches between consecutive launches
of a marker kernel (default: the region build, once per step), split into fill (hipMemsetAsync),
copy (hipMemcpyAsync), torch and library kernels, with the step's span on the device.

  python tools/step_ops.py <trace dir or *_kernel_trace.csv> [marker substring]

The whole trace's kernel_stats also counts the setup before the first step (input generation,
first-touch allocations): VERDICT r5 read 599 fills and 303 copies over 4 traced steps as ~150 +
~75 per step, where a step issues ~20 + ~10."""
import csv
import glob
import os
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "k_part_build"
if os.path.isdir(path):
    path = max(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True), key=os.path.getmtime)
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
print(f"{path}: {len(rows)} dispatches, {len(idx)} steps (marker '{marker}'), "
      f"{idx[0] if idx else len(rows)} dispatches before the first")
print(f"{'step':>4} {'fill':>5} {'copy':>5} {'torch':>5} {'lib':>5}  span_ms")
for s, (a, b) in enumerate(zip(idx, idx[1:] + [len(rows)])):
    c = {"fill": 0, "copy": 0, "torch": 0, "lib": 0}
    for r in rows[a:b]:
        n = r["Kernel_Name"]
        c["fill" if "fillBuffer" in n else "copy" if "copyBuffer" in n else "torch" if "at::native" in n else "lib"] += 1
    span = (max(int(r["End_Timestamp"]) for r in rows[a:b]) - int(rows[a]["Start_Timestamp"])) / 1e6
    print(f"{s:>4} {c['fill']:>5} {c['copy']:>5} {c['torch']:>5} {c['lib']:>5}  {span:8.2f}")
