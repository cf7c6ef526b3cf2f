"""Per-kernel VGPR / scratch / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage.
usage: python tools/kres.py <file.hip> [substring...]"""
import re
import subprocess
import sys

src = sys.argv[1]
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src,
                      "-Rpass-analysis=kernel-resource-usage", "-o", "/tmp/kres.o"],
                     capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
subs = sys.argv[2:]
for f, d in rows.items():
    if subs and not any(s in f for s in subs):
        continue
    print(f"{f[:70]:70s} vgpr={d.get('VGPRs')} agpr={d.get('AGPRs')} scratch={d.get('ScratchSize [bytes/lane]')} "
          f"occ={d.get('Occupancy [waves/SIMD]')} sgpr={d.get('SGPRs')}")
