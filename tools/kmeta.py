"""Register / spill / LDS metadata of kernels in a hipcc --save-temps gfx950 .s file:
  python tools/kmeta.py <file.s> [name substring ...]"""
import re
import sys

txt = open(sys.argv[1]).read()
pats = sys.argv[2:]
meta = txt[txt.find("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name or (pats and not any(p in name.group(1) for p in pats)):
        continue
    f = {k: (re.search(r"\." + k + r":\s+(\d+)", blk) or [None, "?"])[1]
         for k in ("vgpr_count", "vgpr_spill_count", "sgpr_count", "sgpr_spill_count", "group_segment_fixed_size",
                   "private_segment_fixed_size")}
    print(name.group(1)[:90], f)
