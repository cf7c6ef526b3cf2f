"""Per-kernel SQ counter averages from one rocprofv3 --pmc pass (8 SQ counters fit one pass on
gfx950), with the ratios DESIGN.md quotes:
  parked   = SQ_WAIT_ANY / SQ_WAVE_CYCLES           (waves at s_waitcnt / barrier)
  stalled  = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES      (issue stalls)
  active   = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  valu     = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES   (wave cycles issuing VALU)
  lds_bank = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra LDS cycles from bank conflicts)
  python tools/sq_summary.py <pmc dir> [kernel substrings...] > out.json"""
import csv
import glob
import json
import sys

d = sys.argv[1]
pats = sys.argv[2:] or ["k_part_build_pf", "k_part1_convert", "k_win1_rec", "k_win1<", "k_win2", "k_walk_q"]
files = glob.glob(f"{d}/**/*_counter_collection.csv", recursive=True)
acc = {}
for r in csv.DictReader(open(files[0])):
    for pat in pats:
        if pat in r["Kernel_Name"]:
            a = acc.setdefault(pat, {})
            a.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
out = {}
for k, cs in acc.items():
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    w = avg.get("SQ_WAVE_CYCLES") or 0
    lds = avg.get("SQ_LDS_IDX_ACTIVE") or 0
    avg["ratios"] = {"parked": avg.get("SQ_WAIT_ANY", 0) / w if w else None,
                     "stalled": avg.get("SQ_WAIT_INST_ANY", 0) / w if w else None,
                     "active": avg.get("SQ_ACTIVE_INST_ANY", 0) / w if w else None,
                     "valu": avg.get("SQ_ACTIVE_INST_VALU", 0) / w if w else None,
                     "lds_bank": avg.get("SQ_LDS_BANK_CONFLICT", 0) / lds if lds else None}
    out[k] = avg
print(json.dumps(out, indent=1))
