"""One line per bench log: ms/step, phases, verification, skew counters (gpurun_out/*.log)."""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            c = d.get("config", {})
            ph = {k: round(v, 3) for k, v in (d.get("phases_ms") or {}).items()}
            print(f, round(d["ms_per_step"], 3), ph, "ok" if d.get("verified_vs_truth") else "NOT VERIFIED",
                  {k: c[k] for k in ("hot_regions", "spread_regions", "overflow_cas_keys", "walk_rounds") if k in c})
