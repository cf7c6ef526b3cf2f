"""One line per bench.py JSON log: step time, rate, phase times, hot regions, CAS overflow, check.
  python tools/bench_summary.py gpurun_out/bench_*.log"""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        c, p = d["config"], d.get("phases_ms", {})
        print(f"{path.split('/')[-1]:28s} {d['ms_per_step']:8.2f} ms {d['value'] / 1e9:7.2f} G/s "
              f"ins {p.get('k_insert', 0):6.2f} build {p.get('build', 0):6.2f} walk {p.get('walk_kernel', 0):6.2f} "
              f"mat {p.get('materialize', 0):5.2f} hot {c.get('hot_regions')} ovf {c.get('overflow_cas_keys')} "
              f"load {c.get('load_factor')} ok {d.get('verified_vs_truth')}")
