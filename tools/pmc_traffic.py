"""Fold rocprofv3 PMC passes into profiles/pmc_traffic.json (HBM bytes per launch per kernel).

Each counter comes from its own `rocprofv3 --kernel-trace --pmc <C>` pass (MI355X_MICROARCH.md
"rocprofv3 PMC slots": FETCH_SIZE and WRITE_SIZE do not fit one pass). Units are KiB. gfx950
correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of wide coalesced reads,
so reads are counted as 2 * FETCH_SIZE; WRITE_SIZE is taken as is. Other access widths (the
walker's random 16-B probes, 8-B CAS) are uncalibrated: the raw counters are kept beside.

  python tools/pmc_traffic.py <workload> <n> <pmc_dir_prefix> [out.json]
  e.g. python tools/pmc_traffic.py c3 200000000 gpurun_out/pmc_
"""
import csv
import glob
import json
import os
import sys

KERNELS = {"k_insert": "k_insert<", "k_walk": "k_walk<", "k_part1_convert": "k_part1_convert<",
           "k_part1_scatter": "k_part1_scatter<", "k_part2_hist": "k_part2_hist<",
           "k_part2_scatter": "k_part2_scatter<", "k_part_build": "k_part_build<",
           "k_insert_overflow": "k_insert_overflow<"}
PIPELINE = ["k_part1_convert", "k_part1_scatter", "k_part2_hist", "k_part2_scatter", "k_part_build",
            "k_insert_overflow"]


def per_kernel(counter, prefix):
    files = glob.glob(f"{prefix}{counter}/**/*_counter_collection.csv", recursive=True)
    if not files:
        return {}
    vals = {}
    for r in csv.DictReader(open(files[0])):
        for short, pat in KERNELS.items():
            if pat in r["Kernel_Name"]:
                vals.setdefault(short, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    workload, n, prefix = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    fetch = per_kernel("FETCH_SIZE", prefix)
    write = per_kernel("WRITE_SIZE", prefix)
    atom = per_kernel("TCC_EA0_ATOMIC_sum", prefix)
    try:
        doc = json.load(open(out))
    except (OSError, ValueError):
        doc = {}
    e = {"n": n, "unit": "bytes per launch",
         "formula": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH half-count correction)",
         "raw_kib": {"FETCH_SIZE": fetch, "WRITE_SIZE": write}, "atomics": atom}
    for k in KERNELS:
        if k in fetch and k in write:
            e[k] = 2 * fetch[k] * 1024 + write[k] * 1024
    if all(k in e for k in PIPELINE):
        e["insert_pipeline"] = sum(e[k] for k in PIPELINE)
    doc[workload] = e
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(e, indent=1))


if __name__ == "__main__":
    main()
