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

KERNELS = {"k_insert": ("k_insert<",), "k_walk": ("k_walk<", "k_walk_g<", "k_walk_q<", "k_rec_succ<"),
           "k_win1": ("k_win1<",), "k_win1_rec": ("k_win1_rec<",), "k_win2": ("k_win2<",),
           "k_part1_convert": ("k_part1_convert<",), "k_part1_fused": ("k_part1_fused<",),
           "k_part1_scatter": ("k_part1_scatter<",), "k_part2_hist": ("k_part2_hist<",),
           "k_part2_scatter": ("k_part2_scatter<",), "k_part2_res": ("k_part2_res<",),
           "k_part_build": ("k_part_build<", "k_part_build_pf<"), "k_insert_overflow": ("k_insert_overflow<",),
           "k_route_own": ("k_route_own",), "k_route_scatter": ("k_route_scatter",), "k_mw_run": ("k_mw_run",),
           "k_ovf_scatter": ("k_ovf_scatter<",),
           "membench_gather16": ("k_gather16",), "membench_chase16": ("k_chase16",),
           "membench_chase64q": ("k_chasegILi4",), "membench_chase128o": ("k_chasegILi8",)}
# kernels of the insert pipeline (whichever of them ran)
PIPELINE = ["k_part1_convert", "k_part1_fused", "k_win1", "k_win1_rec", "k_part1_scatter", "k_part2_hist", "k_part2_scatter",
            "k_part2_res", "k_win2", "k_ovf_scatter", "k_part_build", "k_insert_overflow", "k_route_own", "k_route_scatter"]
# random-access kernels: FETCH_SIZE is NOT doubled (the 1/2 correction is for wide coalesced
# streaming reads); their requests are calibrated against tools/membench (random 16-B loads)
RANDOM = {"k_walk", "k_insert", "k_insert_overflow", "k_mw_run", "membench_gather16", "membench_chase16",
          "membench_chase64q", "membench_chase128o"}


def per_kernel(counter, prefix):
    files = glob.glob(f"{prefix}{counter}/**/*_counter_collection.csv", recursive=True)
    if not files:
        return {}
    vals = {}
    for r in csv.DictReader(open(files[0])):
        for short, pats in KERNELS.items():
            if any(pat in r["Kernel_Name"] for pat in pats):
                vals.setdefault((short, r.get("Counter_Name", counter)), []).append(float(r["Counter_Value"]))
    out = {}
    for (k, c), v in vals.items():
        out.setdefault(c, {})[k] = sum(v) / len(v)
    return out[counter] if counter in out else out


def main():
    workload, n, prefix = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    fetch = per_kernel("FETCH_SIZE", prefix)
    write = per_kernel("WRITE_SIZE", prefix)
    atom = per_kernel("TCC_EA0_ATOMIC_sum", prefix)
    req = per_kernel("RDREQ", prefix)  # pass with TCC_EA0_RDREQ_sum, _32B_sum, TCC_BUBBLE_sum
    try:
        doc = json.load(open(out))
    except (OSError, ValueError):
        doc = {}
    e = {"n": n, "unit": "bytes per launch",
         "formula": "streaming kernels: 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH half-count correction, "
                    "MI355X_MICROARCH.md HBM); random-access kernels: FETCH_SIZE + WRITE_SIZE (64-B "
                    "read requests, calibrated with tools/membench, see 'requests')",
         "raw_kib": {"FETCH_SIZE": fetch, "WRITE_SIZE": write}, "atomics": atom, "requests": req}
    for k in KERNELS:
        if k in fetch and k in write:
            f = 1 if k in RANDOM else 2
            e[k] = f * fetch[k] * 1024 + write[k] * 1024
    ran = [k for k in PIPELINE if k in e]
    if ran:
        e["insert_pipeline"] = sum(e[k] for k in ran)
        e["insert_pipeline_kernels"] = ran
    doc[workload] = e
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(e, indent=1))


if __name__ == "__main__":
    main()
