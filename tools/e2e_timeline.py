"""Timeline of the last reference-boundary step (bench.py end_to_end) from a rocprofv3
--kernel-trace --memory-copy-trace CSV directory: every copy and kernel from the first record
upload of that step to the end of its text download, with the idle gaps of the device between.
  python tools/e2e_timeline.py <rocprofv3 -d dir> [min_copy_ms]
"""
import csv
import glob
import os
import sys


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main():
    d = sys.argv[1]
    min_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    ev = []
    for r in rows(d, "*kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:70], 0))
    for r in rows(d, "*memory_copy_trace.csv"):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        ev.append((s, e, "C", r.get("Direction", "?"), e - s))  # no byte count in the CSV: duration
    ev.sort()
    # the last step: the last group of >= 4 record uploads (chunked kh_insert) (H2D copies of >= min_ms) -> the D2H after them
    h2d = [e for e in ev if e[2] == "C" and "HOST_TO_DEVICE" in e[3].upper() and e[4] >= min_ms * 1e6]
    if not h2d:
        print("no uploads found")
        return
    # a step ends with a text download (D2H of >= min_ms); its uploads are those since the
    # previous download: take the last step with >= 4 uploads (the chunked kh_insert)
    d2h_all = [e for e in ev if e[2] == "C" and "DEVICE_TO_HOST" in e[3].upper() and e[4] >= min_ms * 1e6]
    g, d2h, prev = None, None, 0
    for d in d2h_all:
        ups = [e for e in h2d if prev <= e[0] < d[0]]
        if len(ups) >= 4:
            g, d2h = ups, [d]
        prev = d[1]
    if g is None:
        print("no chunked step found")
        return
    t0 = g[0][0]
    t1 = d2h[0][1] if d2h else ev[-1][1]
    up_end = g[-1][1]
    sel = [e for e in ev if t0 <= e[0] <= t1]
    busy_end = t0
    idle_after_upload = 0
    print(f"step: first upload at 0, uploads end at {(up_end - t0) / 1e6:.3f} ms, text D2H ends at {(t1 - t0) / 1e6:.3f} ms")
    for s, e, kind, name, nb in sel:
        if kind == "K" and s < up_end:
            continue  # kernels under the upload: summarised below
        if s > busy_end and s > up_end:
            idle_after_upload += s - max(busy_end, up_end)
        print(f"{(s - t0) / 1e6:9.3f} {(e - s) / 1e6:8.3f}  {kind} {name} ")
        busy_end = max(busy_end, e)
    k_under = sum(e - s for s, e, kind, *_ in sel if kind == "K" and s < up_end)
    print(f"kernel time under the upload: {k_under / 1e6:.3f} ms; device idle after the upload: {idle_after_upload / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
