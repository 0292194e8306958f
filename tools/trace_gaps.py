"""Per-step kernel timeline of a rocprofv3 --kernel-trace run: for a window of Arnoldi steps in
the middle of the run, each kernel's start (relative), the idle gap before it on the device and
its duration; then the mean gap / duration per kernel class over every full step of the run.

    python tools/trace_gaps.py gpurun_out/<dir>/run_kernel_trace.csv [--window 12]
"""
import argparse
import collections
import csv
import re
import statistics


def short(name):
    n = name.split("(")[0]
    n = re.sub(r"^void ", "", n)
    return n.replace("vtk::", "")[-48:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window", type=int, default=12)
    ap.add_argument("--anchor", default="k_dc_scalar", help="kernel marking one Arnoldi step")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.anchor in r["Kernel_Name"]]
    if not idx:
        raise SystemExit(f"no {a.anchor} in the trace")
    mid = idx[len(idx) // 2]
    lo = max(0, mid - a.window // 2)
    t0 = int(rows[lo]["Start_Timestamp"])
    prev = None
    for r in rows[lo:lo + a.window]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f"{(s - t0) / 1e3:9.1f} us  gap {gap:6.1f}  dur {(e - s) / 1e3:8.1f}  {short(r['Kernel_Name'])}")
        prev = e
    gaps, durs = collections.defaultdict(list), collections.defaultdict(list)
    for i in range(1, len(rows)):
        s, e = int(rows[i]["Start_Timestamp"]), int(rows[i]["End_Timestamp"])
        g = (s - int(rows[i - 1]["End_Timestamp"])) / 1e3
        if g > 200:   # host-side pauses between solves
            continue
        k = short(rows[i]["Kernel_Name"])
        gaps[k].append(g)
        durs[k].append((e - s) / 1e3)
    print("\nclass                                             n   mean gap before   mean dur")
    for k in sorted(gaps, key=lambda k: -len(gaps[k]))[:14]:
        print(f"{k:48s} {len(gaps[k]):5d} {statistics.mean(gaps[k]):12.1f} us {statistics.mean(durs[k]):10.1f} us")


if __name__ == "__main__":
    main()
