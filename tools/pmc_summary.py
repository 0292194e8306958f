"""Summarise rocprofv3 runs of bench.py into profiles/ (committed, cited by bench.py / DESIGN.md).

    python tools/pmc_summary.py --round r01 [--src gpurun_out]

Reads  <src>/prof/run_kernel_stats.csv            (rocprofv3 --kernel-trace --stats)
       <src>/pmc_fetch/run_counter_collection.csv  (rocprofv3 --pmc FETCH_SIZE)
       <src>/pmc_write/run_counter_collection.csv  (rocprofv3 --pmc WRITE_SIZE)
       <src>/prof/run_kernel_trace.csv            (per-dispatch durations)
Writes profiles/<round>_kernel_stats.csv (copy) and profiles/<round>_pmc_traffic.json:
per kernel the mean FETCH_SIZE / WRITE_SIZE per dispatch (KiB) and the corrected HBM bytes
per launch, following MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of the bytes of a wide
coalesced streaming read on gfx950 -> x2; WRITE_SIZE is exact for 16-B/lane stores.  Values
are per dispatch of the same command, so they compare directly with bench.py's per-launch
algorithmic bytes.  (Infinity-Cache hits are counted by these counters, not excluded.)
durations_us: per class the rocprofv3 mean over all dispatches and over the working ones
(launches past a cycle's stop column exit at entry), the latter comparable with bench.py's
live HIP-event avg_us.
"""
import argparse
import collections
import csv
import hashlib
import json
import os
import sys
import re
import shutil
import statistics

CLASSES = {   # bench/profile class -> demangled-name prefix (regex) in rocprofv3 output (default
              # path: SELL-64 layout, tridiagonal-factor BJ(8), DCGS2; fp64 or fp32 values)
    "band_step": r"void vtk::k_band_step<",
    # k_g4_ring<VT, HALO, RL, MODE, GR>: MODE 0 split step, 2 with step 0's dots, 3 the
    # cycle-start residual; k_lsv_ring_epi<EPI>: 3 residual + BJ, 4 step 0 with its dots
    "spmv_bj_dc": r"void vtk::k_(sell<(double|float), false, 4, 8, true,|g4_ring<(double|float), (false|true), \d+, 2, \d+>|lsv_ring_epi<4>)",
    "spmv": r"void vtk::k_sell<(double|float), false, 0, 1, false,",
    "spmv_bj": r"void vtk::k_(sell<(double|float), false, 2, 8, true,|g4_ring<(double|float), (false|true), \d+, 0, \d+>)",
    "spmv_resid_bj": r"void vtk::k_(sell<(double|float), false, 3, 8, true,|g4_ring<(double|float), (false|true), \d+, 3, \d+>|lsv_ring_epi<3>)",
    "spmv_csr": r"void vtk::k_spmv<(double|float), false, 0, 1",
    "spmv_bj_dc_csr": r"void vtk::k_spmv<(double|float), false, 4, 8",
    "dc_dots": r"void vtk::k_dc_dots(_rows<\d+>)?\(",
    # the line path's DCGS2 step: the sweep with its dots (k_line_apply<SEG, COMPACT, true>) or,
    # one rank with canonical rows, the fused SpMV + sweep + dots (k_line_spmv_dc<SEG>, round 5)
    "line_dc": r"void vtk::k_line_(apply<\d+, (true|false), true>|spmv_dc<\d+>)",
    "line_apply": r"void vtk::k_line_apply<\d+, (true|false)(, false)?>",
    "dc_update": "void vtk::k_dc_update<",
    "dc_scalar": "vtk::k_dc_scalar(",
    "mgs": "vtk::k_mgs(",
    "tail": "vtk::k_tail(",
    "xupdate": "vtk::k_xupdate(",
    "bj_apply": "vtk::k_bj_apply",
    "scale0": "vtk::k_scale0(",
    "spmv_lsv": r"(void )?vtk::k_lsv_(spmv<|ring\()",
}


def load(path):
    """kernel name -> [(counter value, dispatch duration us)] of one --pmc pass (the counter CSV
    carries each dispatch's own start / end stamps)"""
    d = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            d[r["Kernel_Name"]].append((float(r["Counter_Value"]), dur))
    return d


def working(rows):
    """the dispatches that did the work: kernels enqueued past a cycle's stop column return at
    entry (a few us); keep those longer than 5 % of the class's longest dispatch"""
    if not rows:
        return rows
    cut = 0.05 * max(d for _, d in rows)
    return [(v, d) for v, d in rows if d > cut]


def band_j(name):
    """step index J of a band-step instantiation (k_band_step<WU, J, ...>)"""
    m = re.match(r"void vtk::k_band_step<\d+, (\d+),", name)
    return int(m.group(1)) if m else None


def trace_durations(path):
    d = collections.defaultdict(list)
    if not os.path.exists(path):
        return d
    with open(path) as f:
        for r in csv.DictReader(f):
            d[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", required=True)
    ap.add_argument("--src", default="gpurun_out")
    ap.add_argument("--note", default="")
    ap.add_argument("--tag", default="", help="file-name tag after the round (e.g. c4)")
    ap.add_argument("--prof", default="prof")
    ap.add_argument("--fetch", default="pmc_fetch")
    ap.add_argument("--write", default="pmc_write")
    ap.add_argument("--cmd", default="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --spmv-reps 5")
    ap.add_argument("--config", default="C3", help="bench config the profiled command ran (bench.py matches it)")
    ap.add_argument("--sq", default=None, help="dir of a --pmc SQ_* pass: per-kernel mean counters -> <tag>pmc_sq.json")
    ap.add_argument("--patch-bench", default=None,
                    help="bench JSON (one line) of the same call whose roofline traffic fields are refreshed "
                         "from this summary (the bench ran before the PMC passes)")
    a = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    src = os.path.join(root, a.src)
    tag = f"{a.round}_{a.tag}_" if a.tag else f"{a.round}_"
    ks = os.path.join(src, a.prof, "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(prof, f"{tag}kernel_stats.csv"))
    durations = trace_durations(os.path.join(src, a.prof, "run_kernel_trace.csv"))
    fetch = load(os.path.join(src, a.fetch, "run_counter_collection.csv"))
    write = load(os.path.join(src, a.write, "run_counter_collection.csv"))
    sys.path.insert(0, root)
    import bench   # the device sources, hashed in bench.py's KERNEL_SOURCES order
    ksha = bench.kernels_sha16()
    out = {"_how": ("rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of "
                    f"'{a.cmd}'; "
                    "hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE) * 1024 "
                    "(gfx950 FETCH_SIZE half-count correction, MI355X_MICROARCH.md §HBM), averaged over the "
                    "working dispatches (longer than 5 % of the class's longest; early-exit launches past a "
                    "cycle's stop column excluded); band_step_per_j: the same per step index J"),
           "note": a.note, "config": a.config, "kernels_sha16": ksha, "kernels": {}, "durations_us": {}}
    for cls, prefix in CLASSES.items():
        rx = re.compile(prefix if prefix.startswith("void") else re.escape(prefix))
        fk = [t for k, vs in fetch.items() if rx.match(k) for t in vs]
        wk = [t for k, vs in write.items() if rx.match(k) for t in vs]
        dur = [v for k, vs in durations.items() if rx.match(k) for v in vs]
        if dur:
            # kernels enqueued past a cycle's stop column return at entry (a few us); the
            # bench's live HIP-event average counts only the working launches
            cut = 0.05 * max(dur)
            act = [v for v in dur if v > cut]
            out["durations_us"][cls] = {"dispatches": len(dur), "mean_all": statistics.mean(dur),
                                        "working": len(act), "mean_working": statistics.mean(act),
                                        "early_exit": len(dur) - len(act)}
        if not fk:
            continue
        # averaged over the WORKING dispatches only (early-exit launches past a cycle's stop
        # column would dilute the per-launch traffic)
        fw, ww = working(fk), working(wk)
        f_kib = statistics.mean(v for v, _ in fw)
        w_kib = statistics.mean(v for v, _ in ww) if ww else 0.0
        out["kernels"][cls] = {"dispatches": len(fk), "working_dispatches": len(fw), "fetch_kib": f_kib,
                               "write_kib": w_kib, "hbm_bytes_per_launch": (2 * f_kib + w_kib) * 1024}
        if cls == "band_step":   # per step index J (the kernel is instantiated per J)
            perj = {}
            for k, vs in fetch.items():
                jj = band_j(k)
                if jj is not None and rx.match(k):
                    perj.setdefault(jj, [[], []])[0].extend(working(vs))
            for k, vs in write.items():
                jj = band_j(k)
                if jj is not None and rx.match(k):
                    perj.setdefault(jj, [[], []])[1].extend(working(vs))
            out["band_step_per_j"] = {
                str(jj): {"working_dispatches": len(f), "fetch_kib": statistics.mean(v for v, _ in f),
                          "write_kib": statistics.mean(v for v, _ in w) if w else 0.0,
                          "hbm_bytes_per_launch": (2 * statistics.mean(v for v, _ in f) +
                                                   (statistics.mean(v for v, _ in w) if w else 0.0)) * 1024,
                          "mean_duration_us_profiled": statistics.mean(d for _, d in f)}
                for jj, (f, w) in sorted(perj.items()) if f}
    if a.sq:
        rows = collections.defaultdict(lambda: collections.defaultdict(list))
        with open(os.path.join(src, a.sq, "run_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                rows[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        sq = {"_how": f"rocprofv3 --pmc SQ_* of '{a.cmd}'; mean per dispatch; wait fraction = SQ_WAIT_ANY / SQ_WAVE_CYCLES",
              "config": a.config, "kernels_sha16": ksha, "kernels": {}}
        for k, cs in rows.items():
            if not any(re.match(p if p.startswith("void") else re.escape(p), k + "(") for p in CLASSES.values()):
                continue
            m = {c: statistics.mean(v) for c, v in cs.items()}
            if m.get("SQ_WAVE_CYCLES"):
                m["wait_frac"] = m.get("SQ_WAIT_ANY", 0.0) / m["SQ_WAVE_CYCLES"]
            sq["kernels"][k] = m
        with open(os.path.join(prof, f"{tag}pmc_sq.json"), "w") as f:
            json.dump(sq, f, indent=1)
        print("wrote", os.path.join(prof, f"{tag}pmc_sq.json"))
    dst = os.path.join(prof, f"{tag}pmc_traffic.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", dst)
    if a.patch_bench:
        with open(a.patch_bench) as f:
            b = json.loads(f.readline())
        for key, cls in (("roofline", b["roofline"].get("kernel")), ("roofline_spmv", "spmv")):
            k = out["kernels"].get(cls)
            if k is not None:
                b[key]["traffic"] = k["hbm_bytes_per_launch"]
                b[key]["traffic_source"] = os.path.basename(dst)
        with open(a.patch_bench, "w") as f:
            f.write(json.dumps(b) + "\n")
        print("patched", a.patch_bench)
    for k, v in out["kernels"].items():
        print(f"  {k:12s} {v['working_dispatches']:6d} working dispatches  {v['hbm_bytes_per_launch'] / 1e6:10.1f} MB/launch")
    for jj, v in out.get("band_step_per_j", {}).items():
        print(f"  band j={jj:>2s} {v['working_dispatches']:4d} working  {v['hbm_bytes_per_launch'] / 1e6:10.1f} MB/launch")
    for k, v in out["durations_us"].items():
        print(f"  {k:12s} {v['working']:4d} working launches {v['mean_working']:9.1f} us "
              f"(all {v['dispatches']}: {v['mean_all']:.1f} us)")


if __name__ == "__main__":
    main()
