#!/usr/bin/env python3
"""Turn a `tools/gpu.sh bench:WL trace:WL pmc:WL:REP` session (files under
gpurun_out/) into the committed evidence under profiles/: the rocprofv3
kernel stats, the PMC traffic of the dominant kernel that bench.py reports
as roofline.traffic (median of the REP passes, merged into
profiles/pmc_traffic.json under bench.py's key) and a short summary.

  python tools/make_profiles.py <tag> <workload>     e.g.  r02 mnist

HBM bytes follow MI355X_MICROARCH.md sec.HBM: FETCH_SIZE and WRITE_SIZE are
KiB; on gfx950 FETCH_SIZE counts half the bytes of wide streaming reads, so
it is doubled.  Each counter group ran in its own process with
--kernel-trace only (one bench step, one launch of the distance kernel).
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAG = sys.argv[1] if len(sys.argv) > 1 else "r02"
WL = sys.argv[2] if len(sys.argv) > 2 else "mnist"
OUT = os.path.join(ROOT, "gpurun_out")
DST = os.path.join(ROOT, "profiles")


def per_launch(pass_dir):
    """{kernel: {counter: value per dispatch}} of one PMC pass."""
    fs = glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True)
    tot, disp = {}, {}
    for f in fs:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            tot.setdefault(k, {}).setdefault(r["Counter_Name"], 0.0)
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp.setdefault(k, set()).add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in cs.items()} for k, cs in tot.items()}


DIST_KERNELS = ("k_dist_topk", "k_dist_split")
# the source each distance kernel is built from: the PMC record carries its
# sha1, and bench.py reports the traffic only while the source is unchanged
KERNEL_SOURCES = (("k_dist_topk_i8", "mpi-knn_amd/csrc/knn_i8.hip"),
                  ("k_dist_split", "mpi-knn_amd/csrc/knn_split.hip"),
                  ("k_dist_topk", "mpi-knn_amd/csrc/knn_kernels.hip"))


def kernel_source(kname):
    for pre, path in KERNEL_SOURCES:
        if kname and kname.startswith(pre):
            return path
    return None


def sha1_of(path):
    import hashlib
    return hashlib.sha1(open(os.path.join(ROOT, path), "rb").read()).hexdigest()


def dominant(d):
    """the distance kernel with the most dispatches' worth of counters (the
    search's own instantiation, not the int8 re-search's)"""
    ks = [k for k in d if k.startswith(DIST_KERNELS)]
    return ks[0] if ks else None


def steady(trace_dir, bench_line):
    """The traced bench run's distance-kernel launches after its warm-up
    steps (rocprofv3 kernel_trace.csv), against the HIP-event kernel time the
    same process reported (roofline.avg_launch_ms): the roofline fraction
    recomputed from the committed trace, and the step time it sits under."""
    fs = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    if not fs or bench_line is None:
        return None
    rows = []
    for f in fs:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if k.startswith(DIST_KERNELS):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    if not rows:
        return None
    # the search's own instantiation (the int8 re-search of uncertified
    # queries launches a 65-entry-list one beside it)
    tot = {}
    for b, e, k in rows:
        tot[k] = tot.get(k, 0) + (e - b)
    main_k = max(tot, key=tot.get)   # the most time: the search's own launches
    rows = sorted(r for r in rows if r[2] == main_k)
    ro = bench_line["roofline"]
    steps, warm, prof = bench_line["steps"], bench_line["warmup"], ro["profiled_steps"]
    per_step = max(1, len(rows) // (warm + steps + prof))
    keep = rows[warm * per_step:]              # timed + profiled steps
    durs = [(e - b) * 1e-6 for b, e, _ in keep]
    cfg = bench_line["config"]
    flop = 2.0 * cfg["m"] * cfg["m"] * cfg["n"]
    avg = statistics.mean(durs)
    return {"kernel": keep[0][2], "launches_all": len(rows), "launches_steady": len(keep),
            "warmup_steps_skipped": warm, "rocprof_steady_avg_ms": avg, "rocprof_steady_min_ms": min(durs),
            "rocprof_steady_max_ms": max(durs),
            "rocprof_all_avg_ms": statistics.mean([(e - b) * 1e-6 for b, e, _ in rows]),
            "hip_event_avg_launch_ms": ro["avg_launch_ms"], "ms_per_step": bench_line["ms_per_step"],
            "frac_hip_events": ro["frac"], "peak_tops": ro["peak"],
            "frac_rocprof_steady": flop / (avg * 1e-3) / 1e12 / ro["peak"],
            "note": "one process: bench.py --steps %d --warmup %d under rocprofv3 --kernel-trace; the "
                    "first %d steps' launches dropped" % (steps, warm, warm)}


def main():
    os.makedirs(DST, exist_ok=True)
    stats = glob.glob(os.path.join(OUT, "trace_" + WL, "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(DST, "%s_%s_kernel_stats.csv" % (TAG, WL)))
    tl = os.path.join(OUT, "trace_%s.log" % WL)
    tline = None
    if os.path.exists(tl):
        ls = [l for l in open(tl) if l.startswith("{")]
        tline = json.loads(ls[-1]) if ls else None
    st = steady(os.path.join(OUT, "trace_" + WL), tline)
    if st:
        json.dump(st, open(os.path.join(DST, "%s_%s_roofline.json" % (TAG, WL)), "w"), indent=1)
    bench = [l for l in open(os.path.join(OUT, "bench_%s.log" % WL)) if l.startswith("{")][-1]
    bench = json.loads(bench)
    m, n, dt = bench["config"]["m"], bench["config"]["n"], bench["dtype"]
    pdir = os.path.join(OUT, "pmc_" + WL)
    fetch, write, busy, kname = [], [], [], None
    for d in sorted([x for x in glob.glob(os.path.join(pdir, "fetch_size_*")) if os.path.isdir(x)]):
        c = per_launch(d)
        kname = dominant(c) or kname
        if kname:
            fetch.append(c[kname]["FETCH_SIZE"] * 1024 * 2)
    for d in sorted([x for x in glob.glob(os.path.join(pdir, "write_size_*")) if os.path.isdir(x)]):
        c = per_launch(d)
        k = dominant(c)
        if k:
            write.append(c[k]["WRITE_SIZE"] * 1024)
    for d in sorted([x for x in glob.glob(os.path.join(pdir, "sq_valu_mfma_busy_cycles_*")) if os.path.isdir(x)]):
        c = per_launch(d)
        k = dominant(c)
        if k:
            clk = c[k].get("GRBM_GUI_ACTIVE", 0) / 8.0      # per XCD
            busy.append({"mfma_busy": c[k]["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * clk) if clk else None,
                         "wait_any": c[k].get("SQ_WAIT_ANY", 0) / max(c[k].get("SQ_WAVE_CYCLES", 1), 1)})
    es = 8.0 if dt == "f64" else 4.0
    tpath = os.path.join(DST, "pmc_traffic.json")
    traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
    key = "m%d_n%d_p1" % (m, n) + ("" if dt == "f64" else "_" + dt)
    if WL == "mnist-real":
        key += "_real"
    rec = None
    if fetch and write:
        f, w = statistics.median(fetch), statistics.median(write)
        src = kernel_source(kname)
        rec = {"kernel": kname, "source": src, "source_sha1": sha1_of(src) if src else None,
               "profile": "profiles/%s_%s_summary.md" % (TAG, WL),
               "fetch_bytes": f, "write_bytes": w, "hbm_bytes_per_launch": f + w,
               "samples_fetch_bytes": fetch, "samples_write_bytes": write,
               "algorithmic_bytes_per_launch": m * n * es,
               "note": "median of %d passes; FETCH_SIZE x2 (gfx950) + WRITE_SIZE, KiB->B, one launch = "
                       "one full all-kNN (%s %s)" % (len(fetch), TAG, WL)}
        traffic[key] = rec
        json.dump(traffic, open(tpath, "w"), indent=1)
    md = ["# %s profile summary: %s (%dx%d %s, k=%d, 1x MI355X)" % (TAG, WL, m, n, dt, bench["config"]["k"]),
          "", "Source: `tools/gpu.sh bench:%s trace:%s pmc:%s:%d` -> `tools/make_profiles.py %s %s`."
          % (WL, WL, WL, len(fetch), TAG, WL), "", "## bench.py line", "", "```json", json.dumps(bench), "```", ""]
    if rec:
        md += ["## PMC traffic of %s per launch (bytes, median of %d passes)" % (kname, len(fetch)), "",
               "| | median | min | max |", "|---|---|---|---|",
               "| FETCH_SIZE x2 | %.4g | %.4g | %.4g |" % (rec["fetch_bytes"], min(fetch), max(fetch)),
               "| WRITE_SIZE | %.4g | %.4g | %.4g |" % (rec["write_bytes"], min(write), max(write)),
               "| algorithmic (corpus bytes) | %.4g | | |" % rec["algorithmic_bytes_per_launch"], ""]
    if st:
        md += ["## Roofline from the committed trace (%s_%s_roofline.json)" % (TAG, WL), "",
               "| | ms | fraction of the %g TOPS peak |" % st["peak_tops"], "|---|---|---|",
               "| rocprofv3, steady launches (%d, after %d warm-up steps) | %.4f | %.4f |"
               % (st["launches_steady"], st["warmup_steps_skipped"], st["rocprof_steady_avg_ms"],
                  st["frac_rocprof_steady"]),
               "| HIP events, same process (bench.py roofline) | %.4f | %.4f |"
               % (st["hip_event_avg_launch_ms"], st["frac_hip_events"]),
               "| rocprofv3, every launch incl. warm-up | %.4f | |" % st["rocprof_all_avg_ms"],
               "| bench step (ms_per_step, same process) | %.4f | |" % st["ms_per_step"], ""]
    if busy:
        mb = [b["mfma_busy"] for b in busy if b["mfma_busy"] is not None]
        wa = [b["wait_any"] for b in busy]
        md += ["## %s utilisation (%d passes)" % (kname, len(busy)), "",
               "- MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE/8): median %.1f%% "
               "(%.1f..%.1f)" % (100 * statistics.median(mb), 100 * min(mb), 100 * max(mb)),
               "- SQ_WAIT_ANY / SQ_WAVE_CYCLES: median %.1f%%" % (100 * statistics.median(wa))]
    open(os.path.join(DST, "%s_%s_summary.md" % (TAG, WL)), "w").write("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main()
