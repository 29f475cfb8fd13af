#!/usr/bin/env python3
"""Turn a tools/gpu_round.sh run (gpurun_out/round_<wl>/) into the committed
evidence under profiles/: the rocprofv3 kernel stats, the PMC traffic that
bench.py reports as roofline.traffic (merged into profiles/pmc_traffic.json
under bench.py's key), and a short summary.

  python tools/make_profiles.py <tag> <workload>     e.g.  r01 sift

HBM bytes follow MI355X_MICROARCH.md sec.HBM: FETCH_SIZE and WRITE_SIZE
are KiB; on gfx950 FETCH_SIZE counts half the bytes of wide streaming reads,
so it is doubled.  Counters were collected one group per run with
--kernel-trace only.
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAG = sys.argv[1] if len(sys.argv) > 1 else "r01"
WL = sys.argv[2] if len(sys.argv) > 2 else "mnist"
SRC = os.path.join(ROOT, "gpurun_out", "round_" + WL)
DST = os.path.join(ROOT, "profiles")


def counters(name):
    fs = glob.glob(os.path.join(SRC, name, "**", "*counter_collection.csv"), recursive=True)
    out = {}
    for f in fs:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            out.setdefault(k, {}).setdefault(r["Counter_Name"], 0.0)
            out[k][r["Counter_Name"]] += float(r["Counter_Value"])
    return out


def main():
    os.makedirs(DST, exist_ok=True)
    stats = glob.glob(os.path.join(SRC, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(DST, "%s_%s_kernel_stats.csv" % (TAG, WL)))
    fetch, write, mfma = counters("fetch"), counters("write"), counters("mfma")
    bench = json.loads(open(os.path.join(SRC, "bench.json")).read().strip().splitlines()[-1])
    m, n = bench["config"]["m"], bench["config"]["n"]
    dt = bench["dtype"]
    es = 8.0 if dt == "f64" else 4.0
    tpath = os.path.join(DST, "pmc_traffic.json")
    traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
    lines = []
    for k in sorted(set(fetch) | set(write)):
        fb = fetch.get(k, {}).get("FETCH_SIZE", 0.0) * 1024 * 2
        wb = write.get(k, {}).get("WRITE_SIZE", 0.0) * 1024
        lines.append("| %s | %.3g | %.3g |" % (k, fb, wb))
        if k.startswith("k_dist_topk"):
            traffic["m%d_n%d_p1" % (m, n) + ("" if dt == "f64" else "_" + dt)] = {
                "kernel": k, "fetch_bytes": fb, "write_bytes": wb,
                "hbm_bytes_per_launch": fb + wb,
                "algorithmic_bytes_per_launch": m * n * es,
                "note": "FETCH_SIZE x2 (gfx950) + WRITE_SIZE, KiB->B, one launch = one full all-kNN"}
    json.dump(traffic, open(tpath, "w"), indent=1)
    dist = [v for k, v in mfma.items() if k.startswith("k_dist_topk")]
    md = ["# %s profile summary: %s (%dx%d %s, k=%d, 1x MI355X)"
          % (TAG, WL, m, n, dt, bench["config"]["k"]), "",
          "Source: `WL=%s tools/gpu_round.sh` -> `tools/make_profiles.py %s %s`." % (WL, TAG, WL), "",
          "## bench.py line", "", "```json", json.dumps(bench), "```", "",
          "## PMC traffic per launch (bytes)", "", "| kernel | fetch (x2) | write |", "|---|---|---|"]
    md += lines
    if dist:
        d = dist[0]
        clk = d.get("GRBM_GUI_ACTIVE", 0) / 8.0
        md += ["", "## k_dist_topk utilisation", "",
               "- GRBM_GUI_ACTIVE/8 = %.4g cycles per XCD" % clk,
               "- SQ_VALU_MFMA_BUSY_CYCLES = %.4g (/(1024 SIMDs x GRBM/8) = %.1f%% MFMA busy)"
               % (d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0),
                  100.0 * d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * clk) if clk else 0),
               "- SQ_WAIT_ANY / SQ_WAVE_CYCLES = %.1f%%"
               % (100.0 * d.get("SQ_WAIT_ANY", 0) / max(d.get("SQ_WAVE_CYCLES", 1), 1))]
    open(os.path.join(DST, "%s_%s_summary.md" % (TAG, WL)), "w").write("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main()
