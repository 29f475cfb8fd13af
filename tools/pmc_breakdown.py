#!/usr/bin/env python3
"""Per-dispatch PMC values of the distance and merge kernels in one rocprofv3 --pmc
pass (tools/gpu.sh pmcx:WL:GROUP), with the derived ratios the kernel work
is read by: instructions per wave, cycle buckets per wave-cycle, MFMA busy.

  python tools/pmc_breakdown.py gpurun_out/pmcx_mnist/inst [more dirs ...]
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            key = (k, r["Dispatch_Id"])
            out.setdefault(key, {}).setdefault(r["Counter_Name"], 0.0)
            out[key][r["Counter_Name"]] += float(r["Counter_Value"])
    return out


def main():
    res = {}
    for d in sys.argv[1:]:
        for (k, disp), cs in sorted(per_dispatch(d).items()):
            if not k.startswith(("k_dist_topk", "k_dist_split", "k_merge")):
                continue
            rec = dict(cs)
            w = cs.get("SQ_WAVES")
            if w:
                for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU",
                          "SQ_INSTS_VMEM", "SQ_INSTS_BRANCH", "SQ_INSTS_SMEM"):
                    if c in cs:
                        rec[c + "_per_wave"] = cs[c] / w
            wc = cs.get("SQ_WAVE_CYCLES")
            if wc:
                for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                          "SQ_ACTIVE_INST_LDS"):
                    if c in cs:
                        rec[c + "_frac"] = cs[c] / wc
            clk = cs.get("GRBM_GUI_ACTIVE", 0) / 8.0
            if clk and "SQ_VALU_MFMA_BUSY_CYCLES" in cs:
                rec["mfma_busy"] = cs["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * clk)
            if clk and "SQ_VALU_MFMA_COEXEC_CYCLES" in cs:
                rec["coexec"] = cs["SQ_VALU_MFMA_COEXEC_CYCLES"] / (1024 * clk)
            res["%s %s #%s" % (os.path.basename(d.rstrip("/")), k, disp)] = rec
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
