#!/usr/bin/env python3
"""Collect tools/ring_emulate.py runs (gpurun_out/emu_<workload>.log, as
written by `tools/gpu.sh emu:WL[:RANKS[:STEPS]]`) into
profiles/<tag>_ring_emulation.json.

  python tools/emu_record.py r02 "note text" [LOGDIR]

LOGDIR (default gpurun_out): where the emu_<workload>.log files are.
"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def last_json(path):
    text = open(path).read()
    start = text.rfind('\n{\n')
    if start < 0:
        start = text.find('{\n')
    return json.loads(text[start:].strip()) if start >= 0 else None


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    out = {}
    logdir = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "gpurun_out")
    for f in sorted(glob.glob(os.path.join(logdir, "emu_*.log"))):
        rec = last_json(f)
        if rec and "workload" in rec:
            out[rec["workload"]] = rec
    out["_note"] = (sys.argv[2] if len(sys.argv) > 2 else
                    "per-rank compute of a P-GPU ring emulated on one MI355X (tools/ring_emulate.py); "
                    "compute_efficiency = t(Pmin) * Pmin / (P * t(P)) within each workload's run")
    path = os.path.join(ROOT, "profiles", "%s_ring_emulation.json" % tag)
    json.dump(out, open(path, "w"), indent=1)
    for k, v in out.items():
        if k.startswith("_"):
            continue
        print(k, {p: (round(r["rank_ms"], 3), round(r["compute_efficiency"], 3)) for p, r in v["ranks"].items()})


if __name__ == "__main__":
    main()
