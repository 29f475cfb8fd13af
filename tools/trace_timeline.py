#!/usr/bin/env python3
"""Print the kernel timeline of the last search pass in a rocprofv3
kernel-trace CSV (diagnostic: overlap of k_dist_topk / k_merge steps)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
fin = [i for i, r in enumerate(rows) if "k_finalize" in r["Kernel_Name"]]
lo, hi = fin[-2] + 1, fin[-1] + 1
t0 = int(rows[lo]["Start_Timestamp"])
busy = 0
for r in rows[lo:hi]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    print("%-34s %9.1f %9.1f %8.1f" % (r["Kernel_Name"][:34], s, e, e - s))
