#!/usr/bin/env python3
"""Summarise tools/pmc_sweep.sh output: median per-dispatch value of every counter for the
fwd-bwd kernel. Usage: python tools/pmc_table.py gpurun_out/pmc_<tag>"""
import csv
import glob
import statistics
import sys
from collections import defaultdict

vals = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    per = defaultdict(float)
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if "k_fwd_bwd" not in (r.get("Kernel_Name") or ""):
                continue
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (_, c), v in per.items():
        vals[c].append(v)
for c in sorted(vals):
    print(f"{c:32s} {statistics.median(vals[c]):16.0f}  (n={len(vals[c])})")
