#!/usr/bin/env python3
"""Summarise tools/profile_long.sh output: per-call time and HBM traffic of the long-form
fwd-bwd (configs[4]: the segmented kernel's two phase launches + the loss-sum pass) against the
algorithmic 16 B/cell (B*T*U*16 = 819.2 MB). FETCH_SIZE doubled (gfx950 wide-read correction,
MI355X_MICROARCH.md "HBM"), WRITE_SIZE as is, both in KiB."""
import csv
import glob
import json
import shutil
import statistics
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KEYS = ("k_fwd_bwd", "k_loss_sum")
ALGO = 64 * 2000 * 400 * 16


def rows(pattern):
    out = []
    for f in sorted(glob.glob(pattern, recursive=True)):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main(d, tag):
    stats = glob.glob(f"{d}/kt/**/*kernel_stats.csv", recursive=True)
    shutil.copy(stats[0], ROOT / "profiles" / f"{tag}_long_kernel_stats.csv")
    per = {}
    for r in csv.DictReader(open(stats[0])):
        if any(k in r["Name"] for k in KEYS):
            per[r["Name"][:80]] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
    pmc = defaultdict(lambda: defaultdict(list))
    for c in ("fetch", "write"):
        for r in rows(f"{d}/{c}/**/*counter_collection.csv"):
            if any(k in r["Kernel_Name"] for k in KEYS):
                pmc[r["Kernel_Name"][:80]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    traffic = {}
    total = 0.0
    for k, v in pmc.items():
        f = statistics.median(v.get("FETCH_SIZE", [0.0])) * 1024 * 2
        w = statistics.median(v.get("WRITE_SIZE", [0.0])) * 1024
        traffic[k] = {"fetch_bytes_corrected": f, "write_bytes": w}
        total += f + w
    call_us = sum(x["avg_us"] for x in per.values())
    out = {"workload": "configs[4] fwd-bwd B=64 T=2000 U=400 loss+grad", "kernels": per,
           "us_per_call": call_us, "algorithmic_bytes": ALGO,
           "algorithmic_GBps": ALGO / call_us / 1e3, "hbm_frac": ALGO / call_us / 1e3 / 8000,
           "traffic": traffic, "traffic_bytes_per_call": total,
           "traffic_over_algorithmic": total / ALGO}
    (ROOT / "profiles" / f"{tag}_long_summary.json").write_text(json.dumps(out, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
