#!/usr/bin/env python3
"""Summarise rocprofv3 output for the fwd-bwd kernel into profiles/.

Inputs (from tools/profile_gpu.sh): <dir>/kt (kernel trace + stats), <dir>/fetch (FETCH_SIZE
pass), <dir>/write (WRITE_SIZE pass). Writes:
  profiles/<tag>_kernel_stats.csv     -- the rocprofv3 --stats summary (copied)
  profiles/<tag>_fwd_bwd_summary.json -- avg duration + HBM traffic per launch
  profiles/pmc_fwd_bwd.json           -- what bench.py reports as roofline.traffic (with the
                                         kernel instance, source hash and workload it was taken
                                         on: bench.py reports it only for the same three)

HBM bytes per launch, following MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE counts exactly half the bytes of a wide coalesced streaming read, so
the read side is doubled (the kernel's log_trans stream is such a read); WRITE_SIZE is taken as
is. Both raw and corrected numbers are recorded.
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KERNEL_KEY = "k_fwd_bwd"


def _rows(pattern):
    files = sorted(glob.glob(pattern, recursive=True))
    out = []
    for f in files:
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out, files


def _pmc(d, counter):
    rows, files = _rows(os.path.join(d, "**", "*counter_collection.csv"))
    vals = []
    for r in rows:
        name = r.get("Kernel_Name") or r.get("KernelName") or ""
        if KERNEL_KEY in name and r.get("Counter_Name") == counter:
            vals.append(float(r["Counter_Value"]))
    return vals, files


def main():
    d, tag = sys.argv[1], sys.argv[2]
    prof = ROOT / "profiles"
    prof.mkdir(exist_ok=True)
    stats, sfiles = _rows(os.path.join(d, "kt", "**", "*kernel_stats.csv"))
    if sfiles:
        shutil.copy(sfiles[0], prof / f"{tag}_kernel_stats.csv")
    trace, _ = _rows(os.path.join(d, "kt", "**", "*kernel_trace.csv"))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in trace
            if KERNEL_KEY in (r.get("Kernel_Name") or "")]
    fetch, _ = _pmc(os.path.join(d, "fetch"), "FETCH_SIZE")
    write, _ = _pmc(os.path.join(d, "write"), "WRITE_SIZE")
    summ = {"tag": tag, "kernel": KERNEL_KEY, "launches": len(durs)}
    names = sorted({r.get("Kernel_Name") for r in trace if KERNEL_KEY in (r.get("Kernel_Name") or "")})
    summ["kernel_names"] = names
    # the bench line printed under the profiler names the dispatched instance and the sources
    for logf in glob.glob(os.path.join(d, "kt*.log")) + glob.glob(os.path.join(d, "kt", "*.log")):
        for line in Path(logf).read_text(errors="replace").splitlines():
            if line.startswith("{") and '"roofline"' in line:
                rl = json.loads(line)["roofline"]
                cfg = json.loads(line)["config"]
                summ["dispatch"] = rl.get("kernel")
                summ["source_sha"] = rl.get("source_sha")
                summ["workload"] = [cfg["global_batch"] // json.loads(line)["n_gpus"], cfg["T"], cfg["U"]]
    if durs:
        summ["avg_us"] = statistics.mean(durs)
        summ["median_us"] = statistics.median(durs)
        summ["min_us"] = min(durs)
    if fetch and write:
        f_kib = statistics.median(fetch)
        w_kib = statistics.median(write)
        summ.update({
            "fetch_size_kib_raw": f_kib, "write_size_kib_raw": w_kib,
            "hbm_read_bytes": 2 * f_kib * 1024, "hbm_write_bytes": w_kib * 1024,
            "hbm_bytes_per_launch": 2 * f_kib * 1024 + w_kib * 1024,
            "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE x1; KiB->B",
        })
    (prof / f"{tag}_fwd_bwd_summary.json").write_text(json.dumps(summ, indent=1))
    if "hbm_bytes_per_launch" in summ and "dispatch" in summ:
        (prof / "pmc_fwd_bwd.json").write_text(json.dumps(summ, indent=1))
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main()
