#!/usr/bin/env python3
"""A/B of built library variants on one fwd-bwd shape: each variant's timing runs in its own
process (tools/time_fwd_bwd.py with SSNT_TTS_C_LIB), rounds alternate the order.
Usage: python tools/ab_libs.py B T U iters rounds lib1 [lib2 ...]  ('product' = the in-tree lib)"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
B, T, U, iters, rounds = sys.argv[1:6]
libs = sys.argv[6:]
res = {lib: [] for lib in libs}
for r in range(int(rounds)):
    for lib in (libs if r % 2 == 0 else libs[::-1]):
        env = dict(os.environ)
        if lib != "product":
            env["SSNT_TTS_C_LIB"] = str(ROOT / lib)
        out = subprocess.run([sys.executable, str(ROOT / "tools" / "time_fwd_bwd.py"), B, T, U, iters],
                             env=env, capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(json.dumps({"lib": lib, "error": out.stderr[-400:]}), flush=True)
            sys.exit(1)
        res[lib].append(json.loads(out.stdout.strip().splitlines()[-1]))
for lib, rs in res.items():
    print(json.dumps({"lib": lib, "shape": [int(B), int(T), int(U)],
                      "median_us": sorted(x["median_us"] for x in rs)[len(rs) // 2],
                      "min_us": min(x["min_us"] for x in rs), "kernel": rs[0]["kernel"],
                      "checksums": sorted({x["checksum"] for x in rs})}), flush=True)
