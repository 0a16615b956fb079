#!/usr/bin/env python3
"""Kernel time of the streaming kernel under SSNT_EXP timing-experiment masks (make lib-expnd:
the experiment knobs without the diagnostic stamps). Timing only -- most masks give wrong
results. Usage: python tools/ab_exp.py B T U mask1 mask2 ...  -> one JSON line per mask."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ["SSNT_TTS_C_LIB"] = str(ROOT / "ssnt-tts-rust_amd" / "lib" / "expnd" / "libssnt_tts_c.so")
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ssnt_tts_amd as S  # noqa: E402

B, T, U = (int(x) for x in sys.argv[1:4])
masks = [int(x) for x in sys.argv[4:]]
dev = torch.device("cuda:0")
lt = torch.log_softmax(torch.randn((B, T, U, 2), device=dev) * 1.5, -1).contiguous()
sl = torch.full((B,), T, dtype=torch.int32, device=dev)
pl = torch.full((B,), U, dtype=torch.int32, device=dev)
out = {"loss": torch.empty(B, device=dev), "grad": torch.empty((B, T, U, 2), device=dev)}
res = {m: [] for m in masks}
for rnd in range(3):
    for m in masks:
        os.environ["SSNT_EXP"] = str(m)
        for _ in range(2):
            S.ssnt_fwd_bwd(lt, sl, pl, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            S.ssnt_fwd_bwd(lt, sl, pl, out=out)
        e1.record()
        torch.cuda.synchronize()
        res[m].append(e0.elapsed_time(e1) / 10 * 1e3)
for m in masks:
    print(json.dumps({"mask": m, "B": B, "median_us": float(np.median(res[m])), "min_us": float(np.min(res[m]))}), flush=True)
