#!/usr/bin/env python3
"""Kernel time of one fwd-bwd shape with the library named by SSNT_TTS_C_LIB (A/B of built
variants, tools/ab_libs.py): HIP events around `iters` back-to-back calls, median of 5 rounds;
plus a bit-level checksum of loss and grad so variants can be checked for identical results.
Usage: python tools/time_fwd_bwd.py B T U [iters]  -> one JSON line."""
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
import ssnt_tts_amd as S  # noqa: E402

B, T, U = (int(x) for x in sys.argv[1:4])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 5
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
lt = torch.log_softmax(torch.randn((B, T, U, 2), generator=g, device=dev) * 1.5, -1).contiguous()
sl = torch.full((B,), T, dtype=torch.int32, device=dev)
pl = torch.full((B,), U, dtype=torch.int32, device=dev)
out = {"loss": torch.empty(B, device=dev), "grad": torch.empty((B, T, U, 2), device=dev),
       "status": torch.zeros(1, dtype=torch.int32, device=dev)}
S.ssnt_fwd_bwd(lt, sl, pl, out=out, check=True)
S.ssnt_fwd_bwd(lt, sl, pl, out=out, check=True)
torch.cuda.synchronize()
ck = int(out["grad"].view(torch.int32).to(torch.int64).sum().item()) ^ \
    int(out["loss"].view(torch.int32).to(torch.int64).sum().item())
ts = []
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        S.ssnt_fwd_bwd(lt, sl, pl, out=out)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / iters * 1e3)
print(json.dumps({"lib": os.environ.get("SSNT_TTS_C_LIB", "product"), "B": B, "T": T, "U": U,
                  "median_us": float(np.median(ts)), "min_us": float(np.min(ts)),
                  "kernel": S.last_fwd_bwd_kernel(), "checksum": ck}), flush=True)
