#!/usr/bin/env python3
"""Median HIP-event time per ssnt_fwd_bwd call at the long shapes, through whichever product
library SSNT_TTS_C_LIB names (for old/new library A/B runs in alternating processes).
Prints one JSON line per shape with the kernel name and a loss/grad checksum.
Usage: SSNT_TTS_C_LIB=... python tools/time_long.py tag [B T U]..."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
import ssnt_tts_amd as S  # noqa: E402

tag = sys.argv[1]
nums = [int(x) for x in sys.argv[2:]]
shapes = [tuple(nums[i:i + 3]) for i in range(0, len(nums), 3)] or [(64, 2000, 400)]
dev = torch.device("cuda:0")
for B, T, U in shapes:
    g = torch.Generator(device=dev).manual_seed(4)
    lt = torch.log_softmax(torch.randn((B, T, U, 2), device=dev, generator=g) * 1.5, -1).contiguous()
    sl = torch.full((B,), T, dtype=torch.int32, device=dev)
    pl = torch.full((B,), U, dtype=torch.int32, device=dev)
    r = S.ssnt_fwd_bwd(lt, sl, pl, check=True)
    kern = S.last_fwd_bwd_kernel()
    ck = [float(r["loss"].double().sum()), float(r["grad"].double().abs().sum())]
    del r
    out = {"loss": torch.empty(B, device=dev), "grad": torch.empty((B, T, U, 2), device=dev),
           "status": torch.zeros(1, dtype=torch.int32, device=dev)}
    ts = []
    for _ in range(7):
        S.ssnt_fwd_bwd(lt, sl, pl, out=out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(4):
            S.ssnt_fwd_bwd(lt, sl, pl, out=out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 4 * 1e3)
    assert int(out["status"].item()) == 0
    print(json.dumps({"tag": tag, "B": B, "T": T, "U": U, "kernel": kern,
                      "us": round(float(np.median(ts)), 1), "checksum": ck}), flush=True)
    del lt, out
    torch.cuda.empty_cache()
