#!/usr/bin/env python3
"""Median HIP-event time per v2_fwd_bwd (F4) call at the configs[4] shape (B=64 I=400 O=2000
D=16), through whichever product library SSNT_TTS_C_LIB names; loss/grad checksums for
bit-identity across libraries. Usage: SSNT_TTS_C_LIB=... python tools/time_f4.py tag"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
import oracle as OR  # noqa: E402
import ssnt_tts_amd as S  # noqa: E402

dev = torch.device("cuda:0")
B, I, O, D = 64, 400, 2000, 16
d = OR.synth_durations(B, I, O, D, seed=0)
lg = torch.from_numpy(OR.synth_v2_step_logits(d, D, seed=1)).to(dev)
table = torch.arange(D, dtype=torch.int32, device=dev)
il = torch.full((B,), I, dtype=torch.int32, device=dev)
ol = torch.full((B,), O, dtype=torch.int32, device=dev)
r = S.v2_fwd_bwd(lg, table, il, ol, 0, max_total=O)
ck = [float(r["loss"].double().sum()), float(r["grad"].double().abs().sum())]
ts = []
for _ in range(7):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(4):
        S.v2_fwd_bwd(lg, table, il, ol, 0, max_total=O)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 4 * 1e3)
print(json.dumps({"tag": sys.argv[1], "us": round(float(np.median(ts)), 1), "checksum": ck}), flush=True)
