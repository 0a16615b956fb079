#!/usr/bin/env python3
"""configs[4] fwd-bwd (B=64 T=2000 U=400) through the A/B build: the segmented kernel with each
direction in one workgroup (split 0), split over two workgroups (1) and split in phase 2 only (2),
alternating rounds; outputs bit-identical across forms. One JSON line per form (median HIP event
time per call). Run under rocprofv3 --kernel-trace --stats for the per-phase kernel times."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
import ssnt_tts_amd as S  # noqa: E402

# args: [B T U] form... -- a form is "<split>" or "<split>k2" (two positions per lane:
# ssnt_fwd_bwd_wide_lanes(2)); default configs[4] and forms 0 1 2
args = sys.argv[1:]
B, T, U = (int(x) for x in args[:3]) if len(args) >= 3 and int(args[0]) > 2 else (64, 2000, 400)
modes = (args[3:] if len(args) >= 3 and int(args[0]) > 2 else args) or ["0", "1", "2"]


def set_form(ab, m):
    assert ab.ssnt_fwd_bwd_wide_split(int(m[:-2] if m.endswith("k2") else m)) == 0
    assert ab.ssnt_fwd_bwd_wide_lanes(2 if m.endswith("k2") else 1) == 0

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(4)
lt = torch.log_softmax(torch.randn((B, T, U, 2), device=dev, generator=g) * 1.5, -1).contiguous()
sl = torch.full((B,), T, dtype=torch.int32, device=dev)
pl = torch.full((B,), U, dtype=torch.int32, device=dev)
times = {m: [] for m in modes}
kern = {}
with S.use_ab() as ab:
    ref = None
    for m in modes:
        set_form(ab, m)
        r = S.ssnt_fwd_bwd(lt, sl, pl, check=True)
        kern[m] = S.last_fwd_bwd_kernel()
        got = (r["loss"].cpu(), r["grad"].cpu())
        if ref is None:
            ref = got
        else:
            assert torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1]), f"mode {m} differs"
        del r
    out = {"loss": torch.empty(B, device=dev), "grad": torch.empty((B, T, U, 2), device=dev),
           "status": torch.zeros(1, dtype=torch.int32, device=dev)}
    for _ in range(5):
        for m in modes:
            set_form(ab, m)
            S.ssnt_fwd_bwd(lt, sl, pl, out=out)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(4):
                S.ssnt_fwd_bwd(lt, sl, pl, out=out)
            e1.record()
            torch.cuda.synchronize()
            times[m].append(e0.elapsed_time(e1) / 4 * 1e3)
for m in modes:
    print(json.dumps({"B": B, "T": T, "U": U, "form": m, "kernel": kern[m],
                      "us": round(float(np.median(times[m])), 1)}))
