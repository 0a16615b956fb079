#!/usr/bin/env python3
"""Debug: fwd-bwd of one shape with grad pre-filled with NaN (unwritten cells stay NaN), compared
with the oracle; prints how many cells differ, how many were never written, and the first ones.
Usage: SSNT_TTS_C_LIB=... python tools/debug_desc.py B T U [repeats]"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "ssnt-tts-rust_amd"), str(ROOT / "oracle")]
import oracle as O  # noqa: E402
import ssnt_tts_amd as S  # noqa: E402

B, T, U = (int(x) for x in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
dev = torch.device("cuda:0")
lt = O.synth_log_trans(B, T, U, seed=U)
Sl, Pl = [T] * B, [U] * B
o = O.fwd_bwd_xf(lt, Sl, Pl)
x = torch.from_numpy(lt).to(dev)
sl = torch.tensor(Sl, dtype=torch.int32, device=dev)
pl = torch.tensor(Pl, dtype=torch.int32, device=dev)
for r in range(reps):
    g = torch.full((B, T, U, 2), float("nan"), device=dev)
    out = {"grad": g, "loss": torch.empty(B, device=dev), "status": torch.zeros(1, dtype=torch.int32, device=dev)}
    S.ssnt_fwd_bwd(x, sl, pl, out=out, check=True)
    gg = g.cpu().numpy()
    diff = ~((gg == o["grad"]) | (np.isnan(gg) & np.isnan(o["grad"])))
    nan = np.isnan(gg) & ~np.isnan(o["grad"])
    print(f"rep {r}: kernel {S.last_fwd_bwd_kernel()} loss-equal {np.array_equal(out['loss'].cpu().numpy(), o['loss'])} "
          f"diff {int(diff.sum())} unwritten {int(nan.sum())}", flush=True)
    idx = np.argwhere(diff)
    if len(idx):
        rows = sorted(set(map(tuple, idx[:, :2].tolist())))
        print("  (b, s) rows with diffs:", rows[:40], "... total", len(rows))
        for i in idx[:12]:
            t = tuple(i)
            print("  ", t, gg[t], o["grad"][t], hex(np.float32(gg[t]).view(np.uint32)))
