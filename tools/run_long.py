#!/usr/bin/env python3
"""configs[4] fwd-bwd (B=64 T=2000 U=400) run N times back to back -- a target for rocprofv3
kernel traces and PMC passes of the long-row kernel."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
sys.path.insert(0, str(ROOT))
import ssnt_tts_amd as S  # noqa: E402
from bench import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
if len(sys.argv) > 2:  # A/B: positions per lane of the long-row kernel
    import ctypes
    S.load().ssnt_fwd_bwd_wide_lanes.restype = ctypes.c_int
    assert S.load().ssnt_fwd_bwd_wide_lanes(int(sys.argv[2])) == 0
B, T, U = 64, 2000, 400
dev = torch.device("cuda:0")
lt = synth(B, T, U, 0, dev)
sl = torch.full((B,), T, dtype=torch.int32, device=dev)
pl = torch.full((B,), U, dtype=torch.int32, device=dev)
out = {"loss": torch.empty(B, device=dev), "grad": torch.empty((B, T, U, 2), device=dev)}
S.ssnt_fwd_bwd(lt, sl, pl, out=out, check=True)
for _ in range(n):
    S.ssnt_fwd_bwd(lt, sl, pl, out=out)
torch.cuda.synchronize()
print("loss[0]", float(out["loss"][0]))
