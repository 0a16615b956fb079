#!/usr/bin/env python3
"""configs[4] fwd-bwd (B=64 T=2000 U=400): the segmented kernel with a direction in one
workgroup vs split over two (ssnt_fwd_bwd_wide_split 0 / 1), same inputs; the outputs must be
bit-identical. One JSON line per mode (median GPU time of back-to-back calls)."""
import ctypes
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
sys.path.insert(0, str(ROOT / "tools"))
import ssnt_tts_amd as S  # noqa: E402
from bench_configs import gpu_time  # noqa: E402

B, T, U = (int(x) for x in (sys.argv[1:4] if len(sys.argv) >= 4 else (64, 2000, 400)))
LANES = int(sys.argv[4]) if len(sys.argv) > 4 else 1  # positions per lane (ssnt_fwd_bwd_wide_lanes)
dev = torch.device("cuda:0")
lib = S.load()
lib.ssnt_fwd_bwd_wide_split.restype = ctypes.c_int
lib.ssnt_fwd_bwd_wide_lanes.restype = ctypes.c_int
assert lib.ssnt_fwd_bwd_wide_lanes(LANES) == 0
g = torch.Generator(device=dev).manual_seed(4)
lt = torch.log_softmax(torch.randn((B, T, U, 2), device=dev, generator=g) * 1.5, -1).contiguous()
sl = torch.full((B,), T, dtype=torch.int32, device=dev)
pl = torch.full((B,), U, dtype=torch.int32, device=dev)
res = {}
for mode in (0, 1, 0, 1):
    assert lib.ssnt_fwd_bwd_wide_split(mode) == 0
    out = {"loss": torch.empty(B, device=dev), "grad": torch.empty((B, T, U, 2), device=dev),
           "status": torch.zeros(1, dtype=torch.int32, device=dev)}
    S.ssnt_fwd_bwd(lt, sl, pl, out=out, check=True)
    kern = S.last_fwd_bwd_kernel()
    t = gpu_time(lambda: S.ssnt_fwd_bwd(lt, sl, pl, out=out), 10)
    if mode in res:
        same = torch.equal(res[mode][0], out["loss"]) and torch.equal(res[mode][1], out["grad"])
    else:
        res[mode] = (out["loss"].clone(), out["grad"].clone())
        same = True
    print(json.dumps({"B": B, "T": T, "U": U, "lanes": LANES, "split": mode, "kernel": kern, "us": round(t * 1e6, 1),
                      "repeat_identical": same}), flush=True)
lib.ssnt_fwd_bwd_wide_split(-1)
lib.ssnt_fwd_bwd_wide_lanes(1)
ident = torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
print(json.dumps({"split_vs_one_workgroup_bit_identical": ident}), flush=True)
assert ident
