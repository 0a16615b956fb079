#!/usr/bin/env python3
"""A/B of the streaming kernel's ring depth at BASELINE configs[1] (ssnt_fwd_bwd_stream_ring:
0 default = 8 slots + rows in LDS; 16 / 32 slots + rows in the workspace), interleaved rounds in
one process, bit-identical results checked. One JSON line per depth."""
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
import ssnt_tts_amd as S  # noqa: E402

B, T, U = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (256, 200, 80)))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
lt = torch.log_softmax(torch.randn((B, T, U, 2), generator=g, device=dev) * 1.5, -1).contiguous()
sl = torch.full((B,), T, dtype=torch.int32, device=dev)
pl = torch.full((B,), U, dtype=torch.int32, device=dev)
lib = S.load()
lib.ssnt_fwd_bwd_stream_ring.restype = ctypes.c_int
res, ref = {}, None
for rnd in range(4):
    for ring in (0, 16, 32):
        assert lib.ssnt_fwd_bwd_stream_ring(ring) == 0
        out = {"loss": torch.empty(B, device=dev), "grad": torch.empty((B, T, U, 2), device=dev)}
        S.ssnt_fwd_bwd(lt, sl, pl, out=out, check=True)
        if rnd == 0:
            if ref is None:
                ref = (out["loss"].clone(), out["grad"].clone())
            assert torch.equal(ref[0], out["loss"]) and torch.equal(ref[1], out["grad"]), ring
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            S.ssnt_fwd_bwd(lt, sl, pl, out=out)
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(ring, []).append(e0.elapsed_time(e1) / 10 * 1e3)
        kern = S.last_fwd_bwd_kernel()
        res.setdefault(f"k{ring}", kern)
lib.ssnt_fwd_bwd_stream_ring(0)
for ring in (0, 16, 32):
    print(json.dumps({"ring": ring, "B": B, "T": T, "U": U, "median_us": float(np.median(res[ring])),
                      "min_us": float(np.min(res[ring])), "kernel": res[f"k{ring}"]}), flush=True)
