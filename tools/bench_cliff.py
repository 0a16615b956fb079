#!/usr/bin/env python3
"""GPU time of the fwd-bwd at the shapes the streaming kernel declines:
U % K != 0, tensors at an element offset, 512 < U <= 1024 -- default dispatch vs the two-wave
kernel. One JSON line per (shape, variant). Every timed lattice is feasible (T >= U, full
lengths): an infeasible one (S < P) only zero-fills grad and would time a memset, not the
recurrence, so such shapes are rejected before anything runs."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tools"))
import oracle as O  # noqa: E402
import ssnt_tts_amd as S  # noqa: E402
from bench_configs import gpu_time  # noqa: E402

DEV = torch.device("cuda:0")


def case(B, T, U, shift, variant):
    if T < U:
        raise ValueError(f"infeasible timing shape B={B} T={T} U={U}: every utterance has S < P, "
                         "so the kernel would only zero-fill grad")
    if variant:  # the two-wave kernel forced through the A/B build (include/ssnt_tts_c_ab.h)
        with S.use_ab() as ab:
            if ab.ssnt_fwd_bwd_set_variant(variant) != 0:
                return None
            return _case(B, T, U, shift, variant)
    return _case(B, T, U, shift, variant)


def _case(B, T, U, shift, variant):
    lt = O.synth_log_trans(B, T, U, seed=0)
    flat = torch.zeros(lt.size + shift, dtype=torch.float32, device=DEV)
    flat[shift:] = torch.from_numpy(lt.ravel()).to(DEV)
    x = flat[shift:].view(B, T, U, 2)
    sl = torch.full((B,), T, dtype=torch.int32, device=DEV)
    pl = torch.full((B,), U, dtype=torch.int32, device=DEV)
    out = {"loss": torch.empty(B, device=DEV), "grad": torch.empty((B, T, U, 2), device=DEV),
           "status": torch.zeros(1, dtype=torch.int32, device=DEV)}
    try:
        S.ssnt_fwd_bwd(x, sl, pl, out=out, check=True)
    except Exception as e:  # noqa: BLE001 -- a kernel that declines the shape
        return {"B": B, "T": T, "U": U, "offset_floats": shift, "variant": variant, "error": str(e)[:80]}
    t = gpu_time(lambda: S.ssnt_fwd_bwd(x, sl, pl, out=out), 10)
    loss = out["loss"].cpu().numpy()
    assert np.isfinite(loss).all(), "a timed lattice must be feasible"
    return {"B": B, "T": T, "U": U, "offset_floats": shift, "variant": variant, "gpu_us": t * 1e6,
            "cells_per_s": B * T * U / t}


if __name__ == "__main__":
    for (B, T, U, shift) in [(256, 200, 80, 0), (256, 200, 81, 0), (256, 200, 127, 0), (256, 200, 80, 1),
                             (256, 200, 80, 2), (256, 200, 120, 0), (64, 400, 300, 0),
                             (64, 760, 700, 0), (64, 1100, 1024, 0)]:
        for v in (0, 1):
            r = case(B, T, U, shift, v)
            if r:
                print(json.dumps(r), flush=True)
