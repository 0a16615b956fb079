#!/usr/bin/env python3
"""A/B of the fused decodes' step ordering (ssnt_fused_decode_select: 0 full rank, 1 selection)
at BASELINE configs[2] (v1) and configs[4] (v2, tone), plus tie-rich v2 / tone inputs (more
duplicates, so more selection rounds). GPU time only (HIP events, median of 5 rounds), the two
modes alternated. One JSON line per (case, mode)."""
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
from bench_configs import DEV, O, S, gpu_time  # noqa: E402


def cases():
    B, T, U, W = 256, 200, 80, 4
    lat = torch.from_numpy(O.synth_log_trans(B, T, U, seed=3)).to(DEV)
    il = torch.full((B,), U, dtype=torch.int32, device=DEV)
    yield "configs[2] v1", lambda: S.lattice_beam_search_decode(lat, il, W, check=False)
    B, I, Ot, D = 64, 400, 2000, 16
    d = O.synth_durations(B, I, Ot, D, seed=0)
    table = torch.arange(D, dtype=torch.int32, device=DEV)
    il2, ol2 = torch.full((B,), I, dtype=torch.int32, device=DEV), torch.full((B,), Ot, dtype=torch.int32, device=DEV)
    for tr in (False, True):
        lg = torch.from_numpy(O.synth_v2_logits(d, W, D, seed=100, tie_rich=tr)).to(DEV)
        yield f"configs[4] v2{' tie-rich' if tr else ''}", (
            lambda lg=lg: S.v2_lattice_beam_search_decode(lg, table, il2, ol2, W, 0, False, False, check=False))
    for tr in (False, True):
        lgt = torch.from_numpy(O.synth_tone_logits(B, I, W, 5, seed=0, tie_rich=tr)).to(DEV)
        yield f"configs[4] tone{' tie-rich' if tr else ''}", (
            lambda lgt=lgt: S.tone_latent_lattice_beam_search_decode(lgt, il2, W, 0, check=False))


def main():
    lib = S.load()
    lib.ssnt_fused_decode_select.restype = ctypes.c_int
    for name, fn in cases():
        res = {}
        for rep in range(2):
            for mode in (0, 1):
                assert lib.ssnt_fused_decode_select(mode) == 0
                t = gpu_time(fn, 10) * 1e6
                res.setdefault(mode, []).append(t)
        for mode in (0, 1):
            print(json.dumps({"case": name, "mode": ["rank", "select"][mode],
                              "gpu_us": float(np.min(res[mode])), "runs_us": res[mode]}), flush=True)
    lib.ssnt_fused_decode_select(-1)


if __name__ == "__main__":
    main()
