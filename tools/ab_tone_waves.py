#!/usr/bin/env python3
"""A/B of the tone fused decode's rank over 1 / 2 / 4 waves (A/B build knob
ssnt_fused_decode_tone_waves) at configs[4] (B=64 I=400 C=5 W=4), alternating rounds, HIP event
time per call (median). Outputs are checked identical across forms first."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
import oracle as O  # noqa: E402
import ssnt_tts_amd as S  # noqa: E402

dev = torch.device("cuda:0")
B, I, W, C = 64, 400, 4, 5
lg = torch.from_numpy(O.synth_tone_logits(B, I, W, C, seed=0)).to(dev)
il = torch.full((B,), I, dtype=torch.int32, device=dev)
forms = [1, 2, 4]
times = {f: [] for f in forms}
with S.use_ab() as ab:
    ref = None
    for f in forms:
        assert ab.ssnt_fused_decode_tone_waves(f) == 0
        r = S.tone_latent_lattice_beam_search_decode(lg, il, W, 0, check=True)
        got = {k: v.cpu() for k, v in r.items() if k != "status"}
        if ref is None:
            ref = got
        else:
            assert all(torch.equal(ref[k], got[k]) for k in ref), f"tone waves {f} differs"
    for _ in range(7):
        for f in forms:
            ab.ssnt_fused_decode_tone_waves(f)
            S.tone_latent_lattice_beam_search_decode(lg, il, W, 0, check=False)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                S.tone_latent_lattice_beam_search_decode(lg, il, W, 0, check=False)
            e1.record()
            torch.cuda.synchronize()
            times[f].append(e0.elapsed_time(e1) / 10 * 1e3)
print(json.dumps({"tone_waves_us": {f: round(float(np.median(times[f])), 1) for f in forms}}))
