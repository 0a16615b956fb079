#!/usr/bin/env python3
"""Run the decode-side BASELINE workloads a few times each, for `rocprofv3 --kernel-trace --stats`:
configs[2] fused v1 decode (B=256 T=200 U=80 W=4), configs[4] fused v2 decode (B=64 I=400
O=2000 D=16 W=4), configs[4] fused tone decode (B=64 I=400 C=5 W=4) and F4 (the v2 duration
fwd-bwd at the configs[4] v2 shape). Inputs as tools/bench_configs.py. No CPU timing.
Usage: python tools/prof_decode.py [iters]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
import oracle as O  # noqa: E402
import ssnt_tts_amd as S  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
lat = torch.from_numpy(O.synth_log_trans(256, 200, 80, seed=3)).to(dev)
il = torch.full((256,), 80, dtype=torch.int32, device=dev)
B, I, Ot, D, W = 64, 400, 2000, 16, 4
d = O.synth_durations(B, I, Ot, D, seed=0)
lg2 = torch.from_numpy(O.synth_v2_logits(d, W, D, seed=100)).to(dev)
table = torch.arange(D, dtype=torch.int32, device=dev)
il2 = torch.full((B,), I, dtype=torch.int32, device=dev)
ol2 = torch.full((B,), Ot, dtype=torch.int32, device=dev)
lgt = torch.from_numpy(O.synth_tone_logits(B, I, W, 5, seed=0)).to(dev)
lgf = torch.from_numpy(O.synth_v2_step_logits(d, D, seed=1)).to(dev)
for _ in range(it):
    S.lattice_beam_search_decode(lat, il, 4, check=False)
    S.v2_lattice_beam_search_decode(lg2, table, il2, ol2, W, 0, False, False, check=False)
    S.tone_latent_lattice_beam_search_decode(lgt, il2, W, 0, check=False)
    S.v2_fwd_bwd(lgf, table, il2, ol2, 0, max_total=Ot)
torch.cuda.synchronize()
print("ok")
