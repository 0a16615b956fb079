#!/usr/bin/env python3
"""F4 sweep time against the band width: configs[4]-like F4 (B=64 I=400 D=16) at output
lengths O whose v2 band (0.15 O cells) spans 4 to 7 waves of the 512-thread sweep workgroup.
Run under rocprofv3 --kernel-trace: each O runs `it` calls in order (parse the trace in order).
Usage: python tools/probe_f4_window.py [it] O..."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
import oracle as OR  # noqa: E402
import ssnt_tts_amd as S  # noqa: E402

it = int(sys.argv[1])
Os = [int(x) for x in sys.argv[2:]]
dev = torch.device("cuda:0")
B, I, D = 64, 400, 16
table = torch.arange(D, dtype=torch.int32, device=dev)
il = torch.full((B,), I, dtype=torch.int32, device=dev)
for O in Os:
    d = OR.synth_durations(B, I, O, D, seed=0)
    lg = torch.from_numpy(OR.synth_v2_step_logits(d, D, seed=1)).to(dev)
    ol = torch.full((B,), O, dtype=torch.int32, device=dev)
    for _ in range(it):
        S.v2_fwd_bwd(lg, table, il, ol, 0, max_total=O)
    torch.cuda.synchronize()
    print("O", O, flush=True)
