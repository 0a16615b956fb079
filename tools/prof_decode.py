#!/usr/bin/env python3
"""Run the config-3 fused decode a few times (for rocprofv3 --kernel-trace --stats)."""
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
lat = torch.from_numpy(O.synth_log_trans(256, 200, 80, seed=3)).to(dev)
il = torch.full((256,), 80, dtype=torch.int32, device=dev)
for _ in range(10):
    S.lattice_beam_search_decode(lat, il, 4, check=False)
torch.cuda.synchronize()
print("ok")
