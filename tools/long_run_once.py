#!/usr/bin/env python3
"""configs[4] long-form fwd-bwd (B=64 T=2000 U=400, loss + grad) a few times, for profiling
(tools/profile_long.sh). No CPU baseline."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
import ssnt_tts_amd as S  # noqa: E402

B, T, U = 64, 2000, 400
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(4)
lt = torch.log_softmax(torch.randn((B, T, U, 2), device=dev, generator=g) * 1.5, -1).contiguous()
sl = torch.full((B,), T, dtype=torch.int32, device=dev)
pl = torch.full((B,), U, dtype=torch.int32, device=dev)
out = {"loss": torch.empty(B, device=dev), "grad": torch.empty((B, T, U, 2), device=dev),
       "status": torch.zeros(1, dtype=torch.int32, device=dev)}
S.ssnt_fwd_bwd(lt, sl, pl, out=out, check=True)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    S.ssnt_fwd_bwd(lt, sl, pl, out=out)
torch.cuda.synchronize()
print("ok")
