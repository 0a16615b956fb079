"""Save GPU outputs of one long-row fwd-bwd case (tests/test_gpu_fwd_bwd.py WIDE_SHAPES[0])."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "ssnt-tts-rust_amd"), str(ROOT / "oracle")]
import oracle as O  # noqa: E402
import ssnt_tts_amd as S  # noqa: E402

B, T, U = 2, 40, 257
rng = np.random.default_rng(U + T)
lt = O.synth_log_trans(B, T, U, seed=U)
P = [min(U, T)] + [int(x) for x in rng.integers(1, min(U, T) + 1, size=B - 1)]
Sl = [T] + [int(rng.integers(p, T + 1)) for p in P[1:]]
dev = torch.device("cuda:0")
r = S.ssnt_fwd_bwd(torch.from_numpy(lt).to(dev), torch.tensor(Sl, dtype=torch.int32, device=dev),
                   torch.tensor(P, dtype=torch.int32, device=dev), debug=True, check=True)
np.savez(ROOT / "gpurun_out" / "wide_dbg.npz", S=np.array(Sl), P=np.array(P),
         **{k: v.cpu().numpy() for k, v in r.items() if k != "status"})
print("saved", Sl, P)
