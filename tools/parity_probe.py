#!/usr/bin/env python3
"""Localise a fwd-bwd parity failure: per output, the first lattice rows / positions where the
GPU kernel (chosen variant) and the split-exponent oracle disagree. Debug tool, GPU only.

usage: parity_probe.py B T U [variant] [obs]
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ssnt_tts_amd as S  # noqa: E402
from oracle import oracle  # noqa: E402

B, T, U = (int(x) for x in sys.argv[1:4])
variant = int(sys.argv[4]) if len(sys.argv) > 4 else 0
obs = len(sys.argv) > 5 and sys.argv[5] == "1"
lib = S.load()
assert lib.ssnt_fwd_bwd_set_variant(variant) == 0
lt = oracle.synth_log_trans(B, T, U, seed=B * 1000 + T)
lo = (np.random.default_rng(T).standard_normal((B, T, U)) * 15 - 40).astype(np.float32) if obs else None
Sl, Pl = [T] * B, [min(T, U)] * B
dev = torch.device("cuda:0")
r = S.ssnt_fwd_bwd(torch.from_numpy(lt).to(dev), torch.tensor(Sl, dtype=torch.int32, device=dev),
                   torch.tensor(Pl, dtype=torch.int32, device=dev),
                   None if lo is None else torch.from_numpy(lo).to(dev), debug=True, check=False)
g = {k: v.cpu().numpy() for k, v in r.items()}
o = oracle.fwd_bwd_xf(lt, Sl, Pl, log_obs=lo, debug=True)
print("status", g.get("status"))
print("loss gpu", g["loss"], "oracle", o["loss"])
for k in ("log_alpha", "log_beta", "grad") + (("grad_obs",) if obs else ()):
    a, b = g[k], o[k]
    bad = ~((a == b) | (np.isnan(a) & np.isnan(b)))
    print(f"{k}: {bad.sum()} cells differ")
    for bi in range(B):
        rows = np.where(bad[bi].reshape(T, -1).any(axis=1))[0]
        if len(rows):
            s = rows[0] if k != "log_beta" else rows[-1]
            cols = np.where(bad[bi].reshape(T, -1)[s])[0]
            print(f"  b={bi} rows {rows.min()}..{rows.max()} (n={len(rows)}); row {s} cols {cols[:12].tolist()}")
            print("    gpu   ", a[bi].reshape(T, -1)[s][:8])
            print("    oracle", b[bi].reshape(T, -1)[s][:8])
            break
