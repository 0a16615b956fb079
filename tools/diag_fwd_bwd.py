#!/usr/bin/env python3
"""Read the in-kernel stamps of the diagnostic build (make lib-diag): where the chain and
converter waves of the pipelined fwd-bwd kernel spend their cycles. Diagnostic only."""
import ctypes
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ["SSNT_TTS_C_LIB"] = str(ROOT / "ssnt-tts-rust_amd" / "lib" / "diag" / "libssnt_tts_c.so")
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ssnt_tts_amd as S  # noqa: E402

B, T, U = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (256, 200, 80)))
variant = int(sys.argv[4]) if len(sys.argv) > 4 else 0
lib = S.load()
lib.ssnt_diag_read.restype = ctypes.c_int
lib.ssnt_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
lib.ssnt_fwd_bwd_set_variant(variant)
dev = torch.device("cuda:0")
lt = torch.log_softmax(torch.randn((B, T, U, 2), device=dev) * 1.5, -1).contiguous()
sl = torch.full((B,), T, dtype=torch.int32, device=dev)
pl = torch.full((B,), U, dtype=torch.int32, device=dev)
for _ in range(3):
    S.ssnt_fwd_bwd(lt, sl, pl)
torch.cuda.synchronize()
buf = np.zeros((4096 * 4, 8), np.uint64)
n = lib.ssnt_diag_read(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes)
assert n > 0, "not a diagnostic build"
d = buf[:B * 4].reshape(B, 4, 8).astype(np.float64)
names = ["fwd chain", "bwd chain", "fwd conv0", "bwd conv0"]
for r, nm in enumerate(names):
    tot = d[:, r, 0]
    print(f"{nm:10s} total {np.median(tot):9.0f} cyc  wait {np.median(d[:, r, 1]):9.0f}  "
          f"n_wait {np.median(d[:, r, 2]):6.0f}  cut {np.median(d[:, r, 3]):8.0f}  p1 {np.median(d[:, r, 4]):8.0f}"
          f"  per-step {np.median(tot) / T:7.1f}")
hw = buf[:B * 4].reshape(B, 4, 8)[:, :, 5].astype(np.int64)
simd = (hw >> 4) & 3
for r, nm in enumerate(names):
    print(f"{nm:10s} SIMD histogram {np.bincount(simd[:, r], minlength=4).tolist()}")
