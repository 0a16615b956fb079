#!/usr/bin/env python3
"""Read the per-wave s_memtime totals of the diagnostic build (make lib-diag) of the streaming
fwd-bwd kernel: where each role spends its cycles. Diagnostic only (never the product).
Usage: python tools/diag_fwd_bwd.py [B T U]"""
import ctypes
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ["SSNT_TTS_C_LIB"] = str(ROOT / "ssnt-tts-rust_amd" / "lib" / os.environ.get("SSNT_DIAG_LIB", "diag") / "libssnt_tts_c.so")
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ssnt_tts_amd as S  # noqa: E402

NC, NH = 3, 4  # the streaming kernel's K <= 2 wave mix
ROLES = ["alpha chain", "beta chain"] + [f"conv {'fb'[i % 2]}{i // 2}" for i in range(2 * NC)] + \
        [f"grad {'fb'[i % 2]}{i // 2}" for i in range(2 * NH)]
B, T, U = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (256, 200, 80)))
lib = S.load()
lib.ssnt_diag_read.restype = ctypes.c_int
lib.ssnt_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
dev = torch.device("cuda:0")
lt = torch.log_softmax(torch.randn((B, T, U, 2), device=dev) * 1.5, -1).contiguous()
sl = torch.full((B,), T, dtype=torch.int32, device=dev)
pl = torch.full((B,), U, dtype=torch.int32, device=dev)
for _ in range(3):
    S.ssnt_fwd_bwd(lt, sl, pl)
torch.cuda.synchronize()
buf = np.zeros((1024, 18, 8), np.uint64)
n = lib.ssnt_diag_read(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes)
assert n > 0, "not a diagnostic build"
d = buf[:min(B, 1024)].astype(np.float64)
print(f"B={B} T={T} U={U} kernel {S.last_fwd_bwd_kernel()}: median over utterances (cycles)")
times = []
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    S.ssnt_fwd_bwd(lt, sl, pl, check=False)
    e1.record()
    torch.cuda.synchronize()
    times.append(e0.elapsed_time(e1) * 1e3)
print(f"launch (incl. wrapper) median {np.median(times):.1f} us")
for w, nm in enumerate(ROLES):
    tot, wait, nw, cut, cw = (np.median(d[:, w, i]) for i in range(5))
    c0, c1, c2 = (np.median(d[:, w, i]) for i in (5, 6, 7))
    extra = f"  load-wait {c2:7.0f} convert {c0:7.0f} ring-write {c1:7.0f}" if nm.startswith("conv") else ""
    print(f"{nm:12s} total {tot:8.0f}  spinning {wait:8.0f} ({nw:4.0f} spins)  cut@ {cut:8.0f}"
          f" (spun {cw:7.0f} before)  per-step {tot / T:6.1f}{extra}")
