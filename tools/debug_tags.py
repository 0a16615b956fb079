#!/usr/bin/env python3
"""Diagnostic build only: run the streaming kernel with SSNT_DIAG_TAG_FAULT in the environment
and print the status bits (the ring-tag negative control). Debug helper."""
import ctypes
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ["SSNT_TTS_C_LIB"] = str(ROOT / "ssnt-tts-rust_amd" / "lib" / "diag" / "libssnt_tts_c.so")
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
import torch  # noqa: E402
import ssnt_tts_amd as S  # noqa: E402
import oracle as O  # noqa: E402

dev = torch.device("cuda:0")
lib = S.load()
print("env fault:", os.environ.get("SSNT_DIAG_TAG_FAULT"), "getenv:", ctypes.CDLL(None).getenv)
for (B, T, U) in [(4, 60, 80), (2, 40, 33), (2, 60, 64), (2, 60, 66), (2, 60, 65), (2, 70, 128), (2, 140, 130), (1, 200, 80)]:
    lt = O.synth_log_trans(B, T, U, seed=1)
    r = S.ssnt_fwd_bwd(torch.from_numpy(lt).to(dev), torch.full((B,), T, dtype=torch.int32, device=dev),
                       torch.full((B,), U, dtype=torch.int32, device=dev), check=False)
    print(B, T, U, "status", int(r["status"].item()), S.last_fwd_bwd_kernel())
    r = S.ssnt_fwd_bwd(torch.from_numpy(lt).to(dev), torch.full((B,), T, dtype=torch.int32, device=dev),
                       torch.full((B,), U, dtype=torch.int32, device=dev), check=False, debug=True)
    print("   debug status", int(r["status"].item()))
