#!/usr/bin/env python3
"""Per-phase cycles of the fused decode's register kernel (diagnostic build, make lib-diag):
utterance 0's s_memtime totals per step phase at BASELINE configs[2] (v1) and configs[4] (v2,
tone). Diagnostic only (never the product). One JSON line per config."""
import ctypes
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ["SSNT_TTS_C_LIB"] = str(ROOT / "ssnt-tts-rust_amd" / "lib" / "diag" / "libssnt_tts_c.so")
sys.path.insert(0, str(ROOT / "tools"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench_configs import DEV, O, S  # noqa: E402

PHASES = ["generate", "rank", "permute_dedup", "compact_gather", "stage_outputs", "between_steps"]


def read(lib):
    buf = np.zeros(8, np.uint64)
    assert lib.ssnt_diag_decode_read(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes) > 0
    steps = max(int(buf[6]), 1)
    return {"steps": steps, **{p: float(buf[i]) / steps for i, p in enumerate(PHASES)},
            "total_per_step": float(buf[:6].sum()) / steps}


def main():
    lib = S.load()
    lib.ssnt_diag_decode_read.restype = ctypes.c_int
    lib.ssnt_diag_decode_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    B, T, U, W = 256, 200, 80, 4
    lat = torch.from_numpy(O.synth_log_trans(B, T, U, seed=3)).to(DEV)
    il = torch.full((B,), U, dtype=torch.int32, device=DEV)
    for _ in range(2):
        S.lattice_beam_search_decode(lat, il, W)
    torch.cuda.synchronize()
    print(json.dumps({"config": "configs[2] v1", **read(lib)}), flush=True)
    B, I, Ot, D = 64, 400, 2000, 16
    d = O.synth_durations(B, I, Ot, D, seed=0)
    lg = torch.from_numpy(O.synth_v2_logits(d, W, D, seed=100)).to(DEV)
    table = torch.arange(D, dtype=torch.int32, device=DEV)
    il2 = torch.full((B,), I, dtype=torch.int32, device=DEV)
    ol2 = torch.full((B,), Ot, dtype=torch.int32, device=DEV)
    for _ in range(2):
        S.v2_lattice_beam_search_decode(lg, table, il2, ol2, W, 0, False, False)
    torch.cuda.synchronize()
    print(json.dumps({"config": "configs[4] v2", **read(lib)}), flush=True)
    lgt = torch.from_numpy(O.synth_tone_logits(B, I, W, 5, seed=0)).to(DEV)
    for _ in range(2):
        S.tone_latent_lattice_beam_search_decode(lgt, il2, W, 0)
    torch.cuda.synchronize()
    print(json.dumps({"config": "configs[4] tone", **read(lib)}), flush=True)


if __name__ == "__main__":
    main()
