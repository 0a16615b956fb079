#!/usr/bin/env python3
"""Kernel time of the streaming kernel under SSNT_EXP timing-experiment masks (make lib-expnd),
measured like bench.py: K launches captured in one HIP graph, HIP events around the replay, so
no host/wrapper time is included. Timing only -- most masks give wrong results.
Usage: python tools/ab_exp_graph.py B T U mask1 mask2 ...  -> one JSON line per mask."""
import ctypes
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ.setdefault("SSNT_TTS_C_LIB", str(ROOT / "ssnt-tts-rust_amd" / "lib" / "expnd" / "libssnt_tts_c.so"))
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ssnt_tts_amd as S  # noqa: E402

B, T, U = (int(x) for x in sys.argv[1:4])
masks = [int(x) for x in sys.argv[4:]]
dev = torch.device("cuda:0")
torch.manual_seed(0)
lt = torch.log_softmax(torch.randn((B, T, U, 2), device=dev) * 1.5, -1).contiguous()
sl = torch.full((B,), T, dtype=torch.int32, device=dev)
pl = torch.full((B,), U, dtype=torch.int32, device=dev)
loss = torch.empty(B, device=dev)
grad = torch.empty((B, T, U, 2), device=dev)
lib = S.load()
if os.environ.get("SSNT_VARIANT"):  # e.g. 12: the one-step streaming kernel instead of the pair kernel
    assert lib.ssnt_fwd_bwd_set_variant(int(os.environ["SSNT_VARIANT"])) == 0
wsb = int(lib.ssnt_fwd_bwd_workspace_size(B, T, U))
ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
vp = ctypes.c_void_p
K = 20


def launch(stream):
    rc = lib.ssnt_fwd_bwd_device(
        vp(lt.data_ptr()), None, vp(sl.data_ptr()), vp(pl.data_ptr()), B, T, U, 1,
        vp(loss.data_ptr()), vp(grad.data_ptr()), None, None, None,
        vp(ws.data_ptr()) if wsb else None, wsb, None, vp(stream.cuda_stream))
    if rc != 0:
        raise RuntimeError(S.status_string(rc))


res = {m: [] for m in masks}
main = torch.cuda.current_stream(dev)
for m in masks:
    os.environ["SSNT_EXP"] = str(m)
    for _ in range(3):
        launch(main)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(dev)
    with torch.cuda.graph(g, stream=cap):
        for _ in range(K):
            launch(cap)
    g.replay()
    torch.cuda.synchronize()
    for rnd in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        g.replay()
        e1.record(main)
        torch.cuda.synchronize()
        res[m].append(e0.elapsed_time(e1) / K * 1e3)
    print(json.dumps({"mask": m, "B": B, "T": T, "U": U, "kernel_us": float(np.median(res[m])),
                      "min_us": float(np.min(res[m])), "dispatch": S.last_fwd_bwd_kernel()}), flush=True)
