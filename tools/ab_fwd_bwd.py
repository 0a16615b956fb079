#!/usr/bin/env python3
"""In-process A/B of the fwd-bwd kernel variants (interleaved rounds, one process; cf.
cdna_hip_programming.md rule 24). Prints median / min kernel time per variant and shape."""
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
import ssnt_tts_amd as S  # noqa: E402


def bench_shape(B, T, U, variants=(0, 1, 2, 3), rounds=5, iters=10, use_sum=False):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    lt = torch.log_softmax(torch.randn((B, T, U, 2), generator=g, device=dev) * 1.5, -1).contiguous()
    sl = torch.full((B,), T, dtype=torch.int32, device=dev)
    pl = torch.full((B,), U, dtype=torch.int32, device=dev)
    loss = torch.empty(B, device=dev)
    grad = torch.empty((B, T, U, 2), device=dev)
    lib = S.load()
    wsb = int(lib.ssnt_fwd_bwd_workspace_size(B, T, U))
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    vp = ctypes.c_void_p
    st = vp(torch.cuda.current_stream().cuda_stream)
    args = (vp(lt.data_ptr()), None, vp(sl.data_ptr()), vp(pl.data_ptr()), B, T, U, 1,
            vp(loss.data_ptr()), vp(grad.data_ptr()), None, None, None,
            vp(ws.data_ptr()) if wsb else None, wsb, None)
    lsum = torch.zeros(1, device=dev)
    state = torch.zeros(int(lib.ssnt_fwd_bwd_sum_state_size(B)), dtype=torch.uint8, device=dev)
    if use_sum:  # fused batch loss sum (ssnt_fwd_bwd_sum_device)
        args = args + (vp(lsum.data_ptr()), vp(state.data_ptr()), st)
        call = lib.ssnt_fwd_bwd_sum_device
    else:
        args = args + (st,)
        call = lib.ssnt_fwd_bwd_device
    res = {v: [] for v in variants}
    ref = None
    for rnd in range(rounds):
        for v in variants:
            lib.ssnt_fwd_bwd_set_variant(v)
            for _ in range(2):
                rc = call(*args)
                assert rc == 0, f"variant {v}: status {rc}"
            torch.cuda.synchronize()
            if rnd == 0:
                out = (loss.clone(), grad.clone())
                if ref is None:
                    ref = out
                else:
                    assert torch.equal(ref[0], out[0]) and torch.equal(ref[1], out[1]), "variants differ"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                call(*args)
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / iters * 1e3)
    lib.ssnt_fwd_bwd_set_variant(0)
    return {f"v{v}": {"median_us": float(np.median(t)), "min_us": float(np.min(t))} for v, t in res.items()}


if __name__ == "__main__":
    shapes = [(256, 200, 80), (64, 2000, 400), (256, 50, 20), (1024, 200, 80)]
    out = {}
    for sh in shapes:
        out["x".join(map(str, sh))] = bench_shape(*sh, rounds=3 if sh[1] > 1000 else 5)
        print(json.dumps({"shape": sh, **out["x".join(map(str, sh))]}), flush=True)
