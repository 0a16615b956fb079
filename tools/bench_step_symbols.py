#!/usr/bin/env python3
"""Per-call latency of the unchanged per-step reference symbols (host pointers, synchronous) --
the path every existing TF op call takes (ssnt_tts_beam_search_decode_op.cc:116-128 calls
ssnt_tts_beam_search_decode once per decoder step) -- beside the CPU oracle's step.

Both sides are called through ctypes from Python; the cost of an empty ctypes call into the
library is reported so it can be subtracted. GPU: staging mode 0 (one H2D, kernel, one D2H,
sync) and 1 (zero-copy: the kernel reads/writes the pinned staging buffer; launch + sync).
CPU: the oracle's step per call, and amortised over a 4096-element batch (compute only).
"""
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "ssnt-tts-rust_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import torch  # noqa: E402,F401  (binds the HIP runtime first)

import decode_cases as dc  # noqa: E402
import oracle as O  # noqa: E402
from ssnt_tts_amd import _lib, capi  # noqa: E402


def per_call(fn, n=2000, rounds=5):
    fn()
    meds = []
    for _ in range(rounds):
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        meds.append((time.perf_counter() - t0) / n)
    return float(np.median(meds)) * 1e6


def raw_v1(lib, c, n=5000):
    """The v1 W=4 step called through ctypes with its pointers built once (no numpy wrapper in
    the loop), GPU symbol and C oracle alike; plus the GPU call split into its host phases
    (ssnt_diag_step_clock) and the floor under it: an empty kernel launched on the same per-thread
    stream and synchronised (ssnt_diag_null_launch)."""
    W = 4
    vp = ctypes.c_void_p
    h = np.ascontiguousarray(c["h"][0], np.float32)
    hist = np.ascontiguousarray(c["hist"][0], np.float32)
    fin = np.ascontiguousarray(c["fin"][0], np.bool_)
    t = np.ascontiguousarray(c["t"][0], np.int32)
    u = np.ascontiguousarray(c["u"][0], np.int32)
    outs = [np.empty(W, dt) for dt in (np.int32, np.float32, np.int32, np.int32, np.bool_, np.int32)]
    ptr = lambda a: vp(a.ctypes.data)  # noqa: E731
    gargs = [ptr(h), ptr(hist), ptr(fin), ptr(t), ptr(u), 80, W] + [ptr(o) for o in outs]
    f = lib.ssnt_tts_beam_search_decode
    ol = O.lib()
    il = np.array([80], np.int32)
    oouts = [np.empty(W, dt) for dt in (np.int32, np.float32, np.int32, np.int32, np.bool_, np.int32)]
    ol.oracle_v1_step.argtypes = [ctypes.c_int] * 3 + [vp] * 12
    oargs = [1, W, W, ptr(h), ptr(hist), ptr(fin), ptr(t), ptr(u), ptr(il)] + [ptr(o) for o in oouts]
    g = ol.oracle_v1_step
    out = {"raw_gpu_v1_W4_us": per_call(lambda: f(*gargs), n=n),
           "raw_cpu_v1_W4_us": per_call(lambda: g(*oargs), n=n)}
    ph = np.zeros(5)
    lib.ssnt_diag_step_clock(1, None)
    for _ in range(n):
        f(*gargs)
    calls = lib.ssnt_diag_step_clock(0, ph.ctypes.data)
    out["gpu_v1_phase_us"] = {k: float(v) for k, v in zip(
        ("context", "stage_in", "launch", "synchronise", "scatter"), ph)}
    out["gpu_v1_phase_calls"] = calls
    nl = np.zeros(2)
    lib.ssnt_diag_null_launch(n, nl.ctypes.data)
    out["null_kernel_launch_us"], out["null_kernel_sync_us"] = float(nl[0]), float(nl[1])
    return out


def main():
    with _lib.use_ab() as lib:  # the host staging / sync knobs are A/B-build symbols
        _main(lib)


def _main(lib):
    empty = per_call(lambda: lib.ssnt_status_from_bits(0), n=20000)
    res = {"empty_ctypes_call_us": empty}
    # v1 step, W=4, batch 1 (the reference symbol's fixed batch, ssnt_tts_c/src/lib.rs:13)
    c = dc.v1_case(1, B=1, W=4, max_t=80)
    v1 = lambda: capi.ssnt_tts_beam_search_decode(c["h"][0], c["hist"][0], c["fin"][0], c["t"][0],
                                                  c["u"][0], 80, 4)
    # v2 step, B=64 W=4 D=16 at I=400 O=2000
    c2 = dc.v2_case_long(2, 4, 16, B=64)
    c2["test_mode"] = True  # every call succeeds (no abort)
    v2 = lambda: capi.ssnt_tts_v2_beam_search_decode(
        c2["h"], c2["hist"], c2["fin"], c2["total"], c2["table"], c2["t"], c2["u"],
        c2["input_length"], np.zeros(64, np.int32), 64, 4, 16, 0, False, True)
    for mode in (0, 1):
        lib.ssnt_set_host_staging(mode)
        res[f"gpu_v1_W4_us_mode{mode}"] = per_call(v1)
        res[f"gpu_v2_B64_W4_D16_us_mode{mode}"] = per_call(v2, n=500)
    lib.ssnt_set_host_staging(1)
    res["cpu_v1_W4_us_per_call"] = per_call(
        lambda: O.v1_step(c["h"], c["hist"], c["fin"], c["t"], c["u"], c["input_length"]))
    res["cpu_v2_B64_us_per_call"] = per_call(
        lambda: O.v2_step(c2["h"], c2["hist"], c2["fin"], c2["total"], c2["table"], c2["t"],
                          c2["u"], c2["input_length"], np.zeros(64, np.int32), 0, False, True),
        n=500)
    res.update(raw_v1(lib, c))
    prev = lib.ssnt_set_host_sync(0)
    for mode in (0, 1, 2):  # completion: hipStreamSynchronize / hipStreamWriteValue32 / flag kernel
        lib.ssnt_set_host_sync(mode)
        r = raw_v1(lib, c, n=3000)
        res[f"sync{mode}_raw_gpu_v1_W4_us"] = r["raw_gpu_v1_W4_us"]
        res[f"sync{mode}_gpu_v1_phase_us"] = r["gpu_v1_phase_us"]
        res[f"sync{mode}_gpu_v1_W4_us_wrapped"] = per_call(v1)
        res[f"sync{mode}_gpu_v2_B64_W4_D16_us_wrapped"] = per_call(v2, n=500)
    lib.ssnt_set_host_sync(prev)
    big = {k: np.repeat(v, 4096, axis=0) if isinstance(v, np.ndarray) and v.ndim >= 1 else v
           for k, v in c.items()}
    t = per_call(lambda: O.v1_step(big["h"], big["hist"], big["fin"], big["t"], big["u"],
                                   big["input_length"]), n=20)
    res["cpu_v1_W4_us_per_step_amortised"] = t / 4096
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
