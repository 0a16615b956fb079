#!/usr/bin/env python3
"""Measure the BASELINE.json configs besides the headline (bench.py = configs[1]) on one GPU,
with the CPU oracle timed beside each (a bounded sample). One JSON line per config.

  configs[0]  single utterance T=50 U=20 fwd-bwd (the reference's CPU-sized case)
  configs[2]  fused v1 beam-search decode B=256 T=200 U=80 W=4 (+ best-beam backtrace)
  configs[4]  long form fwd-bwd B=64 T=2000 U=400; fused v2 decode B=64 I=400 O=2000 D=16 W=4
              and fused tone decode B=64 I=400 C=5 W=4 (+ every final slot's path)
GPU time: HIP events around `iters` back-to-back calls, median of 5 rounds (steady state).
"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
import oracle as O  # noqa: E402
import ssnt_tts_amd as S  # noqa: E402

DEV = torch.device("cuda:0")
sys.path.insert(0, str(ROOT))
from bench import host_cpu_info  # noqa: E402

HOST = host_cpu_info()
THREADS = HOST["usable"]  # every core this process may run on (affinity, cgroup quota)


def gpu_time(fn, iters, rounds=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / iters * 1e-3)
    return float(np.median(ts))


def cpu_time(fn, min_s=2.0):
    fn()
    ts, t_end = [], time.perf_counter() + min_s
    while len(ts) < 3 or time.perf_counter() < t_end:
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def fwd_bwd_config(name, B, T, U, iters, cpu_sample):
    lt_np = O.synth_log_trans(B, T, U, seed=0)
    lt = torch.from_numpy(lt_np).to(DEV)
    sl = torch.full((B,), T, dtype=torch.int32, device=DEV)
    pl = torch.full((B,), U, dtype=torch.int32, device=DEV)
    out = {"loss": torch.empty(B, device=DEV), "grad": torch.empty((B, T, U, 2), device=DEV),
           "status": torch.zeros(1, dtype=torch.int32, device=DEV)}
    S.ssnt_fwd_bwd(lt, sl, pl, out=out, check=True)
    t = gpu_time(lambda: S.ssnt_fwd_bwd(lt, sl, pl, out=out), iters)
    cells = B * T * U
    nb = min(B, cpu_sample)
    tc = cpu_time(lambda: O.fwd_bwd_xf(lt_np[:nb], [T] * nb, [U] * nb, n_threads=THREADS))
    return {"config": name, "workload": f"fwd-bwd loss+grad B={B} T={T} U={U}",
            "gpu_us": t * 1e6, "cells_per_s": cells / t,
            "algorithmic_GBps": cells * 16 / t / 1e9, "hbm_frac": cells * 16 / t / 8e12,
            "cpu_cells_per_s": nb * T * U / tc, "cpu_threads": THREADS,
            "cpu_sample": f"{nb} utterances"}


def decode_config(B, T, U, W, iters):
    lat_np = O.synth_log_trans(B, T, U, seed=3)
    lat = torch.from_numpy(lat_np).to(DEV)
    il_np = np.full(B, U, np.int32)
    il = torch.from_numpy(il_np).to(DEV)
    S.lattice_beam_search_decode(lat, il, W)
    t = gpu_time(lambda: S.lattice_beam_search_decode(lat, il, W, check=False), iters)
    tc = cpu_time(lambda: O.v1_lattice_decode(lat_np, il_np, W, n_threads=THREADS))
    steps = B * T * W
    return {"config": "configs[2]", "workload": f"fused v1 beam decode B={B} T={T} U={U} W={W} + backtrace",
            "gpu_us": t * 1e6, "beam_steps_per_s": steps / t,
            "cpu_beam_steps_per_s": steps / tc, "cpu_threads": THREADS,
            "note": "latency-bound integer/compare work: HBM fraction << 1% (6.6 MB per launch)"}


def v2_decode_config(B, I, Ototal, D, W, iters):
    """configs[4] v2 path: fused decode of I=400 steps over per-step logits peaked on a sampled
    duration path summing to O=2000, then every final slot's path + durations."""
    d = O.synth_durations(B, I, Ototal, D, seed=0)
    lg_np = O.synth_v2_logits(d, W, D, seed=100)
    table_np = np.arange(D, dtype=np.int32)
    il_np, ol_np = np.full(B, I, np.int32), np.full(B, Ototal, np.int32)
    lg, table = torch.from_numpy(lg_np).to(DEV), torch.from_numpy(table_np).to(DEV)
    il, ol = torch.from_numpy(il_np).to(DEV), torch.from_numpy(ol_np).to(DEV)
    S.v2_lattice_beam_search_decode(lg, table, il, ol, W, 0, False, False)  # checks status
    t = gpu_time(lambda: S.v2_lattice_beam_search_decode(lg, table, il, ol, W, 0, False, False,
                                                         check=False), iters)
    tc = cpu_time(lambda: O.v2_lattice_decode(lg_np, table_np, il_np, ol_np, 0, False, False,
                                              n_threads=THREADS))
    steps = B * I * W
    return {"config": "configs[4] v2", "workload": f"fused v2 decode B={B} I={I} O={Ototal} "
            f"D={D} W={W} + paths/durations", "gpu_us": t * 1e6, "beam_steps_per_s": steps / t,
            "cpu_beam_steps_per_s": steps / tc, "cpu_threads": THREADS,
            "note": f"{B} waves (one per utterance), {I} dependent steps of {W * D} candidates"}


def tone_decode_config(B, I, C, W, iters):
    lg_np = O.synth_tone_logits(B, I, W, C, seed=0)
    il_np = np.full(B, I, np.int32)
    lg, il = torch.from_numpy(lg_np).to(DEV), torch.from_numpy(il_np).to(DEV)
    S.tone_latent_lattice_beam_search_decode(lg, il, W, 0)
    t = gpu_time(lambda: S.tone_latent_lattice_beam_search_decode(lg, il, W, 0, check=False), iters)
    tc = cpu_time(lambda: O.tone_lattice_decode(lg_np, il_np, 0, n_threads=THREADS))
    steps = B * I * W
    return {"config": "configs[4] tone", "workload": f"fused tone decode B={B} I={I} C={C} W={W} "
            "+ paths", "gpu_us": t * 1e6, "beam_steps_per_s": steps / t,
            "cpu_beam_steps_per_s": steps / tc, "cpu_threads": THREADS}


def v2_fwd_bwd_config(B, I, Ototal, D, iters):
    """F4 at the configs[4] v2 shape: duration-class fwd-bwd, loss + grad."""
    d = O.synth_durations(B, I, Ototal, D, seed=0)
    lg_np = O.synth_v2_step_logits(d, D, seed=1)
    table_np = np.arange(D, dtype=np.int32)
    il_np, ol_np = np.full(B, I, np.int32), np.full(B, Ototal, np.int32)
    lg, table = torch.from_numpy(lg_np).to(DEV), torch.from_numpy(table_np).to(DEV)
    il, ol = torch.from_numpy(il_np).to(DEV), torch.from_numpy(ol_np).to(DEV)
    S.v2_fwd_bwd(lg, table, il, ol, 0, max_total=Ototal, check=True)
    t = gpu_time(lambda: S.v2_fwd_bwd(lg, table, il, ol, 0, max_total=Ototal), iters)
    tc = cpu_time(lambda: O.v2_fwd_bwd(lg_np, table_np, il_np, ol_np, Ototal, 0, False, False,
                                       n_threads=THREADS))
    return {"config": "configs[4] F4", "workload": f"v2 duration fwd-bwd B={B} I={I} O={Ototal} "
            f"D={D} loss+grad", "gpu_us": t * 1e6, "utterances_per_s": B / t,
            "cpu_utterances_per_s": B / tc, "cpu_threads": THREADS,
            "note": "one workgroup per utterance, 2 x I dependent steps over the band"}


if __name__ == "__main__":
    print(json.dumps(fwd_bwd_config("configs[0]", 1, 50, 20, iters=50, cpu_sample=1)), flush=True)
    print(json.dumps(decode_config(256, 200, 80, 4, iters=10)), flush=True)
    print(json.dumps(fwd_bwd_config("configs[4]", 64, 2000, 400, iters=3, cpu_sample=16)), flush=True)
    print(json.dumps(v2_decode_config(64, 400, 2000, 16, 4, iters=10)), flush=True)
    print(json.dumps(tone_decode_config(64, 400, 5, 4, iters=10)), flush=True)
    print(json.dumps(v2_fwd_bwd_config(64, 400, 2000, 16, iters=10)), flush=True)
    print(json.dumps({"host": HOST}), flush=True)
