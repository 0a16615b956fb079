#!/usr/bin/env python3
"""Benchmark: lattice forward-backward (loss + grad) throughput on N MI355X GPUs.

Workload (BASELINE.json configs[1], and configs[3] at N=8): per GPU B=256 utterances,
T=200 steps x U=80 positions, f32 log_trans (B,T,U,2) = log_softmax over {emit, shift} of
z ~ N(0, 1.5^2) (synthetic, generated on device, seed = rank). One step = one fused
fwd-bwd launch through the C-ABI (ssnt_fwd_bwd_sum_device) writing loss (B), grad (B,T,U,2)
and the shard's loss sum (formed in the same launch). The K timed steps are one HIP graph at
every N; for N > 1 the K per-step loss sums are all-reduced by one RCCL call over xGMI inside
the timed region (timed_region()).
Weak scaling: per-GPU work is fixed. value = all ranks' lattice cells / max-over-ranks time.

roofline: algorithmic HBM bytes of the fwd-bwd kernel = 16 B/cell (read 2xf32 log_trans, write
2xf32 grad) x cells per launch, over the kernel's average duration measured
with HIP events on the launch stream around the K back-to-back launches of the timed region
(so it includes the ~1 us gaps between launches); peak 8 TB/s (MI355X_MICROARCH.md).
traffic: HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc_traffic.py),
reported only when that summary was taken of the same kernel instance (ssnt_fwd_bwd_last_kernel),
built from the same sources (sha256 of csrc/ + header) on the same workload; null otherwise.
cpu_baseline: the C oracle (oracle/ssnt_oracle.c, same split-exponent arithmetic; the reference
has no forward-backward) on this host's cores, rank 0 at N=1 only.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "ssnt-tts-rust_amd"))

import ssnt_tts_amd as S  # noqa: E402

BASELINE = json.loads((ROOT / "BASELINE.json").read_text())
PEAK_HBM_GBS = 8000.0
BYTES_PER_CELL = 16


def synth(B, T, U, seed, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    z = torch.randn((B, T, U, 2), generator=g, device=dev, dtype=torch.float32) * 1.5
    return torch.log_softmax(z, dim=-1).contiguous()


def host_cpu_info():
    """The cores this process may run on: sched affinity, capped by a cgroup CPU quota when one
    is set (cpu.max); plus nproc and the CPU model string, so the baseline states its host."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    model = "unknown"
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"usable": usable, "affinity": aff, "nproc": os.cpu_count(), "cgroup_quota": quota,
            "model": model}


def cpu_baseline(B, T, U):
    """Time the C oracle on this host over every usable core (OpenMP over the batch, like the
    reference's rayon par_chunks): repeated full config-2 batches for ~10 s of wall time, plus
    a one-thread figure on a 16-utterance sample."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as O
    info = host_cpu_info()
    threads = info["usable"]
    lt = O.synth_log_trans(B, T, U, seed=0)
    sl, pl = [T] * B, [U] * B
    O.fwd_bwd_xf(lt, sl, pl, n_threads=threads)  # warm-up (first touch of every page)
    times = []
    t_end = time.perf_counter() + 10.0
    while len(times) < 5 or time.perf_counter() < t_end:
        t0 = time.perf_counter()
        O.fwd_bwd_xf(lt, sl, pl, n_threads=threads)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    t0 = time.perf_counter()
    O.fwd_bwd_xf(lt[:16], sl[:16], pl[:16], n_threads=1)
    single = 16 * T * U / (time.perf_counter() - t0)
    return {"value": B * T * U / med, "unit": "cells/s", "cores": threads, "kind": "port",
            "sample": f"{len(times)} x full B={B} T={T} U={U} fwd-bwd+grad batches "
                      f"(median {med * 1e3:.1f} ms/batch, {threads} OpenMP threads = every "
                      f"usable core); 1 thread: {single:.3e} cells/s",
            "single_thread_value": single, "host": info}


def kernel_source_sha():
    """sha256 over the kernel sources and the public header (what the .so is built from)."""
    import hashlib
    h = hashlib.sha256()
    files = sorted((ROOT / "ssnt-tts-rust_amd" / "csrc").glob("*")) + [ROOT / "include" / "ssnt_tts_c.h"]
    for f in files:
        if f.suffix in (".hip", ".h"):
            h.update(f.name.encode())
            h.update(f.read_bytes())
    return h.hexdigest()[:16]


def pmc_traffic(kernel, source_sha, B, T, U):
    """HBM bytes per launch from the committed PMC summary (tools/pmc_traffic.py), only when that
    summary was taken of the same kernel instance, built from the same sources, on the same
    workload as this run; else (None, why)."""
    p = ROOT / "profiles" / "pmc_fwd_bwd.json"
    if not p.exists():
        return None, "no PMC summary"
    try:
        d = json.loads(p.read_text())
    except ValueError:
        return None, "unreadable PMC summary"
    if d.get("dispatch") != kernel:
        return None, f"PMC summary is of {d.get('dispatch')!r}, this run dispatched {kernel!r}"
    if d.get("source_sha") != source_sha:
        return None, f"PMC summary taken at sources {d.get('source_sha')}, these are {source_sha}"
    if d.get("workload") != [B, T, U]:
        return None, f"PMC summary workload {d.get('workload')} != {[B, T, U]}"
    return d.get("hbm_bytes_per_launch"), f"profiles/{d.get('tag')}_fwd_bwd_summary.json"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256, help="utterances per GPU")
    ap.add_argument("--T", type=int, default=200)
    ap.add_argument("--U", type=int, default=80)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--variant", type=int, default=0, help="fwd-bwd kernel variant (A/B build, "
                    "include/ssnt_tts_c_ab.h): 0 the product's dispatch, 1 two-wave, 2 segmented")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL); gloo only to rehearse "
                    "the multi-rank path on a one-GPU box")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    local = local % max(1, torch.cuda.device_count())  # (rehearsal: several ranks on one GPU)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist:
        if args.dist_backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=dev)
        else:
            torch.distributed.init_process_group(args.dist_backend)

    B, T, U = args.batch, args.T, args.U
    if args.variant:  # every later call goes through the A/B build (never the bench default)
        S.use_ab().__enter__()
        assert S.load().ssnt_fwd_bwd_set_variant(args.variant) == 0
    lt = synth(B, T, U, seed=rank, dev=dev)
    sl = torch.full((B,), T, dtype=torch.int32, device=dev)
    pl = torch.full((B,), U, dtype=torch.int32, device=dev)
    out = {"loss": torch.empty(B, device=dev), "grad": torch.empty((B, T, U, 2), device=dev),
           "status": torch.zeros(1, dtype=torch.int32, device=dev),
           "loss_sum": torch.zeros(1, device=dev)}

    # correctness/status check once through the full Python mirror, outside the timed region
    r = S.ssnt_fwd_bwd(lt, sl, pl, out=out, check=True, loss_sum=True)
    kernel = S.last_fwd_bwd_kernel()  # the instance the timed launches dispatch (same shapes)
    assert torch.isfinite(r["loss"]).all()
    assert torch.isclose(r["loss_sum"], r["loss"].double().sum().float(), rtol=1e-5).all()

    # The timed loop calls the C ABI directly (pointers bound once). N=1 and N>1 run the same
    # loop: the K steps are one HIP graph of K launches (the host issues nothing per step), each
    # step writing its shard's loss sum into its own slot of `sums`; N>1 then all-reduces the K
    # per-step sums with one RCCL call inside the timed region.
    import ctypes
    lib = S.load()
    wsb = int(lib.ssnt_fwd_bwd_workspace_size(B, T, U))
    # in-launch loss-sum state: zeroed once, then maintained by the library
    sum_state = torch.zeros(int(lib.ssnt_fwd_bwd_sum_state_size(B)), dtype=torch.uint8, device=dev)
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    vp = ctypes.c_void_p
    K = args.steps
    sums = torch.zeros(K, device=dev)

    def launch(stream, k):
        rc = lib.ssnt_fwd_bwd_sum_device(
            vp(lt.data_ptr()), None, vp(sl.data_ptr()), vp(pl.data_ptr()), B, T, U, 1,
            vp(out["loss"].data_ptr()), vp(out["grad"].data_ptr()), None, None, None,
            vp(ws.data_ptr()) if wsb else None, wsb, None, vp(sums[k].data_ptr()),
            vp(sum_state.data_ptr()), vp(stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"ssnt_fwd_bwd_sum_device: {S.status_string(rc)}")

    main_stream = torch.cuda.current_stream(dev)
    for k in range(args.warmup):
        launch(main_stream, k % K)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(dev)
    with torch.cuda.graph(graph, stream=cap):
        for k in range(K):
            launch(cap, k)
    graph.replay()  # first replay uploads the graph (untimed)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def replay():
        e0.record(main_stream)
        graph.replay()
        e1.record(main_stream)

    reduce = (lambda x: torch.distributed.all_reduce(x)) if dist else None
    elapsed = timed_region(replay, sums, reduce, torch.cuda.synchronize,
                           torch.distributed.barrier if dist else None)
    # average kernel duration: the launch stream's events around the K back-to-back launches
    kern_ms = e0.elapsed_time(e1) / K
    if dist:
        t = torch.tensor([elapsed, kern_ms], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
        # every step's reduced sum is the global batch loss (one shard per rank)
        assert torch.isfinite(sums).all()
    per_step = None
    if dist:
        # The same K steps with one all-reduce of each step's loss sum right after it (RCCL on a
        # side stream, overlapped with the next step's kernel) -- the per-step synchronisation a
        # training loop that reduces every step's loss pays. Reported beside the headline, which
        # amortises one all-reduce of the K sums over the K graph-replayed steps.
        comm = torch.cuda.Stream(dev)
        evs = [torch.cuda.Event() for _ in range(K)]

        def step_k(k):
            launch(main_stream, k)
            evs[k].record(main_stream)
            comm.wait_event(evs[k])
            with torch.cuda.stream(comm):
                torch.distributed.all_reduce(sums[k:k + 1])

        ps = per_step_region(step_k, K, torch.cuda.synchronize, torch.distributed.barrier)
        t = torch.tensor([ps], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        per_step = float(t[0])
    if rank == 0:
        res = result_line(world, B, T, U, K, args.warmup, elapsed, kern_ms, dist, kernel)
        if per_step is not None:
            res["per_step_allreduce"] = {
                "ms_per_step": per_step / K * 1e3, "value": world * B * T * U * K / per_step,
                "unit": "cells/s",
                "note": "one RCCL all-reduce per step on a side stream, steps launched one by "
                        "one from the host (the headline value amortises one all-reduce of the "
                        "K per-step sums over a K-launch graph)"}
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(B, T, U)
        print(json.dumps(res), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


def timed_region(replay, sums, reduce, sync, barrier):
    """The timed region shared by every N: barrier + sync; replay() runs the K steps (one HIP
    graph on the GPU); N>1 all-reduces the K per-step loss sums once; sync + barrier. Returns
    the wall time in seconds (this rank's; the caller takes the max over ranks)."""
    if barrier:
        barrier()
    sync()
    t0 = time.perf_counter()
    replay()
    if reduce is not None:
        reduce(sums)
    sync()
    if barrier:
        barrier()
    return time.perf_counter() - t0


def per_step_region(step, K, sync, barrier):
    """K steps issued one by one, each with its own collective (step(k) launches step k and its
    all-reduce); barrier + sync on both sides. Returns this rank's wall time in seconds."""
    if barrier:
        barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(K):
        step(k)
    sync()
    if barrier:
        barrier()
    return time.perf_counter() - t0


def result_line(world, B, T, U, K, warmup, elapsed, kern_ms, dist, kernel=None):
    cells_step = world * B * T * U
    sha = kernel_source_sha()
    traffic, traffic_src = pmc_traffic(kernel, sha, B, T, U)
    value = cells_step * K / elapsed
    achieved = B * T * U * BYTES_PER_CELL / (kern_ms * 1e-3) / 1e9  # GB/s per GPU
    return {
        "metric": BASELINE["metric"],
        "value": value,
        "unit": "cells/s",
        "n_gpus": world,
        "steps": K,
        "warmup": warmup,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (log_softmax of N(0,1.5^2) logits, generated on device)",
        "config": {"workload": f"lattice fwd-bwd loss+grad, B={B}/GPU T={T} U={U} "
                               "(BASELINE configs[1]; configs[3] at N=8)",
                   "global_batch": world * B, "T": T, "U": U,
                   "parallelism": (f"batch-sharded x{world}, one RCCL all-reduce of the K "
                                   "per-step loss sums after the K-launch graph (amortised; "
                                   "per_step_allreduce: one per step)" if dist else "single GPU")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS,
                     "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": kernel, "source_sha": sha,
                     "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": B * T * U * BYTES_PER_CELL},
    }


if __name__ == "__main__":
    main()
