"""The N>1 path on CPU: world_size-2 gloo, the C oracle standing in for the GPU kernel. Checks
that sharding covers the batch exactly once and that the all-reduced loss equals the
single-process full-batch loss."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from ssnt_tts_amd.distributed import shard_bounds


@pytest.mark.parametrize("B,world", [(256, 2), (2048, 8), (7, 3), (1, 2), (0, 4)])
def test_shard_bounds_partition(B, world):
    cover = []
    for r in range(world):
        lo, hi = shard_bounds(B, world, r)
        cover.extend(range(lo, hi))
        assert hi - lo in (B // world, B // world + 1)
    assert cover == list(range(B))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "ssnt-tts-rust_amd"), str(root / "oracle")]
    import oracle as O
    from ssnt_tts_amd.distributed import sharded_fwd_bwd
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    lt = O.synth_log_trans(10, 30, 12, seed=5)
    sl = np.array([30, 29, 25, 30, 12, 18, 30, 27, 30, 22], np.int32)
    pl = np.array([12, 10, 12, 7, 12, 9, 12, 12, 3, 11], np.int32)

    def cpu_fwd_bwd(lt_, sl_, pl_):
        r = O.fwd_bwd_xf(np.asarray(lt_), np.asarray(sl_), np.asarray(pl_))
        return {"loss": torch.from_numpy(r["loss"]), "grad": r["grad"]}

    total, res, (lo, hi) = sharded_fwd_bwd(torch.from_numpy(lt), torch.from_numpy(sl),
                                           torch.from_numpy(pl), fwd_bwd=cpu_fwd_bwd)
    q.put((rank, float(total), lo, hi, res["grad"]))
    torch.distributed.destroy_process_group()


def test_gloo_world2_loss_allreduce():
    import oracle as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    lt = O.synth_log_trans(10, 30, 12, seed=5)
    sl = np.array([30, 29, 25, 30, 12, 18, 30, 27, 30, 22], np.int32)
    pl = np.array([12, 10, 12, 7, 12, 9, 12, 12, 3, 11], np.int32)
    full = O.fwd_bwd_xf(lt, sl, pl)
    want = float(np.sum(full["loss"], dtype=np.float32))
    for rank, total, lo, hi, grad in outs:
        assert abs(total - want) <= 1e-5 * max(1.0, abs(want))
        assert np.array_equal(grad, full["grad"][lo:hi])  # gradients stay local, unchanged


def _bench_worker(rank, world, port, q):
    """bench.py's multi-rank step logic (timed_region + result_line) with gloo; each rank's
    'replay' runs K steps of the C oracle on its shard and writes the per-step loss sums."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root), str(root / "ssnt-tts-rust_amd"), str(root / "oracle")]
    import bench
    import oracle as O
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    Bg, T, U, K = 8, 20, 6, 3
    lo, hi = shard_bounds(Bg, world, rank)
    lt = O.synth_log_trans(Bg, T, U, seed=11)[lo:hi]
    sums = torch.zeros(K)

    def replay():
        for k in range(K):
            sums[k] = float(O.fwd_bwd_xf(lt, [T] * (hi - lo), [U] * (hi - lo))["loss"].sum())

    elapsed = bench.timed_region(replay, sums, lambda x: torch.distributed.all_reduce(x),
                                 lambda: None, torch.distributed.barrier)
    sums2 = torch.zeros(K)

    def step_k(k):  # bench's per-step form: one step, then its own all-reduce
        sums2[k] = float(O.fwd_bwd_xf(lt, [T] * (hi - lo), [U] * (hi - lo))["loss"].sum())
        torch.distributed.all_reduce(sums2[k:k + 1])

    bench.per_step_region(step_k, K, lambda: None, torch.distributed.barrier)
    assert torch.equal(sums2, sums)  # the same reduced per-step sums either way
    t = torch.tensor([elapsed], dtype=torch.float64)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    line = bench.result_line(world, hi - lo, T, U, K, 0, float(t[0]), 0.01, True)
    q.put((rank, sums.numpy().copy(), line, float(t[0])))
    torch.distributed.destroy_process_group()


def test_gloo_world2_bench_step_logic():
    import oracle as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = O.fwd_bwd_xf(O.synth_log_trans(8, 20, 6, seed=11), [20] * 8, [6] * 8)["loss"]
    want = float(np.sum(full, dtype=np.float64))
    for rank, sums, line, elapsed in outs:
        assert np.allclose(sums, want, rtol=1e-5)  # every step: the global batch loss
        assert line["n_gpus"] == world and line["scaling"] == "weak"
        assert line["config"]["global_batch"] == 8
        assert abs(line["value"] - world * 4 * 20 * 6 * 3 / elapsed) < 1e-6 * line["value"]
