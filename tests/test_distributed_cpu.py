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
