"""Batch sharding across GPUs (one process per GPU, torch.distributed over RCCL).

Utterances are independent in both the forward-backward and the decode (the reference already
treats batch elements independently: rayon par_chunks, src/lib.rs:122-133), so a global batch
is split into contiguous shards, one per rank, with no data-path collective. The only exchange
is the scalar training loss: one all-reduce (sum) of the per-shard loss sum -- RCCL over xGMI on
MI355X, gloo on CPU in the tests. Gradients stay local to their shard.
"""
from __future__ import annotations

from typing import Callable

import torch


def shard_bounds(global_batch: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) shard of `global_batch` for `rank` (sizes differ by at most one)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, rem = divmod(global_batch, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def sharded_loss(per_utt_loss: torch.Tensor | None, group=None, average_over: int | None = None,
                 shard_sum: torch.Tensor | None = None):
    """Sum this shard's per-utterance losses and all-reduce the scalar across ranks.
    `shard_sum` (1,) is a shard sum already formed on device (the library's in-launch fixed-order
    sum, ssnt_fwd_bwd_sum_device); it is used as is instead of re-summing `per_utt_loss`.
    `average_over` (the global batch) turns the sum into the global mean."""
    if shard_sum is not None:
        total = shard_sum.reshape(1).to(torch.float32).clone()
    else:
        total = per_utt_loss.sum(dim=0, keepdim=True).to(torch.float32)
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        torch.distributed.all_reduce(total, op=torch.distributed.ReduceOp.SUM, group=group)
    if average_over:
        total = total / float(average_over)
    return total[0]


def sharded_fwd_bwd(log_trans_global, step_len_global, pos_len_global, *,
                    fwd_bwd: Callable | None = None, rank: int | None = None,
                    world: int | None = None, **kw):
    """Run the lattice forward-backward on this rank's shard of a global batch.

    `fwd_bwd(log_trans, step_len, pos_len, **kw) -> {"loss": (b,), "grad": ...}` defaults to
    the GPU kernel (ssnt_tts_amd.ssnt_fwd_bwd); tests plug in the CPU oracle.
    Returns (global_loss_sum, local_result, (lo, hi)).
    """
    if fwd_bwd is None:
        from . import ssnt_fwd_bwd as fwd_bwd
    if world is None:
        world = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
    if rank is None:
        rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
    lo, hi = shard_bounds(log_trans_global.shape[0], world, rank)
    res = fwd_bwd(log_trans_global[lo:hi], step_len_global[lo:hi], pos_len_global[lo:hi], **kw)
    loss = res["loss"]
    if not isinstance(loss, torch.Tensor):
        loss = torch.as_tensor(loss)
    shard_sum = res.get("loss_sum")  # (fwd_bwd called with loss_sum=True: formed in the launch)
    if shard_sum is not None and not isinstance(shard_sum, torch.Tensor):
        shard_sum = torch.as_tensor(shard_sum)
    return sharded_loss(loss, shard_sum=shard_sum), res, (lo, hi)
