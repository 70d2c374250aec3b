"""Multi-GPU sharding (one process per GPU, torch.distributed over RCCL/xGMI).

* matching: image pairs are independent -> contiguous balanced pair ranges per
  rank, descriptors replicated, then ONE all-gather of the fixed-size
  ``matches0`` block so every rank holds the full match graph.
* TSDF: z-slabs [z0, z1) per rank; no exchange during fusion.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Balanced contiguous range [lo, hi) of n units for ``rank`` of ``world``."""
    base, extra = divmod(int(n), int(world))
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def padded_shard(n: int, world: int) -> int:
    """Per-rank row count of the all-gather buffer (ranks pad to equal size)."""
    return -(-int(n) // int(world))


def allgather_rows(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """All-gather equal-size row blocks from every rank and trim the padding.

    ``local`` holds this rank's rows of a [n_total, ...] array split by
    :func:`shard_range`; returns the full array on every rank (one collective)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    per = padded_shard(n_total, world)
    lo, hi = shard_range(n_total, rank, world)
    if local.shape[0] != hi - lo:
        raise ValueError("local rows do not match this rank's shard")
    send = local
    if local.shape[0] < per:
        send = torch.empty((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        send[: local.shape[0]] = local
    stage = local.is_cuda and dist.get_backend(group) == "gloo"   # gloo: host staging (tests only)
    if stage:
        send = send.cpu()
    recv = torch.empty((per * world,) + tuple(local.shape[1:]), dtype=local.dtype, device=send.device)
    # byte view: one collective for any dtype on any backend (gloo has no int16)
    dist.all_gather_into_tensor(recv.view(-1).view(torch.uint8), send.contiguous().view(-1).view(torch.uint8),
                                group=group)
    if stage:
        recv = recv.to(local.device)
    if n_total == per * world:
        return recv
    parts = []
    for r in range(world):
        rl, rh = shard_range(n_total, r, world)
        parts.append(recv[r * per: r * per + (rh - rl)])
    return torch.cat(parts, 0)
