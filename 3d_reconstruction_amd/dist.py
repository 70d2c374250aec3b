"""Multi-GPU sharding (one process per GPU, torch.distributed over RCCL/xGMI).

* matching: image pairs are independent -> contiguous balanced pair ranges per
  rank, descriptors replicated, then ONE all-gather of the fixed-size
  ``matches0`` block so every rank holds the full match graph.
* TSDF: z-slabs [z0, z1) per rank; no exchange during fusion.  The fusion's
  pre-pass table ({min, max} of every 16x16 depth block, ~20 MB for C5) does
  not shrink with the slab (an orbiting camera sees most of any slab), so each
  rank computes the table of 1/N of the frames and one all-gather assembles it
  (:func:`shared_block_table`) instead of every rank reading every depth map.
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


def chunk_rows(n: int, rank: int, world: int, chunks: int) -> list[tuple[int, int]]:
    """Global row ranges of ``rank`` under the chunk-major layout of
    :func:`overlapped_allgather`: chunk c covers rows [c*world*per,
    (c+1)*world*per) and rank r owns [c*world*per + r*per, ... + per) of it
    (clipped to n), with per = ceil(n / (world*chunks))."""
    per = -(-int(n) // (int(world) * int(chunks))) if n else 0
    out = []
    for c in range(chunks):
        lo = c * world * per + rank * per
        out.append((min(lo, n), min(lo + per, n)))
    return out


def overlapped_allgather(compute, n: int, row_shape, dtype, device, chunks: int = 4, group=None,
                         after_compute=None) -> torch.Tensor:
    """Compute this rank's rows chunk by chunk and all-gather each chunk while
    the next one computes (one collective per chunk on a side stream, so the
    match kernels and the RCCL transfers overlap on the GPU).

    ``compute(lo, hi, out)`` fills ``out`` (rows [lo, hi) of the global array,
    shape (hi-lo,) + row_shape) on the current stream; ``after_compute()`` (if
    given) runs once the last chunk is enqueued, before the collectives are
    waited for.  Returns the full (n,) + row_shape array on every rank, rows
    in global order."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    per = -(-int(n) // (world * chunks)) if n else 0
    row_shape = tuple(row_shape)
    out = torch.empty((chunks * world * per,) + row_shape, dtype=dtype, device=device)
    use_streams = out.is_cuda and dist.get_backend(group) == "nccl"
    comm = torch.cuda.Stream(device=device) if use_streams else None
    sends, works = [], []
    for c, (lo, hi) in enumerate(chunk_rows(n, rank, world, chunks)):
        send = torch.zeros((per,) + row_shape, dtype=dtype, device=device)
        if hi > lo:
            compute(lo, hi, send[: hi - lo])
        dst = out[c * world * per:(c + 1) * world * per]
        if use_streams:
            ev = torch.cuda.Event()
            ev.record()
            with torch.cuda.stream(comm):
                comm.wait_event(ev)
                works.append(dist.all_gather_into_tensor(dst.view(-1).view(torch.uint8),
                                                         send.view(-1).view(torch.uint8), group=group,
                                                         async_op=True))
        else:   # gloo (tests): byte view, host tensors
            dist.all_gather_into_tensor(dst.view(-1).view(torch.uint8), send.view(-1).view(torch.uint8),
                                        group=group)
        sends.append(send)
    if after_compute is not None:
        after_compute()
    for w in works:
        w.wait()            # the current stream waits for every chunk's collective
    del sends
    return out[:n]


def shared_block_table(depth: torch.Tensor, group=None, compute=None) -> torch.Tensor:
    """The (F, ceil(Hd/16), ceil(Wd/16), 2) TSDF block table assembled across
    ranks: rank r computes the rows of its frame range (:func:`shard_range`)
    and one all-gather gives every rank the full table (bit-identical to a
    single-process table; pass it to ``tsdf_integrate(block_table=...)``).
    ``compute(depth_rows) -> table_rows`` defaults to the GPU kernel."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard_range(depth.shape[0], rank, world)
    if compute is None:
        from .voxel import tsdf_block_table
        compute = tsdf_block_table
    return allgather_rows(compute(depth[lo:hi]), depth.shape[0], group)
