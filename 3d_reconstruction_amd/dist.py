"""Multi-GPU sharding (one process per GPU).

* matching: image pairs are independent -> contiguous balanced pair ranges per
  rank, descriptors replicated, then ONE all-gather of the fixed-size
  ``matches0`` block so every rank holds the full match graph
  (:func:`match_all_pairs_sharded`).  The collective is the C-ABI's RCCL
  all-gather (``sfmhip_allgather`` through :class:`RcclComm`, ncclAllGather
  over xGMI); torch.distributed is only the bootstrap (it broadcasts RCCL's
  unique id) and the fallback when no communicator is given (gloo in the CPU
  tests).
* TSDF: z-slabs [z0, z1) per rank; no exchange during fusion.  The fusion's
  pre-pass table ({min, max} of every 16x16 depth block, ~20 MB for C5) does
  not shrink with the slab (an orbiting camera sees most of any slab), so each
  rank computes the table of 1/N of the frames and one all-gather assembles it
  (:func:`shared_block_table`).  Slabs are cut by cost, not by thickness
  (:func:`plan_slabs` on :func:`voxel.tsdf_layer_stats`): the centre of an
  orbit scene carries more surface than its ends.
"""
from __future__ import annotations

import ctypes
import sys

import numpy as np
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


def graph_dtype(m_pad: int) -> torch.dtype:
    """Element type of the all-gathered match graph: int16 while every index
    (< m_pad) and the -1 sentinel fit, int32 beyond (no silent wrap)."""
    return torch.int16 if int(m_pad) <= 32767 else torch.int32


# ---------------------------------------------------------------------------
class RcclComm:
    """One rank's RCCL communicator from the C-ABI (``sfmhip_comm_init_rank``).

    ``RcclComm(group)`` bootstraps over a torch.distributed group: rank 0 makes
    the 128-byte unique id (``sfmhip_comm_unique_id``) and broadcasts it; every
    rank then joins on its current HIP device.  ``RcclComm.single()`` is a
    one-rank communicator (no torch.distributed).  ``allgather`` is
    ``sfmhip_allgather`` (ncclAllGather) on the given or current stream."""

    def __init__(self, group=None, _world=None, _rank=None, _uid=None):
        from ._abi import call
        self._call = call
        if _world is None:
            self.world = dist.get_world_size(group)
            self.rank = dist.get_rank(group)
            uid = ctypes.create_string_buffer(128)
            if self.rank == 0:
                call("sfmhip_comm_unique_id", uid)
            obj = [uid.raw]
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast_object_list(obj, src=src, group=group)
            uid = ctypes.create_string_buffer(obj[0], 128)
        else:
            self.world, self.rank, uid = int(_world), int(_rank), _uid
        h = ctypes.c_void_p()
        call("sfmhip_comm_init_rank", self.world, uid, self.rank, ctypes.byref(h))
        self.handle = h

    @classmethod
    def single(cls) -> "RcclComm":
        from ._abi import call
        uid = ctypes.create_string_buffer(128)
        call("sfmhip_comm_unique_id", uid)
        return cls(_world=1, _rank=0, _uid=uid)

    def allgather(self, send: torch.Tensor, recv: torch.Tensor, stream=None) -> None:
        """recv (world * send.numel() elements, rank order) <- every rank's send."""
        from ._abi import DT_OF, stream_ptr
        if recv.numel() != send.numel() * self.world or recv.dtype != send.dtype:
            raise ValueError("recv must hold world * send.numel() elements of send's dtype")
        if not (send.is_contiguous() and recv.is_contiguous()):
            raise ValueError("send and recv must be contiguous")
        st = stream.cuda_stream if isinstance(stream, torch.cuda.Stream) else (stream or stream_ptr())
        self._call("sfmhip_allgather", self.handle, send.data_ptr(), recv.data_ptr(), send.numel(),
                   DT_OF[send.dtype], st)

    def close(self) -> None:
        """Destroy the communicator once every collective it enqueued has
        finished: ``allgather`` returns without a host sync (the transfer runs on
        a side stream), so the device is synchronised first."""
        if self.handle is not None and self.handle.value:
            torch.cuda.synchronize()
            self._call("sfmhip_comm_destroy", self.handle)
        self.handle = None

    def __enter__(self) -> "RcclComm":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def __del__(self):
        # at interpreter shutdown the HIP runtime may already be gone: leave the
        # communicator to process exit rather than call into a torn-down runtime
        if sys.is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass


def _world_rank(group, comm):
    if comm is not None:
        return comm.world, comm.rank
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def _gather_bytes(send: torch.Tensor, recv: torch.Tensor, group, comm) -> None:
    """One all-gather of equal-size blocks: the RCCL comm, or torch.distributed
    (byte views: gloo has no int16; gloo with device tensors stages on the host)."""
    if comm is not None:
        comm.allgather(send.contiguous(), recv)
        return
    if recv.is_cuda and dist.get_backend(group) != "nccl":
        r = torch.empty(recv.shape, dtype=recv.dtype)
        dist.all_gather_into_tensor(r.view(-1).view(torch.uint8), send.cpu().contiguous().view(-1).view(torch.uint8),
                                    group=group)
        recv.copy_(r)
        return
    dist.all_gather_into_tensor(recv.view(-1).view(torch.uint8), send.contiguous().view(-1).view(torch.uint8),
                                group=group)


def allgather_rows(local: torch.Tensor, n_total: int, group=None, comm: RcclComm | None = None) -> torch.Tensor:
    """All-gather equal-size row blocks from every rank and trim the padding.

    ``local`` holds this rank's rows of a [n_total, ...] array split by
    :func:`shard_range`; returns the full array on every rank (one collective)."""
    world, rank = _world_rank(group, comm)
    per = padded_shard(n_total, world)
    lo, hi = shard_range(n_total, rank, world)
    if local.shape[0] != hi - lo:
        raise ValueError("local rows do not match this rank's shard")
    send = local
    if local.shape[0] < per:
        send = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        send[: local.shape[0]] = local
    recv = torch.empty((per * world,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    _gather_bytes(send, recv, group, comm)
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
                         after_compute=None, comm: RcclComm | None = None) -> torch.Tensor:
    """Compute this rank's rows chunk by chunk and all-gather each chunk while
    the next one computes (one collective per chunk on a side stream, so the
    match kernels and the RCCL transfers overlap on the GPU).

    ``compute(lo, hi, out)`` fills ``out`` (rows [lo, hi) of the global array,
    shape (hi-lo,) + row_shape) on the current stream; ``after_compute()`` (if
    given) runs once the last chunk is enqueued, before the collectives are
    waited for.  The collective is ``comm`` (the C-ABI RCCL all-gather) when
    given, else torch.distributed on ``group`` (RCCL via the nccl backend, or
    gloo with host staging for device tensors).  Returns the full (n,) +
    row_shape array on every rank, rows in global order."""
    world, rank = _world_rank(group, comm)
    per = -(-int(n) // (world * chunks)) if n else 0
    row_shape = tuple(row_shape)
    out = torch.empty((chunks * world * per,) + row_shape, dtype=dtype, device=device)
    side = out.is_cuda and (comm is not None or dist.get_backend(group) == "nccl")
    stream = torch.cuda.Stream(device=device) if side else None
    sends, works = [], []
    for c, (lo, hi) in enumerate(chunk_rows(n, rank, world, chunks)):
        send = torch.zeros((per,) + row_shape, dtype=dtype, device=device)
        if hi > lo:
            compute(lo, hi, send[: hi - lo])
        dst = out[c * world * per:(c + 1) * world * per]
        if side:
            ev = torch.cuda.Event()
            ev.record()
            stream.wait_event(ev)
            with torch.cuda.stream(stream):
                if comm is not None:
                    comm.allgather(send, dst, stream=stream)
                else:
                    works.append(dist.all_gather_into_tensor(dst.view(-1).view(torch.uint8),
                                                             send.view(-1).view(torch.uint8), group=group,
                                                             async_op=True))
            send.record_stream(stream)
        else:
            _gather_bytes(send, dst, group, None)
        sends.append(send)
    if after_compute is not None:
        after_compute()
    if side:
        out.record_stream(stream)
        for w in works:
            w.wait()            # the current stream waits for every chunk's collective
        done = torch.cuda.Event()
        done.record(stream)
        torch.cuda.current_stream(device).wait_event(done)
    del sends
    return out[:n]


def match_all_pairs_sharded(bank, pairs, ratio=0.75, exact=None, comm: RcclComm | None = None, group=None,
                            chunks: int | None = None, after_compute=None) -> torch.Tensor:
    """Exhaustive matching (matching.py:20,122-128 over every pair) sharded over
    the ranks: each rank matches its share of ``pairs`` with ``bank.match``
    and ONE all-gather per chunk (``chunks`` > 1: chunk c's transfer overlaps
    chunk c+1's matching) gives every rank the full ``matches0`` graph
    (P, m_pad), -1 = no match, in :func:`graph_dtype` (int16 while m_pad <=
    32767, else int32).  Collective: ``comm`` (C-ABI RCCL) if given, else
    torch.distributed on ``group``; with neither (or one rank) it is a local
    match.  ``after_compute`` runs once the last local launch is enqueued."""
    dvc = getattr(bank, "device", None) or bank.q.device
    pr = torch.as_tensor(np.asarray(pairs, np.int32) if not isinstance(pairs, torch.Tensor) else pairs,
                         dtype=torch.int32).to(dvc).reshape(-1, 2).contiguous()
    P, m_pad = int(pr.shape[0]), int(bank.m_pad)
    dt = graph_dtype(m_pad)
    world, rank = _world_rank(group, comm)
    if chunks is None:
        chunks = 4 if world > 1 else 1
    per = -(-P // (world * chunks)) if P else 0

    def compute(lo, hi, out):   # the kernels write the graph dtype (int16 / int32) in place
        bank.match(pr[lo:hi], ratio=ratio, out=out, exact=exact)

    if world == 1 and comm is None:
        full = torch.empty((P, m_pad), dtype=dt, device=dvc)
        for lo in range(0, P, max(per, 1)):
            hi = min(P, lo + per)
            compute(lo, hi, full[lo:hi])
        if after_compute is not None:
            after_compute()
        return full
    return overlapped_allgather(compute, P, (m_pad,), dt, dvc, chunks=chunks, group=group,
                                after_compute=after_compute, comm=comm)


# ---------------------------------------------------------------------------
def shared_block_table(depth: torch.Tensor, group=None, compute=None, comm: RcclComm | None = None) -> torch.Tensor:
    """The (F, ceil(Hd/16), ceil(Wd/16), 2) TSDF block table assembled across
    ranks: rank r computes the rows of its frame range (:func:`shard_range`)
    and one all-gather gives every rank the full table (bit-identical to a
    single-process table; pass it to ``tsdf_integrate(block_table=...)``).
    ``compute(depth_rows) -> table_rows`` defaults to the GPU kernel."""
    world, rank = _world_rank(group, comm)
    lo, hi = shard_range(depth.shape[0], rank, world)
    if compute is None:
        from .voxel import tsdf_block_table
        compute = tsdf_block_table
    return allgather_rows(compute(depth[lo:hi]), depth.shape[0], group, comm)


def allgather_slabs(local: torch.Tensor, slabs, group=None, comm: RcclComm | None = None) -> torch.Tensor:
    """Rebuild a z-sliced array from per-rank slabs of UNEQUAL thickness
    (:func:`plan_slabs`): rank r holds rows [z0_r, z1_r); one all-gather of
    blocks padded to the thickest slab, then the padding is dropped."""
    world, rank = _world_rank(group, comm)
    if len(slabs) != world:
        raise ValueError("one slab per rank")
    z0, z1 = slabs[rank]
    if local.shape[0] != z1 - z0:
        raise ValueError("local rows do not match this rank's slab")
    per = max(b - a for a, b in slabs)
    send = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    send[: local.shape[0]] = local
    recv = torch.empty((per * world,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    _gather_bytes(send, recv, group, comm)
    return torch.cat([recv[r * per: r * per + (b - a)] for r, (a, b) in enumerate(slabs)], 0)


def plan_slabs(layer_cost, world: int, layer: int = 8, depth: int | None = None) -> list[tuple[int, int]]:
    """Contiguous z-slabs [z0, z1) (multiples of ``layer`` voxels, the fusion's
    tile depth) minimising the largest summed ``layer_cost`` over ``world``
    ranks (exact: dynamic programme over the layer boundaries).  ``depth`` = D
    (the last slab ends there; default len(layer_cost) * layer)."""
    c = np.asarray(layer_cost, np.float64).ravel()
    L = len(c)
    D = L * layer if depth is None else int(depth)
    world = int(world)
    if world < 1:
        raise ValueError("world must be >= 1")
    pre = np.concatenate([[0.0], np.cumsum(c)])
    INF = float("inf")
    # best[k][j]: min over splits of layers [0, j) into k slabs of the max slab cost
    best = np.full((world + 1, L + 1), INF)
    cut = np.zeros((world + 1, L + 1), np.int64)
    best[0][0] = 0.0
    for k in range(1, world + 1):
        for j in range(0, L + 1):
            for i in range(0, j + 1):          # slab k covers layers [i, j) (may be empty)
                v = max(best[k - 1][i], pre[j] - pre[i])
                if v < best[k][j]:
                    best[k][j] = v
                    cut[k][j] = i
    bounds = [L]
    j = L
    for k in range(world, 0, -1):
        j = int(cut[k][j])
        bounds.append(j)
    bounds = bounds[::-1]
    return [(min(D, bounds[r] * layer), min(D, bounds[r + 1] * layer)) for r in range(world)]


def rebalance_slabs(slabs, times, depth: int, align: int = 1, fixed: float = 0.0) -> list[tuple[int, int]]:
    """Re-cut contiguous z-slabs from each rank's MEASURED fusion time (feedback
    balancing for repeated integrations of one scene: measure a call, re-cut,
    repeat).  Rank r's time minus ``fixed`` (the per-call cost that does not
    scale with thickness) is spread evenly over its layers; the cumulative cost
    over z is then cut at equal quantiles (``align`` > 1: the exact min-max
    partition at multiples of ``align`` voxels, :func:`plan_slabs`).
    Any cut gives the same grid (tiles start at z0 and culling is exact:
    tests/test_gpu_voxel.py, tests/test_dist.py); only the balance changes.
    The layer costs of an orbit scene vary by ~+-15 % over z, so
    2-3 rounds bring the slowest slab to the mean."""
    slabs = [(int(a), int(b)) for a, b in slabs]
    t = np.asarray(times, np.float64).ravel()
    world, D = len(slabs), int(depth)
    if len(t) != world or world < 1:
        raise ValueError("one time per slab")
    if slabs[0][0] != 0 or slabs[-1][1] != D or any(slabs[r][1] != slabs[r + 1][0] for r in range(world - 1)):
        raise ValueError("slabs must tile [0, depth) in order")
    dens = np.zeros(D, np.float64)
    for (a, b), tr in zip(slabs, t):
        if b > a:
            dens[a:b] = max(float(tr) - fixed, 1e-12) / (b - a)
    # an empty slab's layers have no measurement: give them the mean density of the measured ones
    meas = dens[dens > 0]
    dens[dens == 0] = meas.mean() if meas.size else 1.0
    if align > 1:   # coarse grid: the exact min-max partition of the aligned layers' costs
        L = -(-D // align)
        return plan_slabs([dens[i * align:(i + 1) * align].sum() for i in range(L)], world, layer=align, depth=D)
    cum = np.concatenate([[0.0], np.cumsum(dens)])
    cuts = [0]
    for r in range(1, world):
        z = int(np.searchsorted(cum, cum[-1] * r / world))
        # the nearer of the two layer boundaries around the quantile, on the align grid
        if z > 0 and cum[z] - cum[-1] * r / world > cum[-1] * r / world - cum[z - 1]:
            z -= 1
        cuts.append(min(max(z, cuts[-1]), D))
    cuts.append(D)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def allgather_times(t: float, group=None) -> list[float]:
    """Every rank's float (e.g. its measured slab time) on every rank, over the
    torch.distributed group (gloo or nccl; a host value, so a CPU tensor for
    gloo and a device tensor for nccl)."""
    world = dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    mine = torch.tensor([float(t)], dtype=torch.float64, device=dev)
    out = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(out, mine, group=group)
    return [float(x.item()) for x in out]
