"""CPU: the multi-GPU sharding path (pair ranges / z-slabs + one all-gather of
the match graph) exercised with the gloo backend, world_size 2 (and 3)."""
import importlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sdist = importlib.import_module("3d_reconstruction_amd.dist")


@pytest.mark.parametrize("n,world", [(32896, 8), (7, 3), (5, 8), (0, 2), (256, 4)])
def test_shard_range_partitions(n, world):
    seen = []
    sizes = []
    for r in range(world):
        lo, hi = sdist.shard_range(n, r, world)
        seen.extend(range(lo, hi))
        sizes.append(hi - lo)
    assert seen == list(range(n))
    assert max(sizes) - min(sizes) <= 1
    assert max(sizes) <= sdist.padded_shard(n, world)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        lo, hi = sdist.shard_range(n_total, rank, world)
        # rank r "matches" its pair range: rows filled with a function of the global pair id
        local = (torch.arange(lo, hi, dtype=torch.int32)[:, None] * 10 +
                 torch.arange(6, dtype=torch.int32)[None, :]).to(torch.int16)
        full = sdist.allgather_rows(local, n_total)
        exp = (torch.arange(n_total, dtype=torch.int32)[:, None] * 10 +
               torch.arange(6, dtype=torch.int32)[None, :]).to(torch.int16)
        q.put((rank, bool(torch.equal(full, exp))))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 11), (3, 10)])
def test_allgather_match_graph_gloo(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=60) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(v is True for v in res.values()), res


def test_zslab_shards_cover_grid():
    R = 256
    for world in (1, 2, 4, 8):
        slabs = [sdist.shard_range(R, r, world) for r in range(world)]
        assert slabs[0][0] == 0 and slabs[-1][1] == R
        assert all(slabs[i][1] == slabs[i + 1][0] for i in range(world - 1))



def _worker_overlap(rank, world, port, n_total, chunks, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)

        def compute(lo, hi, out):
            out.copy_((torch.arange(lo, hi, dtype=torch.int32)[:, None] * 10 +
                       torch.arange(6, dtype=torch.int32)[None, :]).to(torch.int16))

        full = sdist.overlapped_allgather(compute, n_total, (6,), torch.int16, "cpu", chunks=chunks)
        exp = (torch.arange(n_total, dtype=torch.int32)[:, None] * 10 +
               torch.arange(6, dtype=torch.int32)[None, :]).to(torch.int16)
        q.put((rank, bool(torch.equal(full, exp))))
    except Exception as e:
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world,n,chunks", [(2, 11, 4), (3, 100, 4), (2, 3, 4)])
def test_overlapped_allgather_gloo(world, n, chunks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_overlap, args=(r, world, port, n, chunks, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=60) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(v is True for v in res.values()), res


def test_chunk_rows_partition():
    for n, world, chunks in ((32896, 8, 4), (11, 2, 4), (3, 2, 4), (0, 2, 4)):
        rows = sorted(r for rk in range(world) for (lo, hi) in sdist.chunk_rows(n, rk, world, chunks)
                      for r in range(lo, hi))
        assert rows == list(range(n))


def _cpu_block_table(depth):
    from oracle import voxel as ov
    return torch.from_numpy(ov.block_table(depth.numpy()))


def _worker_table(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        g = torch.Generator().manual_seed(0)
        depth = torch.rand((7, 37, 50), generator=g) * 4 - 1
        depth[2, 5, 7] = float("nan")
        full = sdist.shared_block_table(depth, compute=_cpu_block_table)
        q.put((rank, bool(torch.equal(full, _cpu_block_table(depth)))))
    except Exception as e:
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_shared_block_table_gloo(world):
    """The TSDF block table assembled from per-rank frame ranges by one
    all-gather equals the single-process table."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_table, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=60) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(v is True for v in res.values()), res
