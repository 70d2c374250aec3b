"""GPU: the overlapped chunked all-gather of the match graph on RCCL (a
single-rank NCCL group on cuda:0 exercises the side-stream / async path the
multi-GPU bench uses; the multi-rank layout is covered with gloo in
test_dist.py)."""
import importlib
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu
sdist = importlib.import_module("3d_reconstruction_amd.dist")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_overlapped_allgather_nccl_single_rank(sfm, gpu):
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=gpu)
    try:
        syn = importlib.import_module("3d_reconstruction_amd.synthetic")
        x = syn.superpoint_like(6, 300, 128, seed=5, device=gpu)
        bank = sfm.DescriptorBank.from_float(x, mode=1, exact=False)
        pairs = torch.from_numpy(sfm.all_pairs(6)).to(gpu)
        P = pairs.shape[0]
        ref = bank.match(pairs.cpu().numpy(), ratio=0.75).to(torch.int16)
        buf = torch.empty((P, bank.m_pad), dtype=torch.int32, device=gpu)

        def compute(lo, hi, out):
            bank._launch(pairs[lo:hi], 3, 4, buf[lo:hi], None, None)
            out.copy_(buf[lo:hi])

        full = sdist.overlapped_allgather(compute, P, (bank.m_pad,), torch.int16, gpu, chunks=4)
        torch.cuda.synchronize()
        assert torch.equal(full, ref)
    finally:
        dist.destroy_process_group()
