"""Is the plenoxel trainer's Adam time (fresh process ~2.6-3.0 ms, after other
allocations ~2.1 ms: tools/adam_probe.py) set by where its four 2 GiB state
buffers sit relative to each other?  Fresh process; the trainer's param / grad /
exp_avg / exp_avg_sq are re-homed into one allocation at offsets i * (2 GiB + delta)
for several deltas, and the Adam launch is timed on each layout (HIP events, median
of 10).  python tools/adam_layout_probe.py"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
tm = importlib.import_module("3d_reconstruction_amd.train")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
N, B, S = 256, 2048, 192
g = torch.Generator(device=dev)
g.manual_seed(11)
tr = tm.GridTrainer.plenoxel(torch.ones((28, N, N, N), device=dev) / 100, 1.5, lr=1e-2)
ro = torch.randn((B, 3), generator=g, device=dev) * 0.2 + torch.tensor([0.0, 0.0, -3.0], device=dev)
rd = torch.randn((B, 3), generator=g, device=dev) * 0.2 + torch.tensor([0.0, 0.0, 1.0], device=dev)
rd = (rd / rd.norm(dim=1, keepdim=True)).contiguous()
t = torch.linspace(2.0, 6.0, S, device=dev).expand(B, S)
mid = (t[:, :-1] + t[:, 1:]) / 2
z = (torch.cat([t[:, :1], mid], 1) + (torch.cat([mid, t[:, -1:]], 1) - torch.cat([t[:, :1], mid], 1))
     * torch.rand((B, S), generator=g, device=dev)).contiguous()
gt = torch.rand((B, 3), generator=g, device=dev)
names = ("param", "grad", "exp_avg", "exp_avg_sq")
print("fresh addresses:", " ".join(f"{n}={getattr(tr, n).data_ptr():#x}" for n in names), flush=True)


def time_adam(label):
    ad = []
    for k in range(12):
        tr._backward(ro, rd, gt, z)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        tr.optimizer_step()
        e1.record()
        torch.cuda.synchronize()
        ad.append(e0.elapsed_time(e1))
    ad = sorted(ad[2:])
    print(f"{label:34s} adam median {np.median(ad):.3f} ms min {ad[0]:.3f} max {ad[-1]:.3f}", flush=True)


time_adam("separate allocations (fresh)")
n = tr.param.numel()
nb = n * 4
host = {k: getattr(tr, k).cpu() for k in names}
for k in names:
    setattr(tr, k, None)
torch.cuda.empty_cache()
for delta in (0, 256, 4096, 65536, 1 << 20, 3 << 20, (1 << 20) + 4096, 33 << 20, 96 << 20):
    stride = nb + delta
    big = torch.empty(((4 * stride) // 4,), dtype=torch.float32, device=dev)
    for i, k in enumerate(names):
        v = big[i * stride // 4: i * stride // 4 + n].view(tr.touched.shape + (32,))
        v.copy_(host[k].to(dev))
        setattr(tr, k, v)
    time_adam(f"one buffer, delta {delta:#x}")
    for k in names:
        setattr(tr, k, None)
    del big, v
    torch.cuda.empty_cache()
