"""Why does adam_flagged_kernel slow down inside the bench sequence?  One mode
per fresh process (python tools/adam_probe.py MODE):
  fresh   the plenoxel training line's trainer in a fresh process
  after   after the bench's C3 match + C5 TSDF + render/vq buffers were made and freed
  trim    as 'after', then sfmhip_scratch_trim(0) before the trainer
  copy    as 'after', plus a plain torch copy over the trainer's buffers (placement, not kernel)
  warm    fresh, then ~1.5 s of back-to-back HBM copies right before the timed steps (clock ramp)
  sleep   as 'after', then 3 s of GPU idle before the timed steps
  iters   fresh, 200 timed steps instead of 10: does the time drift down as the process runs?
Prints the Adam kernel time (HIP events, median of 10) and a copy bandwidth."""
import importlib
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
tm = importlib.import_module("3d_reconstruction_amd.train")
mode = sys.argv[1] if len(sys.argv) > 1 else "fresh"
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)


def churn():
    x = syn.superpoint_like(257, 4096, 256, seed=1, device=dev)
    bank = sfm.DescriptorBank.from_float(x, mode=sfm.MODE_FLOAT)
    del x
    m = bank.match(sfm.all_pairs(257)[:4096])
    torch.cuda.synchronize()
    del bank, m
    torch.cuda.empty_cache()
    depth, poses, K = syn.tsdf_scene(257, syn.IMG_H, syn.IMG_W, device=dev)
    T = torch.zeros((256,) * 3, device=dev)
    W = torch.zeros_like(T)
    for _ in range(3):
        sfm.tsdf_integrate(T, W, depth, poses, K, (-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / 255)
    torch.cuda.synchronize()
    del depth, T, W
    torch.cuda.empty_cache()
    grid = torch.randn((28, 256, 256, 256), device=dev) * 0.1
    vg = sfm.VoxelGrid.plenoxel(grid, 1.5)
    vg.voxel_major()
    del grid, vg
    torch.cuda.empty_cache()


if mode in ("after", "trim", "copy", "sleep"):
    churn()
if mode == "trim":
    sfm.lib.sfmhip_scratch_trim(0)
N, B, S = 256, 2048, 192
g = torch.Generator(device=dev)
g.manual_seed(11)
tr = tm.GridTrainer.plenoxel(torch.ones((28, N, N, N), device=dev) / 100, 1.5, lr=1e-2)
torch.cuda.empty_cache()
ro = torch.randn((B, 3), generator=g, device=dev) * 0.2 + torch.tensor([0.0, 0.0, -3.0], device=dev)
rd = torch.randn((B, 3), generator=g, device=dev) * 0.2 + torch.tensor([0.0, 0.0, 1.0], device=dev)
rd = (rd / rd.norm(dim=1, keepdim=True)).contiguous()
t = torch.linspace(2.0, 6.0, S, device=dev).expand(B, S)
mid = (t[:, :-1] + t[:, 1:]) / 2
z = (torch.cat([t[:, :1], mid], 1) + (torch.cat([mid, t[:, -1:]], 1) - torch.cat([t[:, :1], mid], 1))
     * torch.rand((B, S), generator=g, device=dev)).contiguous()
gt = torch.rand((B, 3), generator=g, device=dev)
if mode == "warm":
    wa = torch.empty(256 << 20, device=dev)
    wb = torch.empty_like(wa)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.5:
        for _ in range(20):
            wb.copy_(wa)
        torch.cuda.synchronize()
    del wa, wb
if mode == "sleep":
    torch.cuda.synchronize()
    time.sleep(3.0)
ad = []
for k in range(202 if mode == "iters" else 12):
    tr._backward(ro, rd, gt, z)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    tr.optimizer_step()
    e1.record()
    torch.cuda.synchronize()
    ad.append(e0.elapsed_time(e1))
if mode == "iters":
    print("iters: first 20", [round(a, 2) for a in ad[:20]], "last 20", [round(a, 2) for a in ad[-20:]], flush=True)
ad = sorted(ad[2:])
cp = []
if mode == "copy":
    for buf in (tr.param, tr.exp_avg, tr.exp_avg_sq, tr.grad):
        tmp = torch.empty_like(buf)
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            tmp.copy_(buf)
            e1.record()
            torch.cuda.synchronize()
            cp.append(2 * buf.numel() * 4 / e0.elapsed_time(e1) / 1e6)
        del tmp
print(f"mode={mode} adam median {np.median(ad):.3f} ms min {ad[0]:.3f} max {ad[-1]:.3f}"
      + (f" copy GB/s {[round(c) for c in cp]}" if cp else ""), flush=True)
