"""Ray-order experiment for the V2+V4 render: bench.py's render workload
(plenoxel 28x256^3, 16 x 2048 rays x 192 bins, one launch), rendered (a) with the library's
device-side order (Morton cell of the last sample, 8^3), (b) as given, and (c..) with the rays
permuted on the host by wider keys — a 6-D Morton code of (first sample cell, last sample cell)
at 2^b cells per axis — and rendered in that order (SFMHIP_RENDER_SORT=0).  Prints the median
kernel time of each and checks every ordering gives each ray the same colour bits."""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
N, B, S, NB = 256, 2048, 192, 16
vg = sfm.VoxelGrid.plenoxel(torch.randn((28, N, N, N), generator=g, device=dev) * 0.1, 1.5)
vg.voxel_major()
ro = torch.randn((NB * B, 3), generator=g, device=dev) * 0.2 + torch.tensor([0.0, 0.0, -3.0], device=dev)
rd = torch.randn((NB * B, 3), generator=g, device=dev) * 0.2 + torch.tensor([0.0, 0.0, 1.0], device=dev)
rd = rd / rd.norm(dim=1, keepdim=True)
t = torch.linspace(2.0, 6.0, S, device=dev).expand(NB * B, S)
mid = (t[:, :-1] + t[:, 1:]) / 2
u = torch.rand((NB * B, S), generator=g, device=dev)
z = (torch.cat([t[:, :1], mid], 1) + (torch.cat([mid, t[:, -1:]], 1) - torch.cat([t[:, :1], mid], 1)) * u).contiguous()


def cells(p, bits):
    n = 1 << bits
    c = ((p + 1.5) / 3.0 * n).floor().clamp(0, n - 1).long()
    return c


def morton(coords, bits):
    """interleave the bits of k coordinates (each < 2^bits), coordinate 0 lowest"""
    k = len(coords)
    key = torch.zeros_like(coords[0])
    for b in range(bits):
        for a, c in enumerate(coords):
            key |= ((c >> b) & 1) << (b * k + a)
    return key


def perm_key(bits, mode):
    p0 = ro + rd * z[:, :1]
    p1 = ro + rd * z[:, -1:]
    if mode == "entry+exit":
        c0, c1 = cells(p0, bits), cells(p1, bits)
        key = morton([c0[:, 0], c0[:, 1], c0[:, 2], c1[:, 0], c1[:, 1], c1[:, 2]], bits)
    elif mode == "mid+dir":     # the ray's centre point and direction
        pm = ro + rd * z[:, S // 2:S // 2 + 1]
        cm = cells(pm, bits)
        cd = ((rd + 1) / 2 * (1 << bits)).floor().clamp(0, (1 << bits) - 1).long()
        key = morton([cm[:, 0], cm[:, 1], cm[:, 2], cd[:, 0], cd[:, 1]], bits)
    else:
        raise ValueError(mode)
    return torch.argsort(key, stable=True)


def timed(fn, reps=10):
    fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts)), out


def setsort(v):
    os.environ["SFMHIP_RENDER_SORT"] = str(v)
    sfm.knobs_reload()


variants = [("device order (exit cell 8^3, shipped)", None, 1), ("as given", None, 0)]
for bits in (3, 4, 5, 6):
    variants.append((f"host: entry+exit cells 2^{bits}", ("entry+exit", bits), 0))
for bits in (4, 5, 6):
    variants.append((f"host: mid cell + direction 2^{bits}", ("mid+dir", bits), 0))
ref = None
for rnd in range(2):
    for name, key, srt in variants:
        setsort(srt)
        if key is None:
            ms, rgb = timed(lambda: vg.render(ro, rd, z))
        else:
            pm = perm_key(key[1], key[0])
            rop, rdp, zp = ro[pm].contiguous(), rd[pm].contiguous(), z[pm].contiguous()
            ms, rgbp = timed(lambda: vg.render(rop, rdp, zp))
            rgb = torch.empty_like(rgbp)
            rgb[pm] = rgbp
        if ref is None:
            ref = rgb.clone()
        same = torch.equal(rgb, ref)
        print(f"round {rnd}  {name:40s} {ms:.3f} ms  same bits: {same}", flush=True)
        assert same
setsort(1)
