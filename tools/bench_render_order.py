"""Render time vs ray order on bench.py's V2+V4 workload (plenoxel 28x256^3,
16 x 2048 rays x 192 bins): (1) the library's own ordering off (SFMHIP_RENDER_SORT=0) with
the rays permuted by torch argsort outside the timed region under several spatial keys;
(2) sfmhip_render_rays' device-side ordering (sort kernels inside the timed call) under
its env knobs.  Colours are checked identical per ray."""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(7)
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


def morton3(q):   # q (n,3) int in [0, 1024): 30-bit Morton code
    def spread(v):
        v = v & 0x3FF
        v = (v | (v << 16)) & 0x30000FF
        v = (v | (v << 8)) & 0x300F00F
        v = (v | (v << 4)) & 0x30C30C3
        v = (v | (v << 2)) & 0x9249249
        return v
    return spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)


def grid_q(p, bits):
    return ((p / 1.5 + 1) * 0.5 * (1 << bits)).clamp(0, (1 << bits) - 1).long()


def keys():
    out = {"given": None}
    pe = ro + rd * ((1.5 - ro[:, 2:3]) / rd[:, 2:3])
    q = ((pe[:, :2] + 3) * 32).clamp(0, 255).long()
    out["exit_xy"] = q[:, 1] * 256 + q[:, 0]
    for nm, s in (("first", 0), ("mid", S // 2), ("last", S - 1)):
        p = ro + rd * z[:, s:s + 1]
        for bits in (4, 6, 8):
            out[f"morton_{nm}_{bits}b"] = morton3(grid_q(p, bits))
    # midpoint of the in-box part of the samples
    p = ro[:, None, :] + rd[:, None, :] * z[:, :, None]
    inb = (p.abs() < 1.5).all(-1)
    cnt = inb.sum(1).clamp(min=1)
    pm = (p * inb[..., None]).sum(1) / cnt[:, None]
    for bits in (5, 7):
        out[f"morton_inbox_mid_{bits}b"] = morton3(grid_q(pm, bits))
    return out


os.environ["SFMHIP_RENDER_SORT"] = "0"
ref = vg.render(ro, rd, z)
res = {}


def timed(o2, d2, z2):
    ts = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        vg.render(o2, d2, z2)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


dev_cfgs = {"dev b3": {}, "dev b2": {"BITS": "2"}, "dev b4": {"BITS": "4"}, "dev b3 x2": {"XCHUNK": "2"},
            "dev b3 x8": {"XCHUNK": "8"}, "dev b3 s0": {"SIDX": "0"}, "dev b3 s191": {"SIDX": "191"}}
for rep in range(2):
    for nm, cfg in dev_cfgs.items():
        os.environ["SFMHIP_RENDER_SORT"] = "1"
        for k in ("BITS", "XCHUNK", "SIDX"):
            os.environ.pop("SFMHIP_RENDER_SORT_" + k, None)
        for k, v in cfg.items():
            os.environ["SFMHIP_RENDER_SORT_" + k] = v
        assert torch.equal(vg.render(ro, rd, z), ref), nm
        res.setdefault(nm, []).append(timed(ro, rd, z))
    os.environ["SFMHIP_RENDER_SORT"] = "0"
    for nm, key in keys().items():
        if key is None:
            perm = torch.arange(NB * B, device=dev)
        else:
            perm = torch.argsort(key, stable=True)
        o2, d2, z2 = ro[perm].contiguous(), rd[perm].contiguous(), z[perm].contiguous()
        out = vg.render(o2, d2, z2)
        assert torch.equal(out, ref[perm]), nm
        res.setdefault(nm, []).append(timed(o2, d2, z2))
for nm, v in res.items():
    print(f"{nm:24s} " + " ".join(f"{x:.3f}" for x in v) + " ms", flush=True)
