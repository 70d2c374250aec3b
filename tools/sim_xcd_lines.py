"""Per-XCD distinct depth lines of the TSDF fusion's gathers on the C5 scene, for the
super-brick -> XCD assignments the fusion could use: the round-robin deal (sb % 8) and
cost-balanced contiguous runs of a space-filling order.  Each XCD has its own L2, so a
line gathered by tiles of k XCDs in one frame is fetched at least k times: the sum over
XCDs of the per-frame distinct lines is the floor of the fusion's depth traffic for an
assignment.  CPU only (torch), a sample of frames of the 257-frame orbit.

    python tools/sim_xcd_lines.py [n_sample_frames]
"""
import importlib
import sys

import numpy as np
import torch

syn = importlib.import_module("3d_reconstruction_amd.synthetic")

R, F, BLK, NX = 256, 257, 16, 8
ns = int(sys.argv[1]) if len(sys.argv) > 1 else 6
frames = np.linspace(0, F - 1, ns).astype(int)
Rs, ts = syn.orbit_cameras(F, seed=5)
orig = syn.orbit_cameras
syn.orbit_cameras = lambda n, radius=4.0, seed=5: (Rs[frames], ts[frames])
depth, poses, K = syn.tsdf_scene(ns, seed=5)
syn.orbit_cameras = orig
Hd, Wd = depth.shape[1:]
mu = 3 * 2.4 / (R - 1)
g = torch.linspace(-1.2, 1.2, R)
zz, yy, xx = torch.meshgrid(g, g, g, indexing="ij")
V = torch.stack([xx, yy, zz], -1).reshape(-1, 3)
del zz, yy, xx
idx = torch.arange(R ** 3)
vx, vy, vz = idx % R, (idx // R) % R, idx // (R * R)
SBX, SBY, SBZ = 3 * 8, 2 * 8, 8 * 8          # super-brick in voxels
nsx, nsy, nsz = -(-R // SBX), -(-R // SBY), -(-R // SBZ)
sbx, sby, sbz = vx // SBX, vy // SBY, vz // SBZ
sb = sbx + nsx * (sby + nsy * sbz)
nsb = nsx * nsy * nsz
del idx, vx, vy, vz

# per frame: the voxels that gather and their 128-B line keys
need_sb, need_key = [], []
for i in range(ns):
    P = poses[i]
    Xc = V @ P[:, :3].T + P[:, 3]
    z = Xc[:, 2]
    u = torch.floor(K[i, 0] * Xc[:, 0] / z + K[i, 2] + 0.5)
    v = torch.floor(K[i, 1] * Xc[:, 1] / z + K[i, 3] + 0.5)
    ok = (z > 0) & (u >= 0) & (u < Wd) & (v >= 0) & (v < Hd)
    ui, vi = u[ok].long(), v[ok].long()
    zo = z[ok]
    d = depth[i]
    bmx = torch.nn.functional.max_pool2d(d[None, None], BLK, ceil_mode=True)[0, 0]
    bmn = -torch.nn.functional.max_pool2d(-d[None, None], BLK, ceil_mode=True)[0, 0]
    mx = bmx[vi // BLK, ui // BLK]
    mn = bmn[vi // BLK, ui // BLK]
    need = ~((mn > 0) & ((mn - zo) / mu >= 1)) & ~((mx <= 0) | (mx - zo < -mu))
    need_sb.append(sb[ok][need])
    need_key.append(vi[need] * ((Wd + 31) // 32) + ui[need] // 32)
cost = torch.zeros(nsb, dtype=torch.float64)
for s in need_sb:
    cost += torch.bincount(s, minlength=nsb).double()


def morton(coords, bits=5):
    out = torch.zeros_like(coords[0])
    for b in range(bits):
        for k, c in enumerate(coords):
            out |= ((c >> b) & 1) << (len(coords) * b + k)
    return out


def balanced(order):
    """class of each super-brick: 8 contiguous runs of `order` with equal cost"""
    c = cost[order]
    pre = torch.cumsum(c, 0) - c
    cls = torch.clamp((pre * NX / c.sum()).long(), max=NX - 1)
    out = torch.empty(nsb, dtype=torch.long)
    out[order] = cls
    return out


ib = torch.arange(nsb)
bx, by, bz = ib % nsx, (ib // nsx) % nsy, ib // (nsx * nsy)
assign = {
    "round-robin sb % 8 (current)": ib % NX,
    "morton xyz, cost-balanced": balanced(torch.argsort(morton([bx, by, bz]))),
    "morton xz then y, cost-balanced": balanced(torch.argsort(morton([bx, bz]) * nsy + by)),
    "x-major rows, cost-balanced": balanced(torch.argsort(bx * nsz * nsy + bz * nsy + by)),
}
s = F / ns
tot_lines = sum(k.unique().numel() for k in need_key)
print(f"distinct 128-B lines per call (one fetch per line and frame): {tot_lines * s * 128 / 1e9:.2f} GB")
for name, cls in assign.items():
    lines = 0
    for sbs, keys in zip(need_sb, need_key):
        c = cls[sbs]
        lines += sum(keys[c == x].unique().numel() for x in range(NX))
    load = torch.bincount(cls, weights=cost, minlength=NX)
    print(f"{name:34s}: per-XCD lines {lines * s * 128 / 1e9:.2f} GB ({lines / tot_lines:.2f}x), "
          f"gather-cost max/mean over XCDs {float(load.max() / load.mean()):.2f}", flush=True)
