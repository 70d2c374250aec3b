"""Estimate, on the C5 scene, how the (tile, frame) pairs of the TSDF fusion
split into: culled (no voxel updates), free space (every voxel updates with
tsdf = 1, so no depth gather is needed) and full (gathers).  Exact per-voxel
classification plus the conservative 16x16-block test the cull kernel can do.
CPU only (torch), a sample of frames of the 257-frame orbit.

    python tools/sim_tsdf_free.py [n_sample_frames]
"""
import importlib
import sys

import numpy as np
import torch

syn = importlib.import_module("3d_reconstruction_amd.synthetic")

R, F, TILE, BLK = 256, 257, 8, 16
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
V = torch.stack([xx, yy, zz], -1).reshape(-1, 3).double()
tot = {"cull": 0, "free": 0, "full": 0, "free_cons": 0, "full_vox": 0, "full_vox_needs_depth": 0}
for i in range(ns):
    P = poses[i].double()
    Xc = V @ P[:, :3].T + P[:, 3]
    z = Xc[:, 2]
    u = torch.floor(K[i, 0] * Xc[:, 0] / z + K[i, 2] + 0.5)
    v = torch.floor(K[i, 1] * Xc[:, 1] / z + K[i, 3] + 0.5)
    inimg = (z > 0) & (u >= 0) & (u < Wd) & (v >= 0) & (v < Hd)
    ui, vi = u.clamp(0, Wd - 1).long(), v.clamp(0, Hd - 1).long()
    d = depth[i][vi, ui].double()
    sdf = d - z
    upd = inimg & (d > 0) & (sdf >= -mu)
    free = inimg & (d > 0) & (sdf >= mu)

    def tiles(a):
        a = a.reshape(R // TILE, TILE, R // TILE, TILE, R // TILE, TILE)
        return a.permute(0, 2, 4, 1, 3, 5).reshape(-1, TILE ** 3)

    tu, tf = tiles(upd), tiles(free)
    any_upd = tu.any(1)
    all_free = tf.all(1)
    tot["cull"] += int((~any_upd).sum())
    tot["free"] += int(all_free.sum())
    tot["full"] += int((any_upd & ~all_free).sum())
    # conservative: tile pixel bbox -> 16x16 blocks' min depth >= max Zc + mu, bbox inside the image
    bmin = -torch.nn.functional.max_pool2d(-depth[i][None, None], BLK, ceil_mode=True)[0, 0].double()
    ut, vt, zt = tiles(u), tiles(v), tiles(z)
    ok = tiles(inimg).all(1)
    u0, u1 = ut.min(1).values - 1, ut.max(1).values + 1
    v0, v1 = vt.min(1).values - 1, vt.max(1).values + 1
    ok &= (u0 >= 0) & (u1 < Wd) & (v0 >= 0) & (v1 < Hd)
    zmax = zt.max(1).values
    cons = torch.zeros_like(ok)
    for t in torch.nonzero(ok).flatten().tolist():
        b = bmin[int(v0[t]) // BLK:int(v1[t]) // BLK + 1, int(u0[t]) // BLK:int(u1[t]) // BLK + 1]
        cons[t] = bool((b.min() > 0) & (b.min() >= zmax[t] + mu * (1 + 2 ** -20)))
    tot["free_cons"] += int(cons.sum())
    # inside full tiles: per-voxel test against the pixel's 16x16 block min / max
    bmx = torch.nn.functional.max_pool2d(depth[i][None, None], BLK, ceil_mode=True)[0, 0].double()
    bi, bj = (vi // BLK), (ui // BLK)
    vmin, vmax = bmin[bi, bj], bmx[bi, bj]
    vfree = inimg & (vmin > 0) & (vmin - z >= mu)
    vcull = ~inimg | (vmax <= 0) | (vmax - z < -mu)
    need = ~(vfree | vcull)
    fullt = any_upd & ~cons
    tot["full_vox"] += int(fullt.sum()) * TILE ** 3
    tot["full_vox_needs_depth"] += int((tiles(need) & fullt[:, None]).sum())
    print(i, frames[i], {k: v for k, v in tot.items()}, flush=True)
n = ns * (R // TILE) ** 3
print({k: round(v / n, 3) for k, v in tot.items() if "vox" not in k})
print("voxels in non-free tiles needing a depth gather:", round(tot["full_vox_needs_depth"] / tot["full_vox"], 3))
