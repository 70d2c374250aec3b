"""CPU simulation of a brick-level (32^3 voxel) cull pre-test in front of the
tile-level (8^3) test: what fraction of (brick, frame) pairs does the brick
test alone decide (culled / free space), and what fraction of tile tests would
that remove?  Same interval footprint as voxel.hip:box_footprint, on a frame
subset of the C5 scene.  python tools/sim_brick_cull.py [n_frames]"""
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
syn = importlib.import_module("3d_reconstruction_amd.synthetic")

NF = int(sys.argv[1]) if len(sys.argv) > 1 else 16
R, BLK = 256, 16
mn_b, mx_b = -1.2, 1.2
mu = 3 * 2.4 / (R - 1)
idx = np.linspace(0, 256, NF).round().astype(int)


def footprint(P, k, lo, hi, Hd, Wd):
    """Vectorised box_footprint over boxes lo/hi (n,3) voxel index ranges (x, y, z)."""
    s = (mx_b - mn_b) / (R - 1)
    c_w = mn_b + 0.5 * (lo + hi) * s
    h = 0.5 * (hi - lo) * s
    mw = np.abs(c_w) + h
    c = c_w @ P[:, :3].T + P[:, 3]
    e = h @ np.abs(P[:, :3]).T
    mag = mw @ np.abs(P[:, :3]).T + np.abs(P[:, 3])
    eps = 2.0 ** -24
    zlo = c[:, 2] - e[:, 2] - 8 * eps * mag[:, 2]
    zhi = c[:, 2] + e[:, 2] + 8 * eps * mag[:, 2]
    ok = zlo > 1e-3
    with np.errstate(divide="ignore", invalid="ignore"):
        izl, izh = 1 / zlo, 1 / zhi
        xl, xh = c[:, 0] - e[:, 0] - 8 * eps * mag[:, 0], c[:, 0] + e[:, 0] + 8 * eps * mag[:, 0]
        yl, yh = c[:, 1] - e[:, 1] - 8 * eps * mag[:, 1], c[:, 1] + e[:, 1] + 8 * eps * mag[:, 1]
        qx = np.stack([xl * izl, xl * izh, xh * izl, xh * izh])
        qy = np.stack([yl * izl, yl * izh, yh * izl, yh * izh])
    u0 = np.floor(k[0] * qx.min(0) + k[2] + 0.5 - 1e-3)
    u1 = np.floor(k[0] * qx.max(0) + k[2] + 0.5 + 1e-3)
    v0 = np.floor(k[1] * qy.min(0) + k[3] + 0.5 - 1e-3)
    v1 = np.floor(k[1] * qy.max(0) + k[3] + 0.5 + 1e-3)
    off = ok & ((u1 < 0) | (v1 < 0) | (u0 >= Wd) | (v0 >= Hd))
    inside = ok & (u0 >= 0) & (v0 >= 0) & (u1 < Wd) & (v1 < Hd)
    return ok, off, inside, np.clip(u0, 0, Wd - 1), np.clip(u1, 0, Wd - 1), np.clip(v0, 0, Hd - 1), \
        np.clip(v1, 0, Hd - 1), zlo, zhi


def decide(P, k, tab_min, tab_max, lo, hi, Hd, Wd, blk=BLK, cap=256):
    ok, off, inside, u0, u1, v0, v1, zlo, zhi = footprint(P, k, lo, hi, Hd, Wd)
    n = len(lo)
    cul = off.copy()
    fre = np.zeros(n, bool)
    for i in np.nonzero(ok & ~off)[0]:
        bu0, bu1, bv0, bv1 = int(u0[i]) // blk, int(u1[i]) // blk, int(v0[i]) // blk, int(v1[i]) // blk
        if (bu1 - bu0 + 1) * (bv1 - bv0 + 1) > cap:
            continue
        m = tab_max[bv0:bv1 + 1, bu0:bu1 + 1].max()
        mn = tab_min[bv0:bv1 + 1, bu0:bu1 + 1].min()
        if m <= 0 or m + mu < zlo[i]:
            cul[i] = True
        elif inside[i] and mn - zhi[i] >= mu:
            fre[i] = True
    return cul, fre


def boxes(edge):
    n = R // edge
    g = np.stack(np.meshgrid(np.arange(n), np.arange(n), np.arange(n), indexing="ij"), -1).reshape(-1, 3) * edge
    return g, g + edge - 1


def main():
    blo, bhi = boxes(32)
    tlo, thi = boxes(8)
    stats = np.zeros(6)
    for f in idx:
        depth, poses, K = _one_frame(f)
        Hd, Wd = depth.shape
        t = depth.reshape(Hd // BLK, BLK, Wd // BLK, BLK)
        tab_max = t.max(axis=(1, 3))
        tab_min = np.where(np.isnan(t), -np.inf, t).min(axis=(1, 3))
        bc, bf = decide(poses, K, tab_min, tab_max, blo, bhi, Hd, Wd)
        for cb, cap in ((4, 16), (4, 64), (8, 16), (8, 32)):
            nbv, nbu = tab_max.shape
            pv, pu = -nbv % cb, -nbu % cb
            cmax = np.pad(tab_max, ((0, pv), (0, pu)), constant_values=-np.inf)
            cmin = np.pad(tab_min, ((0, pv), (0, pu)), constant_values=np.inf)
            cmax = cmax.reshape(cmax.shape[0] // cb, cb, -1, cb).max(axis=(1, 3))
            cmin = cmin.reshape(cmin.shape[0] // cb, cb, -1, cb).min(axis=(1, 3))
            xc, xf = decide(poses, K, cmin, cmax, blo, bhi, Hd, Wd, blk=BLK * cb, cap=cap)
            print(f"   coarse x{cb} cap {cap}: culled {xc.mean():.3f} free {xf.mean():.3f}")
        # tile level: a sample of tiles, and every tile of the undecided bricks
        tc, tf = decide(poses, K, tab_min, tab_max, tlo, thi, Hd, Wd)
        brick_of_tile = ((tlo // 32) * np.array([64, 8, 1])).sum(1)
        und = ~(bc | bf)
        stats += [bc.mean(), bf.mean(), und.mean(), tc.mean(), tf.mean(), und[brick_of_tile].mean()]
        print(f"frame {f}: brick culled {bc.mean():.3f} free {bf.mean():.3f}; tile culled {tc.mean():.3f} "
              f"free {tf.mean():.3f}; tiles in undecided bricks {und[brick_of_tile].mean():.3f}", flush=True)
    s = stats / len(idx)
    print(f"MEAN brick culled {s[0]:.3f} free {s[1]:.3f} undecided {s[2]:.3f}; tile culled {s[3]:.3f} "
          f"free {s[4]:.3f}; tile tests left {s[5]:.3f}")


def _one_frame(f):
    """Frame f of syn.tsdf_scene(257) (same orbit and ray casting, one frame only)."""
    import torch
    Rs, ts = syn.orbit_cameras(257, radius=4.0, seed=5)
    Hd, Wd, fo = syn.IMG_H, syn.IMG_W, syn.FOCAL
    R = torch.tensor(Rs[f], dtype=torch.float32)
    c = torch.tensor(-Rs[f].T @ ts[f], dtype=torch.float32)
    us, vs = torch.arange(Wd, dtype=torch.float32), torch.arange(Hd, dtype=torch.float32)
    dc = torch.stack(torch.broadcast_tensors((us[None, :] - Wd / 2.0) / fo, (vs[:, None] - Hd / 2.0) / fo,
                                             torch.ones(1)), -1)
    dw = dc @ R
    best = torch.full(dw.shape[:2], float("inf"))
    for (sx, sy, sz, sr) in syn.SPHERES:
        oc = c - torch.tensor([sx, sy, sz])
        a = (dw * dw).sum(-1)
        b = 2 * (dw * oc).sum(-1)
        disc = b * b - 4 * a * float((oc * oc).sum() - sr * sr)
        tt = (-b - torch.sqrt(disc.clamp_min(0))) / (2 * a)
        best = torch.where((disc >= 0) & (tt > 0) & (tt < best), tt, best)
    tp = (syn.FLOOR_Y - c[1]) / dw[..., 1]
    best = torch.where((tp > 0) & (dw[..., 1].abs() > 1e-9) & (tp < best), tp, best)
    d = torch.where(torch.isfinite(best), best, torch.zeros_like(best)).numpy().astype(np.float64)
    P = np.concatenate([Rs[f], ts[f][:, None]], 1).astype(np.float32).astype(np.float64)
    return d, P, np.array([fo, fo, Wd / 2.0, Hd / 2.0], np.float32).astype(np.float64)


if __name__ == "__main__":
    main()
