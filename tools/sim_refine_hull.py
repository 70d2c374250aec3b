"""CPU study of the TSDF refinement test on C5 (a frame subset): for the wave
sub-tiles (8x2x8 voxels) that the interval-quotient footprint leaves
"projected", how many would an exact corner-hull footprint decide, and how many
need projecting at all (per-voxel truth: some voxel updates with tsdf < 1)?
Numbers are f64 approximations of the kernels' tests (statistics, not parity).
python tools/sim_refine_hull.py [n_frames]"""
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sbc = importlib.import_module("sim_brick_cull")

R, BLK = 256, 16
mu = 3 * 2.4 / (R - 1)
s = 2.4 / (R - 1)


class RangeTable:
    """2-D sparse table: min / max over any block rectangle in 4 lookups."""

    def __init__(self, a, op):
        self.op = op
        self.t = {}
        nv, nu = a.shape
        ky = 0
        row = a
        while (1 << ky) <= nv:
            kx, cur = 0, row
            while (1 << kx) <= nu:
                self.t[(ky, kx)] = cur
                h = 1 << kx
                if 2 * h > nu:
                    break
                cur = op(cur[:, :-h], cur[:, h:])
                kx += 1
            h = 1 << ky
            if 2 * h > nv:
                break
            row = op(row[:-h], row[h:])
            ky += 1

    def query(self, v0, v1, u0, u1):
        ky = np.floor(np.log2(v1 - v0 + 1)).astype(int)
        kx = np.floor(np.log2(u1 - u0 + 1)).astype(int)
        out = np.empty(len(v0))
        for key in set(zip(ky.tolist(), kx.tolist())):
            m = (ky == key[0]) & (kx == key[1])
            t = self.t[key]
            a, b = v0[m], v1[m] - (1 << key[0]) + 1
            c, d = u0[m], u1[m] - (1 << key[1]) + 1
            out[m] = self.op(self.op(t[a, c], t[a, d]), self.op(t[b, c], t[b, d]))
        return out


def decide_boxes(P, k, tmin, tmax, lo, hi, Hd, Wd, hull):
    """culled / free for boxes lo..hi (voxel index, x y z); hull: exact corner footprint."""
    ok, off, inside, u0, u1, v0, v1, zlo, zhi = sbc.footprint(P, k, lo, hi, Hd, Wd)
    if hull:
        cs = np.stack(np.meshgrid([0, 1], [0, 1], [0, 1], indexing="ij"), -1).reshape(-1, 3)
        corners = -1.2 + (lo[:, None, :] + cs[None] * (hi - lo)[:, None, :]) * s
        X = corners @ P[:, :3].T + P[:, 3]
        with np.errstate(divide="ignore", invalid="ignore"):
            u = k[0] * X[..., 0] / X[..., 2] + k[2] + 0.5
            v = k[1] * X[..., 1] / X[..., 2] + k[3] + 0.5
        m = 1e-3 + 1e-5 * np.abs(u).max(1)
        hu0, hu1 = np.floor(u.min(1) - m), np.floor(u.max(1) + m)
        hv0, hv1 = np.floor(v.min(1) - m), np.floor(v.max(1) + m)
        off = ok & ((hu1 < 0) | (hv1 < 0) | (hu0 >= Wd) | (hv0 >= Hd))
        inside = ok & (hu0 >= 0) & (hv0 >= 0) & (hu1 < Wd) & (hv1 < Hd)
        u0, u1 = np.clip(hu0, 0, Wd - 1), np.clip(hu1, 0, Wd - 1)
        v0, v1 = np.clip(hv0, 0, Hd - 1), np.clip(hv1, 0, Hd - 1)
    cul = off.copy()
    fre = np.zeros(len(lo), bool)
    q = ok & ~off
    bu0, bu1 = (u0[q] // BLK).astype(int), (u1[q] // BLK).astype(int)
    bv0, bv1 = (v0[q] // BLK).astype(int), (v1[q] // BLK).astype(int)
    small = (bu1 - bu0 + 1) * (bv1 - bv0 + 1) <= 256
    mx = tmax.query(bv0, bv1, bu0, bu1)
    mn = tmin.query(bv0, bv1, bu0, bu1)
    c = small & ((mx <= 0) | (mx + mu < zlo[q]))
    f = small & ~c & inside[q] & (mn - zhi[q] >= mu)
    cul[np.nonzero(q)[0][c]] = True
    fre[np.nonzero(q)[0][f]] = True
    return cul, fre


def truth(P, k, depth, lo, hi):
    """Per sub-tile: any voxel updating with tsdf < 1 (needs projection), any voxel updating."""
    g = np.stack(np.meshgrid(np.arange(8), np.arange(2), np.arange(8), indexing="ij"), -1).reshape(-1, 3)
    vox = lo[:, None, :] + g[None]
    w = -1.2 + vox * s
    X = w @ P[:, :3].T + P[:, 3]
    Hd, Wd = depth.shape
    with np.errstate(divide="ignore", invalid="ignore"):
        u = np.floor(k[0] * X[..., 0] / X[..., 2] + k[2] + 0.5)
        v = np.floor(k[1] * X[..., 1] / X[..., 2] + k[3] + 0.5)
    okp = (X[..., 2] > 0) & (u >= 0) & (v >= 0) & (u < Wd) & (v < Hd)
    d = np.zeros(u.shape)
    d[okp] = depth[v[okp].astype(int), u[okp].astype(int)]
    sdf = d - X[..., 2]
    upd = okp & (d > 0) & (sdf >= -mu)
    part = upd & (sdf < mu)
    return part.any(1), upd.any(1), (upd == okp).all(1) & upd.all(1)


def main():
    nf = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    idx = np.linspace(0, 256, nf).round().astype(int)
    # wave sub-tiles: x 8, y 2, z 8
    gx, gy, gz = np.meshgrid(np.arange(0, R, 8), np.arange(0, R, 2), np.arange(0, R, 8), indexing="ij")
    lo = np.stack([gx, gy, gz], -1).reshape(-1, 3)
    hi = lo + np.array([7, 1, 7])
    acc = np.zeros(5)
    for f in idx:
        depth, P, K = sbc._one_frame(f)
        Hd, Wd = depth.shape
        t = depth.reshape(Hd // BLK, BLK, Wd // BLK, BLK)
        tmax = RangeTable(t.max(axis=(1, 3)), np.maximum)
        tmin = RangeTable(t.min(axis=(1, 3)), np.minimum)
        c0, f0 = decide_boxes(P, K, tmin, tmax, lo, hi, Hd, Wd, hull=False)
        proj = ~(c0 | f0)
        sel = np.nonzero(proj)[0]
        c1, f1 = decide_boxes(P, K, tmin, tmax, lo[sel], hi[sel], Hd, Wd, hull=True)
        need, anyu, allfree = truth(P, K, depth, lo[sel], hi[sel])
        r = np.array([proj.mean(), (c1 | f1).mean(), need.mean(), (~anyu).mean(), allfree.mean()])
        acc += r
        print(f"frame {f}: projected {r[0]:.3f}; of those hull decides {r[1]:.3f}; truly need {r[2]:.3f} "
              f"(no voxel updates {r[3]:.3f})", flush=True)
    a = acc / len(idx)
    print(f"MEAN projected {a[0]:.3f}; hull decides {a[1]:.3f}; truly need projection {a[2]:.3f}; "
          f"no update at all {a[3]:.3f}")


if __name__ == "__main__":
    main()
