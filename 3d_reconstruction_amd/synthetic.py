"""Synthetic workloads of BASELINE.json's configs (there is no network for the
real dataset's features or depth maps).  Generated with torch on any device
from a seed, so the same call gives the same data on CPU (tests / oracle) and
GPU (bench) up to the generator's device stream.

* C2: 64 images x 2048 SIFT-128 (integer values 0..255 stored as f32)
* C3/C4: 257 images x 4096 SuperPoint-256 (L2-normalised f32)
* BA/DLT scene: cameras on an orbit with the sfm.py camera (f = 2378.98305085,
  principal point 0), noisy observations of random 3D points per pair
* C5: 257 analytic depth maps (plane + spheres) 1936 x 1296 around a 256^3 grid
"""
from __future__ import annotations

import math

import numpy as np
import torch

FOCAL = 2378.98305085   # sfm.py:24
IMG_W, IMG_H = 1936, 1296


def _gen(device, seed):
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    return g


def _shared_indices(n_img, m, share, window, g, device):
    """Pool index of every (image, slot): own feature, or with prob ``share`` a
    random feature of an image within +-window (the overlap between views)."""
    k = torch.arange(n_img, device=device)[:, None].expand(n_img, m)
    s = torch.arange(m, device=device)[None, :].expand(n_img, m)
    own = k * m + s
    nb = (k + torch.randint(-window, window + 1, (n_img, m), generator=g, device=device)).clamp(0, n_img - 1)
    other = nb * m + torch.randint(0, m, (n_img, m), generator=g, device=device)
    pick = torch.rand((n_img, m), generator=g, device=device) < share
    return torch.where(pick, other, own)


def sift_like(n_img=64, m=2048, d=128, seed=0, share=0.4, window=3, noise=8.0, device="cpu"):
    """f32 (n_img, m, d) with integer values in 0..255 (config C2)."""
    g = _gen(device, seed)
    pool = torch.randint(0, 256, (n_img * m, d), generator=g, device=device, dtype=torch.int16).float()
    idx = _shared_indices(n_img, m, share, window, g, device)
    x = pool[idx] + noise * torch.randn((n_img, m, d), generator=g, device=device)
    return x.round_().clamp_(0, 255)


def superpoint_like(n_img=257, m=4096, d=256, seed=1, share=0.4, window=3, noise=0.08, device="cpu"):
    """L2-normalised f32 (n_img, m, d) (configs C3/C4)."""
    g = _gen(device, seed)
    pool = torch.randn((n_img * m, d), generator=g, device=device)
    pool = pool / pool.norm(dim=1, keepdim=True)
    idx = _shared_indices(n_img, m, share, window, g, device)
    x = pool[idx]
    x = x + noise * torch.randn(x.shape, generator=g, device=device) / math.sqrt(d)
    return x / x.norm(dim=-1, keepdim=True)


# ---------------------------------------------------------------------------
def _rodrigues_np(r):
    th = float(np.linalg.norm(r))
    if th < 1e-15:
        return np.eye(3)
    k = r / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + math.sin(th) * Kx + (1 - math.cos(th)) * Kx @ Kx


def _look_at(c, target=np.zeros(3), up=np.array([0.0, 1.0, 0.0])):
    """World->camera R, t for a camera at c looking at target (z forward)."""
    z = target - c
    z /= np.linalg.norm(z)
    x = np.cross(up, z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    R = np.stack([x, y, z])
    return R, -R @ c


def orbit_cameras(n, radius=4.0, height=0.6, seed=3):
    rng = np.random.default_rng(seed)
    Rs, ts = [], []
    for i in range(n):
        a = 2 * math.pi * i / n
        c = np.array([radius * math.cos(a), height + 0.2 * rng.standard_normal(), radius * math.sin(a)])
        R, t = _look_at(c)
        Rs.append(R)
        ts.append(t)
    return np.stack(Rs), np.stack(ts)


def ba_scene(n_pairs=256, n_obs=4096, seed=4, noise_px=0.5):
    """Per pair (i, i+1): P (n_pairs,2,3,4), x0/x1 (2,n) for DLT; and the BA
    inputs of sfm.py:36-38 for camera j: cam (n_pairs,6)=[rvec,t], K, X (n,3)
    (perturbed initial points), pts2d (n,2) (view j); pair_of_obs (n,)."""
    rng = np.random.default_rng(seed)
    Rs, ts = orbit_cameras(n_pairs + 1, seed=seed)
    K = np.array([[FOCAL, 0, 0], [0, FOCAL, 0], [0, 0, 1.0]])
    P = np.empty((n_pairs, 2, 3, 4))
    cam = np.empty((n_pairs, 6))
    n = n_pairs * n_obs
    X = rng.uniform(-1, 1, (n, 3))
    x0 = np.empty((2, n))
    x1 = np.empty((2, n))
    for p in range(n_pairs):
        sl = slice(p * n_obs, (p + 1) * n_obs)
        for v, cidx in enumerate((p, p + 1)):
            Rt = np.hstack([Rs[cidx], ts[cidx][:, None]])
            P[p, v] = K @ Rt
            Xh = np.hstack([X[sl], np.ones((n_obs, 1))])
            pr = (P[p, v] @ Xh.T)
            uv = pr[:2] / pr[2] + rng.normal(0, noise_px, (2, n_obs))
            (x0 if v == 0 else x1)[:, sl] = uv
        # rvec of R_{j}: inverse Rodrigues via axis-angle
        R = Rs[p + 1]
        ang = math.acos(max(-1.0, min(1.0, (np.trace(R) - 1) / 2)))
        if ang < 1e-12:
            rv = np.zeros(3)
        else:
            rv = ang / (2 * math.sin(ang)) * np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
        cam[p, :3] = rv
        cam[p, 3:] = ts[p + 1]
    pair_of_obs = np.repeat(np.arange(n_pairs, dtype=np.int32), n_obs)
    Xinit = X + rng.normal(0, 0.01, X.shape)
    Kb = np.broadcast_to(K, (n_pairs, 3, 3)).copy()
    return dict(P=P, x0=x0, x1=x1, cam=cam, K=Kb, X=Xinit, pts2d=x1.T.copy(), pair_of_obs=pair_of_obs)


def two_view_pairs(n_pairs=256, n_pts=2048, outlier_frac=0.3, noise_px=0.5, seed=6, step=1):
    """Matched keypoints for pairs (i, i+step) of an orbit, in the reference's
    centred pixel convention (K = diag(f, f, 1), matching.py:133): pts0/pts1
    lists of (n, 2) f32 (like m_kpts0/1, matching.py:126-127), a fraction
    ``outlier_frac`` replaced by random image points; also the true R, t
    (camera i -> camera i+step) and the inlier flags.  ``n_pts`` may be a
    per-pair sequence."""
    rng = np.random.default_rng(seed)
    Rs, ts = orbit_cameras(n_pairs + step, seed=seed)
    K = np.array([[FOCAL, 0, 0], [0, FOCAL, 0], [0, 0, 1.0]])
    sizes = np.broadcast_to(np.asarray(n_pts), (n_pairs,))
    out = dict(pts0=[], pts1=[], R=[], t=[], inlier=[], K=K)
    for p in range(n_pairs):
        n = int(sizes[p])
        X = rng.uniform(-1, 1, (n, 3))
        uv = []
        for c in (p, p + step):
            Xc = X @ Rs[c].T + ts[c]
            uv.append(Xc[:, :2] / Xc[:, 2:] * FOCAL + rng.normal(0, noise_px, (n, 2)))
        bad = rng.random(n) < outlier_frac
        uv[1][bad] = rng.uniform([-IMG_W / 2, -IMG_H / 2], [IMG_W / 2, IMG_H / 2], (int(bad.sum()), 2))
        out["pts0"].append(uv[0].astype(np.float32))
        out["pts1"].append(uv[1].astype(np.float32))
        R = Rs[p + step] @ Rs[p].T
        out["R"].append(R)
        out["t"].append(ts[p + step] - R @ ts[p])
        out["inlier"].append(~bad)
    return out


def sfm_scene(n_img=6, n_pts=800, noise_px=0.3, wrong_frac=0.08, seed=8):
    """Inputs of sfm.py's loop for a chain of pairs (0,1), (1,2), ...: every
    image sees every point (keypoints in a per-image random order, centred
    pixels, f32), all_matches[p] = [idx0, idx1, track ids] with a fraction of
    wrong correspondences, random colours."""
    rng = np.random.default_rng(seed)
    Rs, ts = orbit_cameras(4 * n_img, seed=seed)
    X = rng.uniform(-1, 1, (n_pts, 3))
    perm, pts = [], []
    for c in range(n_img):
        pm = rng.permutation(n_pts)
        Xc = X @ Rs[c].T + ts[c]
        uv = Xc[:, :2] / Xc[:, 2:] * FOCAL + rng.normal(0, noise_px, (n_pts, 2))
        kp = np.empty((n_pts, 2), np.float32)
        kp[pm] = uv                                   # keypoint pm[g] is point g
        pts.append(kp)
        perm.append(pm)
    img_pairs, all_matches = [], []
    for c in range(n_img - 1):
        g = rng.permutation(n_pts)[: int(0.9 * n_pts)]
        idx0, idx1 = perm[c][g], perm[c + 1][g].copy()
        wrong = rng.random(len(g)) < wrong_frac
        idx1[wrong] = rng.integers(0, n_pts, int(wrong.sum()))
        img_pairs.append((c, c + 1))
        all_matches.append([idx0.astype(np.int64), idx1.astype(np.int64), g.astype(np.int64)])
    colors = [rng.integers(0, 256, (n_pts, 3)).astype(np.uint8) for _ in range(n_img)]
    return dict(img_pairs=img_pairs, all_matches=all_matches, all_points=pts, all_colors=colors, X=X,
                R=Rs[:n_img], t=ts[:n_img])


# ---------------------------------------------------------------------------
SPHERES = ((0.0, -0.2, 0.0, 0.45), (0.5, 0.1, 0.3, 0.25), (-0.45, 0.0, -0.35, 0.3))
FLOOR_Y = -0.6


def tsdf_scene(n_frames=257, Hd=IMG_H, Wd=IMG_W, focal=FOCAL, radius=4.0, seed=5, device="cpu",
               chunk_rows=256):
    """Analytic depth maps (camera z of the first hit; 0 = miss) of a floor plane
    y = FLOOR_Y plus spheres, seen from an orbit.  Returns depth (F,Hd,Wd) f32,
    poses (F,3,4) f32 world->camera, K (F,4) f32 [fx, fy, cx, cy]."""
    Rs, ts = orbit_cameras(n_frames, radius=radius, seed=seed)
    poses = np.concatenate([Rs, ts[:, :, None]], 2).astype(np.float32)
    K = np.tile(np.array([[focal, focal, Wd / 2.0, Hd / 2.0]], np.float32), (n_frames, 1))
    depth = torch.empty((n_frames, Hd, Wd), dtype=torch.float32, device=device)
    us = torch.arange(Wd, device=device, dtype=torch.float32)
    for f in range(n_frames):
        R = torch.tensor(Rs[f], dtype=torch.float32, device=device)
        c = torch.tensor(-Rs[f].T @ ts[f], dtype=torch.float32, device=device)
        for r0 in range(0, Hd, chunk_rows):
            vs = torch.arange(r0, min(Hd, r0 + chunk_rows), device=device, dtype=torch.float32)
            dc = torch.stack(torch.broadcast_tensors((us[None, :] - Wd / 2.0) / focal,
                                                     (vs[:, None] - Hd / 2.0) / focal,
                                                     torch.ones(1, device=device)), -1)  # camera dir, z = 1
            dw = dc @ R  # world direction (R^T dc), z-component 1 in camera frame
            best = torch.full(dw.shape[:2], float("inf"), device=device)
            for (sx, sy, sz, sr) in SPHERES:
                oc = c - torch.tensor([sx, sy, sz], device=device)
                a = (dw * dw).sum(-1)
                b = 2 * (dw * oc).sum(-1)
                cc = float((oc * oc).sum() - sr * sr)
                disc = b * b - 4 * a * cc
                tt = (-b - torch.sqrt(disc.clamp_min(0))) / (2 * a)
                ok = (disc >= 0) & (tt > 0)
                best = torch.where(ok & (tt < best), tt, best)
            tp = (FLOOR_Y - c[1]) / dw[..., 1]
            okp = (tp > 0) & (dw[..., 1].abs() > 1e-9)
            best = torch.where(okp & (tp < best), tp, best)
            depth[f, r0:r0 + vs.shape[0]] = torch.where(torch.isfinite(best), best, torch.zeros_like(best))
    return depth, torch.from_numpy(poses).to(device), torch.from_numpy(K).to(device)
