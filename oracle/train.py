"""Oracle for §8f row 4 (one grid training step).  TEST INFRASTRUCTURE ONLY.

The step of the reference's training loops — plenoxel.py:100-111 (train) and
sdf.py:427-438 (__main__):
    rgb = render_rays(model, rays_o, rays_d, ...)        # plenoxel.py:71-93 / SDFGrid.forward sdf.py:391-406
    loss = mse_loss(gt, rgb); optimizer.zero_grad(); loss.backward(); optimizer.step()
with torch.optim.Adam(lr=1e-2) (torch's single-tensor CPU path, torch/optim/adam.py).

* ``render_loss_grad`` — the forward of oracle.voxel.render plus the analytic
  backward of that graph w.r.t. the (C,D,H,W) grid: mse -> composite (the
  transmittance suffix recurrence V_{i-1} = a_i e_i + (1 - a_i) V_i) -> alpha =
  1 - exp(-sigma delta) -> relu -> SH basis -> grid_sample (ATen's
  grid_sampler_3d backward: the same 8 trilinear weights, scatter-add).
* ``adam_step`` — exp_avg.lerp_(g, 1-b1) (the vectorised CPU lerp is
  fmadd(w, g - m, m)), exp_avg_sq.mul_(b2).addcmul_(g, g, value=1-b2) (the
  vectorised addcmul is fmadd(value*g, g, v*b2)),
  denom = sqrt(v) / sqrt(1 - b2^t) + eps, p += (-lr / (1 - b1^t)) * m / denom.
Pinned by tests/golden/train_golden.npz (the reference's render_rays /
NerfModel + torch autograd + torch Adam on CPU).
"""
from __future__ import annotations

import math

import numpy as np

from .voxel import F32, grid_sample, normalise, sh_colour

SH_C = (0.282095, 0.488603, 1.092548, 0.315392, 0.546274)


def sh_basis(d) -> np.ndarray:
    """d (P,3) -> (P,9): the coefficient of k[..., m] in eval_spherical_function."""
    d = np.asarray(d, F32)
    x, y, z = d[:, 0], d[:, 1], d[:, 2]
    C0, C1, C2, C3, C4 = (F32(c) for c in SH_C)
    return np.stack([np.full_like(x, C0), (-C1) * y, C1 * z, -(C1 * x), (C2 * x) * y, -((C2 * y) * z),
                     C3 * (((F32(2.0) * z) * z - x * x) - y * y), ((-C2) * x) * z, C4 * (x * x - y * y)], 1)


def _corners(g, D, H, W):
    ix = ((g[:, 0] + F32(1)) / F32(2)) * F32(W - 1)
    iy = ((g[:, 1] + F32(1)) / F32(2)) * F32(H - 1)
    iz = ((g[:, 2] + F32(1)) / F32(2)) * F32(D - 1)
    fx, fy, fz = np.floor(ix), np.floor(iy), np.floor(iz)
    x1, y1, z1 = fx + F32(1), fy + F32(1), fz + F32(1)
    w = [(x1 - ix) * (y1 - iy) * (z1 - iz), (ix - fx) * (y1 - iy) * (z1 - iz),
         (x1 - ix) * (iy - fy) * (z1 - iz), (ix - fx) * (iy - fy) * (z1 - iz),
         (x1 - ix) * (y1 - iy) * (iz - fz), (ix - fx) * (y1 - iy) * (iz - fz),
         (x1 - ix) * (iy - fy) * (iz - fz), (ix - fx) * (iy - fy) * (iz - fz)]
    return fx.astype(np.int64), fy.astype(np.int64), fz.astype(np.int64), w


def render_loss_grad(grid, bmin, bmax, mask_mode, rays_o, rays_d, z, gt):
    """-> (loss, rgb (B,3), grad (C,D,H,W)) for mse_loss(gt, render(...))."""
    grid = np.asarray(grid, F32)
    if grid.ndim == 5:
        grid = grid[0]
    C, D, H, W = grid.shape
    o = np.asarray(rays_o, F32).reshape(-1, 3)
    d = np.asarray(rays_d, F32).reshape(-1, 3)
    z = np.asarray(z, F32)
    gt = np.asarray(gt, F32)
    B, S = z.shape
    pts = (o[:, None, :] + d[:, None, :] * z[:, :, None]).reshape(-1, 3)
    s = grid_sample(grid, pts, bmin, bmax, mask_mode)
    dd = np.repeat(d, S, 0)
    tmp0 = s[:, 0].reshape(B, S)
    col = sh_colour(s[:, 1:], dd).reshape(B, S, 3)
    sigma = np.maximum(tmp0, F32(0))
    delta = np.concatenate([z[:, 1:] - z[:, :-1], np.full((B, 1), F32(1e10))], 1)
    E = np.exp((-sigma) * delta).astype(F32)
    alpha = F32(1) - E
    T = np.cumprod(F32(1) - alpha, 1, dtype=F32)
    T = np.concatenate([np.ones((B, 1), F32), T[:, :-1]], 1)
    w = T * alpha
    rgb = (((w[:, :, None] * col).sum(1, dtype=F32) + F32(1)) - w.sum(-1, dtype=F32)[:, None]).astype(F32)
    diff = rgb - gt
    loss = float(np.mean(diff.astype(np.float64) ** 2))
    g = (F32(2.0 / (3 * B)) * diff).astype(F32)                         # dL/drgb
    e = ((col - F32(1)) * g[:, None, :]).sum(-1, dtype=F32)             # sum_ch g_ch (c_ch - 1)
    V = np.zeros((B, S), F32)
    acc = np.zeros(B, F32)
    for i in range(S - 1, -1, -1):                                       # V_i = sum_{k>i} ...
        V[:, i] = acc
        acc = alpha[:, i] * e[:, i] + (F32(1) - alpha[:, i]) * acc
    dalpha = T * (e - V)
    dsigma = (dalpha * E) * delta
    dtmp0 = np.where(tmp0 > 0, dsigma, F32(0)).astype(F32)
    dcol = w[:, :, None] * g[:, None, :]                                 # (B,S,3)
    basis = sh_basis(dd).reshape(B, S, 1, 9)
    dk = (dcol[:, :, :, None] * basis).reshape(B * S, 27)
    dtmp = np.concatenate([dtmp0.reshape(-1, 1), dk], 1).astype(F32)     # (P, 28)
    inside, gg = normalise(pts, bmin, bmax, mask_mode)
    grad = np.zeros((C, D, H, W), np.float64)
    bx, by, bz, wts = _corners(gg[inside], D, H, W)
    di = dtmp[inside].astype(np.float64)
    for k in range(8):
        x = bx + (k & 1)
        y = by + ((k >> 1) & 1)
        zz = bz + ((k >> 2) & 1)
        ok = (x >= 0) & (x < W) & (y >= 0) & (y < H) & (zz >= 0) & (zz < D)
        contrib = (wts[k][ok, None].astype(np.float64) * di[ok])       # (n_ok, C)
        for c in range(C):
            np.add.at(grad[c], (zz[ok], y[ok], x[ok]), contrib[:, c])
    return loss, rgb, grad.astype(F32)


def adam_step(param, grad, exp_avg, exp_avg_sq, step: int, lr: float = 1e-2, betas=(0.9, 0.999),
              eps: float = 1e-8):
    """torch.optim.Adam single-tensor step (step = the count after increment).
    Returns new (param, exp_avg, exp_avg_sq), all f32."""
    b1, b2 = betas
    p = np.asarray(param, F32)
    g = np.asarray(grad, F32)
    m = np.asarray(exp_avg, F32)
    v = np.asarray(exp_avg_sq, F32)
    w = F32(1 - b1)
    m = (m.astype(np.float64) + np.float64(w) * (g - m).astype(np.float64)).astype(F32)  # fmadd: one rounding
    # addcmul's vectorised CPU kernel: fmadd(value * t1, t2, self)
    v = ((F32(1 - b2) * g).astype(np.float64) * g.astype(np.float64) + (v * F32(b2)).astype(np.float64)).astype(F32)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    step_size = lr / bc1
    denom = (np.sqrt(v) / F32(math.sqrt(bc2)) + F32(eps)).astype(F32)
    p = (p + (F32(-step_size) * m) / denom).astype(F32)
    return p, m, v
