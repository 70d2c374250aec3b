"""Oracle for V1-V5 (voxel path).  TEST INFRASTRUCTURE ONLY.

float32 restatements with the reference's op order:
  voxel_traversal  voxel_travesal.py:1-73 (torch.floor_divide = Python floor
                   division: c10::div_floor_floating; same in numpy's npy_divmod)
  grid_sample      sdf.py:284-342 / plenoxel.py:31-43 -> ATen grid_sampler_3d
                   (bilinear, zeros padding, align_corners=True)
  sh_colour        sdf.py:361-369 / plenoxel.py:9-16
  composite        sdf.py:391-406 / plenoxel.py:71-93
  tsdf_integrate   build-defined, parity unpinned; order-free
                   fixed-point fusion (tsdf_integrate_seq: the sequential form).
  block_table      the TSDF pre-pass table (build-defined): {min, max} per 16x16
                   depth block, min poisoned by NaN, max ignoring NaN.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


# ---------------------------------------------------------------------------
def voxel_traversal(rays: np.ndarray, bin_size: float) -> np.ndarray:
    """(N,8) f32 -> (N,S,3) f32, synchronous-loop semantics of the reference."""
    r = np.asarray(rays, F32)
    b = F32(bin_size)
    o, d, near, far = r[:, :3], r[:, 3:6], r[:, 6:7], r[:, 7:8]
    start = o + d * near
    end = o + d * far
    cur = np.floor_divide(start, b)
    last = np.floor_divide(end, b)
    step = np.where(d < 0, F32(-1), F32(1)).astype(F32)
    nvb = (cur + step) * b
    with np.errstate(divide="ignore", invalid="ignore"):
        tmax = ((nvb - start) / d).astype(F32)
        tdelta = ((step * b) / d).astype(F32)
    tmax[d == 0] = np.inf
    tdelta[d == 0] = np.inf

    def active(c):
        with np.errstate(invalid="ignore"):
            return np.any((c == c) & (step * c < step * last), axis=1)

    out = [cur.copy()]
    m = active(cur)
    guard = 0
    while m.any():
        tx, ty, tz = tmax[:, 0], tmax[:, 1], tmax[:, 2]
        with np.errstate(invalid="ignore"):
            mx = (tx < ty) & (tx < tz) & m
            my = (ty <= tx) & (ty < tz) & m
            mz = (((tx >= ty) & (ty >= tz)) | ((tx >= tz) & (ty > tx))) & m
        for a, ma in ((0, mx), (1, my), (2, mz)):
            cur[ma, a] = cur[ma, a] + step[ma, a]
            tmax[ma, a] = tmax[ma, a] + tdelta[ma, a]
        out.append(cur.copy())
        m = active(cur)
        cur[~m] = np.nan
        guard += 1
        if guard > 1 << 20:
            raise RuntimeError("voxel_traversal oracle: runaway loop")
    return np.stack(out, 1)


# ---------------------------------------------------------------------------
def normalise(pts, bmin, bmax, mask_mode):
    p = np.asarray(pts, F32).reshape(-1, 3)
    mn = np.asarray(bmin, F32).ravel()
    mx = np.asarray(bmax, F32).ravel()
    if mask_mode == 0:
        inside = np.all(p >= mn, 1) & np.all(p <= mx, 1)
        g = ((p - mn) / (mx - mn)) * F32(2) - F32(1)
    else:
        s = mx[0]
        inside = np.all(np.abs(p) < s, 1)
        g = np.clip(p / s, F32(-1), F32(1))
    return inside, g.astype(F32)


def grid_sample(grid, pts, bmin, bmax, mask_mode=0) -> np.ndarray:
    """grid (C,D,H,W) f32 -> (P,C); zero outside the mask."""
    grid = np.asarray(grid, F32)
    if grid.ndim == 5:
        grid = grid[0]
    C, D, H, W = grid.shape
    inside, g = normalise(pts, bmin, bmax, mask_mode)
    P = g.shape[0]
    out = np.zeros((P, C), F32)
    gi = g[inside]
    ix = ((gi[:, 0] + F32(1)) / F32(2)) * F32(W - 1)
    iy = ((gi[:, 1] + F32(1)) / F32(2)) * F32(H - 1)
    iz = ((gi[:, 2] + F32(1)) / F32(2)) * F32(D - 1)
    fx, fy, fz = np.floor(ix), np.floor(iy), np.floor(iz)
    x1, y1, z1 = fx + F32(1), fy + F32(1), fz + F32(1)
    w = [
        (x1 - ix) * (y1 - iy) * (z1 - iz),
        (ix - fx) * (y1 - iy) * (z1 - iz),
        (x1 - ix) * (iy - fy) * (z1 - iz),
        (ix - fx) * (iy - fy) * (z1 - iz),
        (x1 - ix) * (y1 - iy) * (iz - fz),
        (ix - fx) * (y1 - iy) * (iz - fz),
        (x1 - ix) * (iy - fy) * (iz - fz),
        (ix - fx) * (iy - fy) * (iz - fz),
    ]
    acc = np.zeros((gi.shape[0], C), F32)
    bx, by, bz = fx.astype(np.int64), fy.astype(np.int64), fz.astype(np.int64)
    for k in range(8):
        x = bx + (k & 1)
        y = by + ((k >> 1) & 1)
        z = bz + ((k >> 2) & 1)
        ok = (x >= 0) & (x < W) & (y >= 0) & (y < H) & (z >= 0) & (z < D)
        v = np.zeros((gi.shape[0], C), F32)
        v[ok] = grid[:, z[ok], y[ok], x[ok]].T
        acc = np.where(ok[:, None], acc + v * w[k][:, None], acc).astype(F32)
    out[inside] = acc
    return out


def sh_colour(k, d) -> np.ndarray:
    """sdf.py:361-369: k (P,27) as (P,3,9), d (P,3) -> (P,3), Python op order."""
    k = np.asarray(k, F32).reshape(-1, 3, 9)
    d = np.asarray(d, F32).reshape(-1, 3)
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    C0, C1, C2, C3, C4 = F32(0.282095), F32(0.488603), F32(1.092548), F32(0.315392), F32(0.546274)
    kk = [k[..., m] for m in range(9)]
    inner = ((((C2 * x) * y) * kk[4] - ((C2 * y) * z) * kk[5])
             + (C3 * (((F32(2.0) * z) * z - x * x) - y * y)) * kk[6]) + (((-C2) * x) * z) * kk[7]
    inner2 = inner + (C4 * (x * x - y * y)) * kk[8]
    return ((((C0 * kk[0] + ((-C1) * y) * kk[1]) + (C1 * z) * kk[2]) - (C1 * x) * kk[3]) + inner2).astype(F32)


def render(grid, bmin, bmax, mask_mode, rays_o, rays_d, z) -> np.ndarray:
    """Sample + SH colour + composite (sdf.py:391-406): (B,3)."""
    o = np.asarray(rays_o, F32).reshape(-1, 3)
    d = np.asarray(rays_d, F32).reshape(-1, 3)
    z = np.asarray(z, F32)
    B, S = z.shape
    pts = o[:, None, :] + d[:, None, :] * z[:, :, None]
    s = grid_sample(grid, pts.reshape(-1, 3), bmin, bmax, mask_mode)
    sdf = s[:, 0].reshape(B, S)
    col = sh_colour(s[:, 1:], np.repeat(d, S, 0)).reshape(B, S, 3)
    sigma = np.maximum(sdf, F32(0))
    delta = np.concatenate([z[:, 1:] - z[:, :-1], np.full((B, 1), F32(1e10))], 1)
    alpha = F32(1) - np.exp((-sigma) * delta).astype(F32)
    T = np.cumprod(F32(1) - alpha, 1, dtype=F32)
    T = np.concatenate([np.ones((B, 1), F32), T[:, :-1]], 1)
    w = (T * alpha)[:, :, None]
    c = (w * col).sum(1, dtype=F32)
    ws = w.sum(-1).sum(-1, dtype=F32)
    return ((c + F32(1)) - ws[:, None]).astype(F32)


# ---------------------------------------------------------------------------
TSDF_STEP = 512        # frames per integration step (tsdf.hip kTsdfMaxFrames)
TSDF_QBITS = 21        # tsdf fixed point (tsdf.hip kTsdfQBits)


def _tsdf_frames(Ts, Ws, depth, poses, K, bmin, bmax, trunc, z0, z1, D, step):
    """Per frame: (ok, ts) of every voxel of the slab [z0, z1) -- the projection and skip
    rules of the definition, every f32 op one IEEE RN step in the order written."""
    Dz, H, W = Ts.shape
    mn = np.asarray(bmin, F32).ravel()
    mx = np.asarray(bmax, F32).ravel()
    sx = (mx[0] - mn[0]) / F32(W - 1)
    sy = (mx[1] - mn[1]) / F32(H - 1)
    sz = (mx[2] - mn[2]) / F32(D - 1)
    vx = (mn[0] + np.arange(W, dtype=F32) * sx)[None, None, :]
    vy = (mn[1] + np.arange(H, dtype=F32) * sy)[None, :, None]
    vz = (mn[2] + np.arange(z0, z1, dtype=F32) * sz)[:, None, None]
    dep_all = np.asarray(depth, F32)
    F, Hd, Wd = dep_all.shape
    poses = np.asarray(poses, F32).reshape(F, 12)
    K = np.asarray(K, F32).reshape(F, 4)
    tr = F32(trunc)
    inv_tr = F32(1) / tr
    big, zlo, zhi = F32(2.0 ** 60), F32(2.0 ** -60), F32(2.0 ** 60)
    for f in range(F):
        P = poses[f]
        with np.errstate(invalid="ignore"):
            if not (np.abs(np.concatenate([P, K[f]])) < big).all():
                yield f, None, None
                continue
        Xc = P[1] * vy + ((P[0] * vx + P[2] * vz) + P[3])
        Yc = P[5] * vy + ((P[4] * vx + P[6] * vz) + P[7])
        Zc = P[9] * vy + ((P[8] * vx + P[10] * vz) + P[11])
        ok = (Zc >= zlo) & (Zc < zhi)
        cxh = K[f, 2] + F32(0.5)
        cyh = K[f, 3] + F32(0.5)
        with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
            iz = F32(1) / np.where(ok, Zc, F32(1))
            fu = np.floor((K[f, 0] * Xc) * iz + cxh)
            fv = np.floor((K[f, 1] * Yc) * iz + cyh)
        ok &= (fu >= 0) & (fu < Wd) & (fv >= 0) & (fv < Hd)
        ui = np.where(ok, fu, 0).astype(np.int64)
        vi = np.where(ok, fv, 0).astype(np.int64)
        dep = dep_all[f][vi, ui]
        with np.errstate(invalid="ignore", over="ignore"):
            ok &= dep > 0
            sdf = dep - Zc
            ok &= ~(sdf < -tr)
            ts = np.minimum(F32(1), sdf * inv_tr)
        yield f, ok, ts


def _slab_views(T, Wt, z0, z1, grid_depth):
    T = np.array(T, F32, copy=True)
    Wt = np.array(Wt, F32, copy=True)
    D = T.shape[0]
    slab_only = grid_depth is not None
    if slab_only:
        z1 = z0 + D if z1 is None else z1
        if z1 - z0 != D:
            raise ValueError("slab arrays must hold z1 - z0 slices")
        D = int(grid_depth)
    z1 = D if z1 is None else z1
    return T, Wt, D, z1, slab_only


def tsdf_integrate(T, Wt, depth, poses, K, bmin, bmax, trunc, z0=0, z1=None, grid_depth=None):
    """Build-defined TSDF integration, on copies; returns (T, Wt).
    The HIP path (tsdf.hip) computes exactly this, bit for bit.

    ``grid_depth``: when given, T/Wt hold only the z-slices [z0, z1) of a grid
    of that depth (the slab a CPU worker thread owns), else the whole grid.

    Per voxel and frame (every f32 operation one IEEE round-to-nearest step, in
    the order written):
      voxel (z,y,x) -> v = bmin + idx*(bmax-bmin)/(R-1)  (align_corners, x->W: sdf.py:284-304)
      Q = (P[r,0] vx + P[r,2] vz) + P[r,3];  c_r = P[r,1] vy + Q      (r = X, Y, Z rows)
      frames with any non-finite or |.| >= 2^60 pose/intrinsic are skipped
      skip unless 2^-60 <= Zc < 2^60;  iz = 1/Zc
      pixel = floor((fx Xc) iz + (cx + 0.5)), floor((fy Yc) iz + (cy + 0.5))
      skip off-image or depth <= 0; sdf = depth - Zc; skip sdf < -mu
      tsdf = min(1, sdf * (1/mu))
    The frames of one integration step (512 frames; longer inputs are consecutive
    steps) are fused order-free:
      q = rint(tsdf * 2^21) (exact integer);  S = sum q;  n = number of updates
      where n > 0:  T = f32((f64(T) f64(W) + f64(S) 2^-21) / (f64(W) + n));  W = W + f32(n)
    which telescopes the running average T = (T W + tsdf)/(W + 1), W += 1 of
    :func:`tsdf_integrate_seq` (2^-22 per update of the exact mean)."""
    T, Wt, D, z1, slab_only = _slab_views(T, Wt, z0, z1, grid_depth)
    Ts, Ws = (T, Wt) if slab_only else (T[z0:z1], Wt[z0:z1])
    F = np.asarray(depth).shape[0]
    for s0 in range(0, F, TSDF_STEP):
        s1 = min(F, s0 + TSDF_STEP)
        S = np.zeros(Ts.shape, np.int64)
        n = np.zeros(Ts.shape, np.int64)
        sl = (np.asarray(depth, F32)[s0:s1], np.asarray(poses, F32).reshape(-1, 12)[s0:s1],
              np.asarray(K, F32).reshape(-1, 4)[s0:s1])
        for _, ok, ts in _tsdf_frames(Ts, Ws, *sl, bmin, bmax, trunc, z0, z1, D, s0):
            if ok is None:
                continue
            with np.errstate(invalid="ignore"):
                q = np.rint(np.where(ok, ts, F32(0)) * F32(2.0 ** TSDF_QBITS))
            S += q.astype(np.int64)
            n += ok
        upd = n > 0
        with np.errstate(invalid="ignore", over="ignore", divide="ignore"):
            num = Ts.astype(np.float64) * Ws.astype(np.float64) + S.astype(np.float64) * 2.0 ** -TSDF_QBITS
            den = Ws.astype(np.float64) + n.astype(np.float64)
            Tn = (num / den).astype(F32)
            Wn = (Ws + n.astype(F32)).astype(F32)
        Ts = np.where(upd, Tn, Ts).astype(F32)
        Ws = np.where(upd, Wn, Ws).astype(F32)
    if slab_only:
        return Ts, Ws
    T[z0:z1] = Ts
    Wt[z0:z1] = Ws
    return T, Wt


def tsdf_integrate_seq(T, Wt, depth, poses, K, bmin, bmax, trunc, z0=0, z1=None, grid_depth=None):
    """The sequential running-average form of the same definition (rounds 1-4 of the
    build): per frame in order, T = (T W + tsdf)/(W + 1), W += 1, each f32 op one RN
    step.  tsdf_integrate equals it within the accumulated roundings (tests)."""
    T, Wt, D, z1, slab_only = _slab_views(T, Wt, z0, z1, grid_depth)
    Ts, Ws = (T, Wt) if slab_only else (T[z0:z1], Wt[z0:z1])
    for _, ok, ts in _tsdf_frames(Ts, Ws, depth, poses, K, bmin, bmax, trunc, z0, z1, D, 0):
        if ok is None:
            continue
        with np.errstate(invalid="ignore", over="ignore"):
            Tn = (Ts * Ws + ts) / (Ws + F32(1))
        Ts = np.where(ok, Tn, Ts).astype(F32)
        Ws = np.where(ok, Ws + F32(1), Ws).astype(F32)
    if slab_only:
        return Ts, Ws
    T[z0:z1] = Ts
    Wt[z0:z1] = Ws
    return T, Wt


# ---------------------------------------------------------------------------
def block_table(depth) -> np.ndarray:
    """(F,Hd,Wd) f32 -> (F, ceil(Hd/16), ceil(Wd/16), 2) f32 {min, max} of every
    16x16 block (blocks clipped at the image edge): min is -inf when the block
    holds a NaN, max ignores NaN (-inf when every pixel is NaN)."""
    d = np.asarray(depth, F32)
    F, Hd, Wd = d.shape
    nbv, nbu = -(-Hd // 16), -(-Wd // 16)
    out = np.empty((F, nbv, nbu, 2), F32)
    for bv in range(nbv):
        for bu in range(nbu):
            b = d[:, bv * 16:(bv + 1) * 16, bu * 16:(bu + 1) * 16].reshape(F, -1)
            nan = np.isnan(b)
            out[:, bv, bu, 0] = np.where(nan.any(1), -np.inf, np.where(nan, np.inf, b).min(1))
            out[:, bv, bu, 1] = np.where(nan, -np.inf, b).max(1)
    return out


def ray_aabb(rays_o, rays_d, bmin, bmax):
    """GradientBasedSampler.ray_aabb_intersection (sdf.py:154-165), f32, NaN-propagating."""
    o = np.asarray(rays_o, F32).reshape(-1, 3)
    d = np.asarray(rays_d, F32).reshape(-1, 3)
    mn = np.asarray(bmin, F32).ravel()
    mx = np.asarray(bmax, F32).ravel()
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = (F32(1.0) / d).astype(F32)
        t0 = ((mn - o) * inv).astype(F32)
        t1 = ((mx - o) * inv).astype(F32)
    tn = np.max(np.minimum(t0, t1), axis=-1)
    tf = np.min(np.maximum(t0, t1), axis=-1)
    tn = np.maximum(tn, F32(0))
    with np.errstate(invalid="ignore"):
        valid = tf > tn
    return tn.astype(F32), tf.astype(F32), valid


def torch_linspace01(S):
    """torch.linspace(0, 1, S) f32 (RangeFactoriesKernel.cpp): start + step*k for
    k < S/2, end - step*(S-k-1) after, each a fused multiply-add (the compiled
    kernel contracts it; emulated in f64, the product is exact)."""
    step = F32(1.0) / F32(S - 1)
    k = np.arange(S)
    lo = (np.float64(step) * k).astype(F32)
    hi = (1.0 - np.float64(step) * (S - k - 1)).astype(F32)
    return np.where(k < S // 2, lo, hi).astype(F32)


def sample_uniform(t_near, t_far, S, t_rand=None):
    """GradientBasedSampler.sample_uniform (sdf.py:167-180) with the jitter given."""
    t = torch_linspace01(S)
    tn = np.asarray(t_near, F32)[:, None]
    tf = np.asarray(t_far, F32)[:, None]
    z = (tn * (F32(1) - t) + tf * t).astype(F32)
    if t_rand is None:
        return z
    mids = (F32(0.5) * (z[:, 1:] + z[:, :-1])).astype(F32)
    upper = np.concatenate([mids, z[:, -1:]], 1)
    lower = np.concatenate([z[:, :1], mids], 1)
    return (lower + (upper - lower) * np.asarray(t_rand, F32)).astype(F32)
