"""V1-V5: voxel-grid kernels with the reference's torch signatures.

* :func:`voxel_traversal` — ``voxel_travesal.py:1-73`` (quirks included:
  one-cell-late negative-direction boundary, overshoot, NaN padding, a ray that
  starts inactive is emitted twice).
* :class:`VoxelGrid` — ``SDFGrid.get_sdf`` / ``get_sdf_sh`` (``sdf.py:284-342``),
  ``NerfModel.forward`` (``plenoxel.py:31-43``) and the composite of
  ``SDFGrid.forward`` / ``render_rays`` (``sdf.py:391-406``,
  ``plenoxel.py:71-93``) for a given sample set ``z`` (the reference draws it
  with ``torch.rand``; callers pass it explicitly).
* :func:`ray_aabb`, :func:`sample_uniform` and :meth:`VoxelGrid.sdf_forward` —
  ``GradientBasedSampler`` (sdf.py:154-180, 220-256; its importance samples
  are discarded by the reference at 251-252) + ``SDFGrid.forward``.
* :func:`tsdf_integrate` — TSDF fusion of depth maps into a (D,H,W) grid laid
  out like the ``sdf.py`` grid (build-defined).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ._abi import call, dev, ptr, require_gpu, stream_ptr

MASK_SDF = 0       # sdf.py test_points: bmin <= p <= bmax (inclusive)
MASK_PLENOXEL = 1  # plenoxel: |p| < scale (strict), p/scale clipped to [-1, 1]


def _f3(v) -> np.ndarray:
    a = np.asarray(v if not isinstance(v, torch.Tensor) else v.detach().cpu().numpy(), dtype=np.float32)
    return np.ascontiguousarray(np.broadcast_to(a.ravel(), (3,)) if a.size == 1 else a.ravel()[:3])


def _host_ptr(a: np.ndarray) -> int:
    """Address of a host array; the caller must keep `a` referenced until the call returns."""
    return a.ctypes.data


def voxel_traversal(rays: torch.Tensor, _bin_size, max_steps: int = 1 << 20) -> torch.Tensor:
    """(N,8) rays [o, d, near, far] -> (N, S, 3) visited voxel indices (float, NaN padded)."""
    require_gpu()
    r = dev(rays, torch.float32)
    N = r.shape[0]
    b = float(_bin_size)
    steps = torch.empty(N, dtype=torch.int32, device=r.device)
    # one walk into rows of width `cap` when they fit a bounded buffer (DDA_CAP; 0 = always two passes):
    # the prefix of the rows is the two-pass result whenever every ray ends within cap - 1 steps
    cap = min(int(os.environ.get("SFMHIP_DDA_CAP", "1024")), int(max_steps) + 1)
    if N > 0 and cap >= 2 and N * cap * 12 <= (256 << 20):
        buf = torch.empty((N, cap, 3), dtype=torch.float32, device=r.device)
        call("sfmhip_voxel_traversal_capped", ptr(r), N, b, cap, ptr(buf), ptr(steps), stream_ptr())
        longest = int(steps.max().item())
        if longest < cap:
            out = torch.empty((N, 1 + longest, 3), dtype=torch.float32, device=r.device)
            call("sfmhip_voxel_traversal_rows", ptr(buf), cap, ptr(steps), N, 1 + longest, ptr(out), stream_ptr())
            return out
    call("sfmhip_voxel_traversal_count", ptr(r), N, b, int(max_steps), ptr(steps), stream_ptr())
    longest = int(steps.max().item()) if N > 0 else 0
    if longest > max_steps:
        raise RuntimeError(f"voxel_traversal: a ray is still active after max_steps={max_steps} "
                           "(the reference loop would not terminate)")
    S = 1 + longest
    out = torch.empty((N, S, 3), dtype=torch.float32, device=r.device)
    call("sfmhip_voxel_traversal", ptr(r), N, b, S, ptr(out), stream_ptr())
    return out


def ray_aabb(rays_o: torch.Tensor, rays_d: torch.Tensor, min_bound, max_bound):
    """sdf.py:154-165 -> (t_near (B,), t_far (B,), valid (B,) bool) device tensors."""
    require_gpu()
    o = dev(rays_o, torch.float32).reshape(-1, 3)
    d = dev(rays_d, torch.float32).reshape(-1, 3)
    B = o.shape[0]
    tn = torch.empty(B, dtype=torch.float32, device=o.device)
    tf = torch.empty_like(tn)
    valid = torch.empty(B, dtype=torch.uint8, device=o.device)
    bmn, bmx = _f3(min_bound), _f3(max_bound)   # kept alive across the call
    call("sfmhip_ray_aabb", ptr(o), ptr(d), B, _host_ptr(bmn), _host_ptr(bmx), ptr(tn), ptr(tf), ptr(valid),
         stream_ptr())
    return tn, tf, valid.bool()


def sample_uniform(t_near: torch.Tensor, t_far: torch.Tensor, num_samples: int, t_rand=None,
                   perturb: bool = True) -> torch.Tensor:
    """sdf.py:167-180: stratified samples (B, S); ``t_rand`` (B, S) is the jitter
    the reference draws with torch.rand_like (drawn here when omitted)."""
    tn = dev(t_near, torch.float32)
    tf = dev(t_far, torch.float32)
    B = tn.shape[0]
    if perturb and t_rand is None:
        t_rand = torch.rand((B, num_samples), device=tn.device)
    tr = dev(t_rand, torch.float32) if perturb else None
    z = torch.empty((B, num_samples), dtype=torch.float32, device=tn.device)
    call("sfmhip_stratified_samples", ptr(tn), ptr(tf), ptr(tr), B, int(num_samples), 1 if perturb else 0,
         ptr(z), stream_ptr())
    return z


class VoxelGrid:
    """An SDF + SH-2 colour grid (1, 28, D, H, W) in the reference layout.

    ``mask_mode`` MASK_SDF reproduces sdf.py (bounds min_bound/max_bound),
    MASK_PLENOXEL reproduces plenoxel.py (bounds +-scale)."""

    def __init__(self, grid: torch.Tensor, min_bound, max_bound, mask_mode: int = MASK_SDF):
        require_gpu()
        g = grid.detach()
        if g.dim() == 5:
            g = g[0]
        self.grid = dev(g, torch.float32)
        self.C, self.D, self.H, self.W = (int(s) for s in self.grid.shape)
        self.bmin = _f3(min_bound)
        self.bmax = _f3(max_bound)
        self.mask_mode = int(mask_mode)
        self._vm = None
        self._finite = None
        self._ver = None

    def invalidate(self) -> None:
        """Drop the cached voxel-major copy and finiteness flag (they are also dropped
        automatically when ``self.grid`` is modified in place: its version counter)."""
        self._vm = None
        self._finite = None
        self._ver = None

    def _sync_cache(self) -> None:
        # self.grid may alias the caller's tensor (dev() does not copy): an in-place update
        # bumps its version, and the derived copies must follow it
        if self._ver is not None and self._ver != self.grid._version:
            self.invalidate()
        self._ver = self.grid._version

    @classmethod
    def plenoxel(cls, voxel_grid: torch.Tensor, scale: float = 1.5) -> "VoxelGrid":
        return cls(voxel_grid, (-scale,) * 3, (scale,) * 3, MASK_PLENOXEL)

    def sample(self, points: torch.Tensor) -> torch.Tensor:
        """All C channels at the points: (P, C) f32 (zero outside)."""
        p = dev(points, torch.float32).reshape(-1, 3)
        out = torch.empty((p.shape[0], self.C), dtype=torch.float32, device=p.device)
        call("sfmhip_grid_sample", ptr(self.grid), self.C, self.D, self.H, self.W, _host_ptr(self.bmin),
             _host_ptr(self.bmax), self.mask_mode, ptr(p), p.shape[0], ptr(out), stream_ptr())
        return out

    def nerf_forward(self, x: torch.Tensor, d: torch.Tensor):
        """NerfModel.forward (plenoxel.py:31-43): (color (P,3), sigma (P,)) at
        points x (P,3) seen along unit directions d (P,3); zero outside."""
        if self.C != 28:
            raise ValueError("nerf_forward needs the 28-channel SDF+SH grid")
        p = dev(x, torch.float32).reshape(-1, 3)
        dd = dev(d, torch.float32).reshape(-1, 3)
        if dd.shape != p.shape:
            raise ValueError("x and d must both be (P, 3)")
        color = torch.empty((p.shape[0], 3), dtype=torch.float32, device=p.device)
        sigma = torch.empty(p.shape[0], dtype=torch.float32, device=p.device)
        call("sfmhip_nerf_forward", ptr(self.grid), self.D, self.H, self.W, _host_ptr(self.bmin), _host_ptr(self.bmax),
             self.mask_mode, ptr(p), ptr(dd), p.shape[0], ptr(color), ptr(sigma), stream_ptr())
        return color, sigma

    def get_sdf(self, points: torch.Tensor) -> torch.Tensor:
        return self.sample(points)[:, 0]

    def get_sdf_sh(self, points: torch.Tensor):
        s = self.sample(points)
        return s[:, 0], s[:, 1:]

    def voxel_major(self) -> torch.Tensor:
        self._sync_cache()
        if self._vm is None:
            if self.C > 32:
                raise ValueError("voxel-major layout supports C <= 32")
            vm = torch.empty((self.D, self.H, self.W, 32), dtype=torch.float32, device=self.grid.device)
            call("sfmhip_grid_to_voxel_major", ptr(self.grid), self.C, self.D, self.H, self.W, ptr(vm),
                 stream_ptr())
            self._vm = vm
        return self._vm

    def sdf_forward(self, rays_o, rays_d, num_samples: int = 160, t_rand=None, perturb: bool = True):
        """SDFGrid.forward (sdf.py:391-406) with its sampler (sdf.py:220-256):
        -> (rgb (Bv,3), pts (Bv,S,3), valid (B,) bool)."""
        o = dev(rays_o, torch.float32).reshape(-1, 3)
        d = dev(rays_d, torch.float32).reshape(-1, 3)
        tn, tf, valid = ray_aabb(o, d, self.bmin, self.bmax)
        if not bool(valid.any()):
            raise ValueError("No valid rays intersect the grid.")
        idx = torch.nonzero(valid).squeeze(1)
        ov, dv = o[idx].contiguous(), d[idx].contiguous()
        z = sample_uniform(tn[idx].contiguous(), tf[idx].contiguous(), num_samples, t_rand, perturb)
        pts = ov[:, None, :] + dv[:, None, :] * z[:, :, None]
        return self.render(ov, dv, z), pts, valid

    def render(self, rays_o: torch.Tensor, rays_d: torch.Tensor, z: torch.Tensor) -> torch.Tensor:
        """Fused sample + SH colour + composite for sorted sample depths z (B,S): (B,3)."""
        if self.C != 28:
            raise ValueError("render needs the 28-channel SDF+SH grid")
        o = dev(rays_o, torch.float32).reshape(-1, 3)
        d = dev(rays_d, torch.float32).reshape(-1, 3)
        zz = dev(z, torch.float32)
        B, S = zz.shape
        rgb = torch.empty((B, 3), dtype=torch.float32, device=o.device)
        vm = self.voxel_major()
        if self.finite():   # sdf from the compact channel-0 plane, voxel lines only where alpha != 0
            call("sfmhip_render_rays_sdf", ptr(vm), ptr(self.grid[0]), self.D, self.H, self.W, _host_ptr(self.bmin),
                 _host_ptr(self.bmax), self.mask_mode, ptr(o), ptr(d), ptr(zz), B, S, ptr(rgb), stream_ptr())
        else:
            call("sfmhip_render_rays", ptr(vm), self.D, self.H, self.W, _host_ptr(self.bmin),
                 _host_ptr(self.bmax), self.mask_mode, ptr(o), ptr(d), ptr(zz), B, S, ptr(rgb), stream_ptr())
        return rgb

    def finite(self) -> bool:
        """Whether every grid value is finite (cached with the voxel-major copy): the render
        may then skip the colour lines of samples with alpha = 0, bit-identically."""
        self._sync_cache()
        if getattr(self, "_finite", None) is None:
            self._finite = bool(torch.isfinite(self.grid).all().item())
        return self._finite


def tsdf_integrate(T: torch.Tensor, Wt: torch.Tensor, depth: torch.Tensor, poses: torch.Tensor,
                   K: torch.Tensor, bmin, bmax, trunc: float, z0: int = 0, z1: int | None = None,
                   block_table: torch.Tensor | None = None) -> None:
    """In-place TSDF update of z-slices [z0, z1) of T/Wt (D,H,W) from F depth maps.

    depth (F,Hd,Wd) f32 (<=0 invalid), poses (F,3,4) world->camera f32,
    K (F,4) [fx, fy, cx, cy] f32, bounds in world units, trunc = mu.
    block_table: optional (F, ceil(Hd/16), ceil(Wd/16), 2) f32 device table from
    tsdf_block_table (e.g. assembled across ranks by dist.shared_block_table);
    the result is bit-identical, the call's own pass over the depth maps skipped.

    Batching: the frames of ONE call are fused order-free in integration steps of
    at most 512 frames (integer fixed-point sums S = sum rint(tsdf 2^21), n = #updates,
    then one finish per voxel and step: T' = (T W + S 2^-21) / (W + n); include/sfmhip.h
    V5 block).  The result therefore depends on how frames are grouped into calls:
    one call with F <= 512 frames gives different low bits than F calls of one frame
    (each a step of its own), and both differ from a sequential running average
    T <- (T W + tsdf)/(W + 1) by at most ~2^-22 per update.  Any z-slab / rank split
    of one call is bit-identical to the whole call.  A caller that streams frames and
    needs batching-independent bits integrates them one frame per call (each frame
    its own step, which IS the sequential running average up to the 2^-21 quantum).
    There is no TSDF in the reference (build-defined)."""
    gpu = require_gpu()
    if T.dtype != torch.float32 or Wt.dtype != torch.float32 or not T.is_contiguous() or not Wt.is_contiguous():
        raise ValueError("T and Wt must be contiguous float32 device tensors")
    if T.dim() != 3 or tuple(Wt.shape) != tuple(T.shape):
        raise ValueError(f"T and Wt must be (D,H,W) tensors of one shape, got {tuple(T.shape)} and "
                         f"{tuple(Wt.shape)}")
    if T.device != gpu or Wt.device != gpu:
        raise ValueError(f"T and Wt must live on the current HIP device {gpu}, got {T.device} / {Wt.device}")
    D, H, W = T.shape
    z1 = D if z1 is None else int(z1)
    if not 0 <= int(z0) <= z1 <= D:
        raise ValueError(f"z-slab [{z0}, {z1}) outside [0, {D}]")
    dp = dev(depth, torch.float32)
    ps = dev(poses, torch.float32)
    kk = dev(K, torch.float32)
    if dp.dim() != 3:
        raise ValueError(f"depth must be (F,Hd,Wd), got {tuple(dp.shape)}")
    F, Hd, Wd = dp.shape
    if tuple(ps.shape) != (F, 3, 4):
        raise ValueError(f"poses must be ({F},3,4) to match depth, got {tuple(ps.shape)}")
    if tuple(kk.shape) != (F, 4):
        raise ValueError(f"K must be ({F},4) to match depth, got {tuple(kk.shape)}")
    bmn, bmx = _f3(bmin), _f3(bmax)
    if block_table is None:
        call("sfmhip_tsdf_integrate", ptr(T), ptr(Wt), D, H, W, int(z0), z1, ptr(dp), F, Hd, Wd, ptr(ps), ptr(kk),
             _host_ptr(bmn), _host_ptr(bmx), float(trunc), stream_ptr())
        return
    if tuple(block_table.shape) != block_table_shape(F, Hd, Wd) or block_table.dtype != torch.float32 or \
            not block_table.is_contiguous() or block_table.device != T.device:
        raise ValueError(f"block_table must be a contiguous float32 {block_table_shape(F, Hd, Wd)} tensor on {T.device}")
    call("sfmhip_tsdf_integrate_tab", ptr(T), ptr(Wt), D, H, W, int(z0), z1, ptr(dp), F, Hd, Wd, ptr(ps), ptr(kk),
         _host_ptr(bmn), _host_ptr(bmx), float(trunc), ptr(block_table), stream_ptr())


def block_table_shape(F: int, Hd: int, Wd: int) -> tuple:
    return (int(F), -(-int(Hd) // 16), -(-int(Wd) // 16), 2)


def tsdf_block_table(depth: torch.Tensor, f0: int = 0, f1: int | None = None,
                     out: torch.Tensor | None = None) -> torch.Tensor:
    """{min, max} of every 16x16 block of depth maps [f0, f1) (rows f0..f1 of `out`,
    an (F, ceil(Hd/16), ceil(Wd/16), 2) f32 device table, allocated when None)."""
    require_gpu()
    dp = dev(depth, torch.float32)
    F, Hd, Wd = dp.shape
    f1 = F if f1 is None else int(f1)
    if out is None:
        out = torch.empty(block_table_shape(F, Hd, Wd), dtype=torch.float32, device=dp.device)
    elif tuple(out.shape) != block_table_shape(F, Hd, Wd) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous float32 {block_table_shape(F, Hd, Wd)} tensor")
    call("sfmhip_tsdf_block_table", ptr(dp), F, Hd, Wd, int(f0), f1, ptr(out), stream_ptr())
    return out


def tsdf_layer_stats(shape, depth: torch.Tensor, poses: torch.Tensor, K: torch.Tensor, bmin, bmax,
                     trunc: float) -> np.ndarray:
    """Per 8-voxel z layer of the grid `shape` = (D,H,W): (tested, culled, free)
    counts of (wave sub-tile, frame) pairs -- what :func:`tsdf_integrate`'s
    pre-passes decide.  Feeds dist.plan_slabs (cost-balanced z-slabs)."""
    require_gpu()
    D, H, W = (int(v) for v in shape)
    dp = dev(depth, torch.float32)
    ps = dev(poses, torch.float32)
    kk = dev(K, torch.float32)
    F, Hd, Wd = dp.shape
    out = np.zeros((-(-D // 8), 3), np.int64)
    bmn, bmx = _f3(bmin), _f3(bmax)
    call("sfmhip_tsdf_layer_stats", D, H, W, ptr(dp), F, Hd, Wd, ptr(ps), ptr(kk), _host_ptr(bmn), _host_ptr(bmx),
         float(trunc), out.ctypes.data, stream_ptr())
    return out


def tsdf_layer_cost(stats: np.ndarray, w_proj: float = 1.0, w_free: float = 0.12, w_tested: float = 0.02) -> np.ndarray:
    """Cost model of a tile layer from :func:`tsdf_layer_stats`: projected
    (sub-tile, frame) pairs dominate the fusion, free-space runs cost a
    fraction, every tested pair a little (mask walk, cull test)."""
    st = np.asarray(stats, np.float64)
    proj = st[:, 0] - st[:, 1] - st[:, 2]
    return w_proj * proj + w_free * st[:, 2] + w_tested * st[:, 0]


def tsdf_cull_stats(shape, depth: torch.Tensor, poses: torch.Tensor, K: torch.Tensor, bmin, bmax, trunc: float,
                    z0: int = 0, z1: int | None = None) -> dict:
    """Diagnostics of tsdf_integrate's pre-passes on grid `shape` = (D,H,W):
    how many (8x2x8 wave sub-tile, frame) pairs are culled and how many are
    fused as free space (tsdf = 1, no depth gather)."""
    require_gpu()
    D, H, W = (int(v) for v in shape)
    z1 = D if z1 is None else int(z1)
    dp = dev(depth, torch.float32)
    ps = dev(poses, torch.float32)
    kk = dev(K, torch.float32)
    F, Hd, Wd = dp.shape
    st = np.zeros(3, np.int64)
    bmn, bmx = _f3(bmin), _f3(bmax)   # kept alive across the call
    call("sfmhip_tsdf_cull_stats", D, H, W, int(z0), z1, ptr(dp), F, Hd, Wd, ptr(ps), ptr(kk),
         _host_ptr(bmn), _host_ptr(bmx), float(trunc), st.ctypes.data, stream_ptr())
    n = max(int(st[0]), 1)
    return {"tested": int(st[0]), "culled": int(st[1]), "free": int(st[2]),
            "culled_frac": st[1] / n, "free_frac": st[2] / n, "full_frac": 1 - (st[1] + st[2]) / n}
