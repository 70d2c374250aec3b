"""§8f row 4: the grid training step of the reference, on the GPU.

``GridTrainer.step(rays_o, rays_d, gt, z)`` is one iteration of
plenoxel.py:100-111 (``train``) / sdf.py:427-438 (``__main__``)::

    rgb = render_rays(model, rays_o, rays_d)     # NerfModel / SDFGrid forward
    loss = mse_loss(gt, rgb)
    optimizer.zero_grad(); loss.backward(); optimizer.step()   # Adam(lr=1e-2)

as two launches: ``sfmhip_render_train`` (fused sample + SH colour + composite
forward, mse gradient, analytic backward, trilinear scatter-add into the
gradient — ATen grid_sampler_3d's backward weights) and ``sfmhip_adam_step``
(torch's single-tensor Adam with the gradient reset fused in).  The
parameters, gradient and Adam moments live in the voxel-major layout
(D, H, W, 32) the renderer reads; ``grid`` exports the reference's
(1, 28, D, H, W) tensor.  The sample depths ``z`` are an explicit input (the
reference draws the jitter with ``torch.rand``).
"""
from __future__ import annotations

import numpy as np
import torch

from ._abi import call, dev, ptr, require_gpu, stream_ptr
from .voxel import MASK_PLENOXEL, MASK_SDF, _f3, _host_ptr, ray_aabb, sample_uniform


class GridTrainer:
    def __init__(self, grid, min_bound, max_bound, mask_mode: int = MASK_SDF, lr: float = 1e-2,
                 betas=(0.9, 0.999), eps: float = 1e-8):
        require_gpu()
        g = grid.detach() if isinstance(grid, torch.Tensor) else torch.as_tensor(grid)
        if g.dim() == 5:
            g = g[0]
        g = dev(g, torch.float32)
        self.C, self.D, self.H, self.W = (int(s) for s in g.shape)
        if self.C > 32:
            raise ValueError("GridTrainer supports C <= 32 channels")
        self.bmin, self.bmax = _f3(min_bound), _f3(max_bound)
        self.mask_mode = int(mask_mode)
        self.lr, self.betas, self.eps = float(lr), (float(betas[0]), float(betas[1])), float(eps)
        self.step_count = 0
        shape = (self.D, self.H, self.W, 32)
        self.param = torch.empty(shape, dtype=torch.float32, device=g.device)
        call("sfmhip_grid_to_voxel_major", ptr(g), self.C, self.D, self.H, self.W, ptr(self.param), stream_ptr())
        self.grad = torch.zeros(shape, dtype=torch.float32, device=g.device)
        self.exp_avg = torch.zeros(shape, dtype=torch.float32, device=g.device)
        self.exp_avg_sq = torch.zeros(shape, dtype=torch.float32, device=g.device)
        # 1 per voxel whose gradient line the scatter added to since the last zero_grad step:
        # elsewhere grad is 0, so Adam neither reads nor re-zeroes it
        self.touched = torch.zeros(shape[:3], dtype=torch.uint8, device=g.device)

    @classmethod
    def plenoxel(cls, voxel_grid, scale: float = 1.5, **kw) -> "GridTrainer":
        """NerfModel(N, scale) (plenoxel.py:19-43): mask |x| < scale, idx = x / scale."""
        return cls(voxel_grid, (-scale,) * 3, (scale,) * 3, MASK_PLENOXEL, **kw)

    def _export(self, vm: torch.Tensor) -> torch.Tensor:
        out = torch.empty((self.C, self.D, self.H, self.W), dtype=torch.float32, device=vm.device)
        call("sfmhip_grid_from_voxel_major", ptr(vm), self.C, self.D, self.H, self.W, ptr(out), stream_ptr())
        return out[None]

    @property
    def grid(self) -> torch.Tensor:
        """The parameter in the reference layout (1, C, D, H, W)."""
        return self._export(self.param)

    def state(self) -> dict:
        return dict(exp_avg=self._export(self.exp_avg), exp_avg_sq=self._export(self.exp_avg_sq),
                    step=self.step_count)

    def backward(self, rays_o, rays_d, gt, z):
        """Forward + loss + backward only (accumulates into self.grad).
        Returns (loss float, rgb (B,3) tensor)."""
        loss, rgb, B = self._backward(rays_o, rays_d, gt, z)
        return (float(loss.item()) / (3 * B) if B else float("nan")), rgb

    def _backward(self, rays_o, rays_d, gt, z):
        """backward() without the host synchronisation: (sum of squared errors as a
        device f64 scalar, rgb, B)."""
        o = dev(rays_o, torch.float32).reshape(-1, 3)
        d = dev(rays_d, torch.float32).reshape(-1, 3)
        zz = dev(z, torch.float32)
        t = dev(gt, torch.float32).reshape(-1, 3)
        B, S = zz.shape
        if o.shape[0] != B or d.shape[0] != B or t.shape[0] != B:
            raise ValueError("rays_o, rays_d, gt and z must have the same number of rays")
        rgb = torch.empty((B, 3), dtype=torch.float32, device=o.device)
        sq = torch.empty(B, dtype=torch.float32, device=o.device)
        call("sfmhip_render_train", ptr(self.param), self.D, self.H, self.W, _host_ptr(self.bmin),
             _host_ptr(self.bmax), self.mask_mode, ptr(o), ptr(d), ptr(zz), ptr(t), B, S, ptr(rgb), ptr(sq),
             ptr(self.grad), ptr(self.touched), stream_ptr())
        return sq.double().sum(), rgb, B

    def optimizer_step(self, zero_grad: bool = True) -> None:
        self.step_count += 1
        # only the voxels the scatter touched can have a non-zero gradient (flag per 32-float line)
        call("sfmhip_adam_step_flagged", ptr(self.param), ptr(self.grad), ptr(self.exp_avg), ptr(self.exp_avg_sq),
             self.param.numel(), self.lr, self.betas[0], self.betas[1], self.eps, self.step_count,
             1 if zero_grad else 0, ptr(self.touched), 5, stream_ptr())

    def step(self, rays_o, rays_d, gt, z, events=None) -> float:
        """One training iteration; returns loss.item() (plenoxel.py:105-111 reads it
        every step).  The host waits once, after the Adam step is enqueued.
        ``events``: optional (start, end) torch.cuda.Event pair recorded around the
        Adam launch on the current stream (timing only)."""
        loss, _, B = self._backward(rays_o, rays_d, gt, z)
        if events is not None:
            events[0].record()
        self.optimizer_step()
        if events is not None:
            events[1].record()
        return float(loss.item()) / (3 * B) if B else float("nan")

    def sdf_step(self, rays_o, rays_d, gt, num_samples: int = 160, t_rand=None, events=None):
        """One iteration of sdf.py's training loop (sdf.py:427-438) on an SDF-mode
        trainer: the sampler's ray-box test (sdf.py:154-165; rays that miss
        are dropped, sdf.py:229-232), ``num_samples`` stratified depths with the
        jitter ``t_rand`` (Bv, S) (torch.rand_like at sdf.py:176; drawn here
        when omitted), forward, ``mse_loss(gt[valid], rgb)``, backward and
        Adam.  Returns (loss.item(), valid (B,) bool device tensor)."""
        if self.mask_mode != MASK_SDF:
            raise ValueError("sdf_step needs an SDF-mode trainer (mask_mode=MASK_SDF)")
        o = dev(rays_o, torch.float32).reshape(-1, 3)
        d = dev(rays_d, torch.float32).reshape(-1, 3)
        t = dev(gt, torch.float32).reshape(-1, 3)
        tn, tf, valid = ray_aabb(o, d, self.bmin, self.bmax)
        idx = torch.nonzero(valid).squeeze(1)
        if idx.numel() == 0:
            raise ValueError("No valid rays intersect the grid.")
        z = sample_uniform(tn[idx].contiguous(), tf[idx].contiguous(), num_samples, t_rand)
        loss = self.step(o[idx].contiguous(), d[idx].contiguous(), t[idx].contiguous(), z, events)
        return loss, valid
