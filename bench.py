#!/usr/bin/env python
"""bench.py — headline benchmark of the SfM dense-compute path on MI355X.

Primary line (BASELINE.json metric, config C3/C4): image-pairs matched/sec —
all 32,896 pairs of 257 synthetic images x 4096 SuperPoint-like 256-d
descriptors (int8-quantised, resident in HBM), BF-L2 + ratio test 0.75 on the
MFMA kernel.  With N ranks (one process per GPU, torch.distributed over RCCL)
the pairs are split into N contiguous ranges (strong scaling over the fixed
dataset) and ONE all-gather of the int16 match graph runs inside the step.

Secondary lines (same JSON object):
  * TSDF Mvoxel/sec — 256^3 grid fused from 257 synthetic 1936x1296 depth maps
    (C5), z-slab sharded over ranks (N > 1: the depth block table is built per
    frame range and all-gathered; no grid data is exchanged).
  * BA obs/sec — DLT triangulation + residual + FD Jacobian over 256 pairs x
    4096 observations.
  * N = 1 only: DDA traversal, plenoxel render, vq, geometric verification,
    PnP and the plenoxel training step, each with a CPU
    baseline sample.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
        python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_IMG, M_KPT, DIM = 257, 4096, 256
TSDF_R, TSDF_F = 256, 257
BA_PAIRS, BA_OBS = 256, 4096
PEAK_INT8_TOPS = 5000.0       # MI355X dense int8 MFMA (MI355X_MICROARCH.md: 2x bf16 2.5 PF)
PEAK_HBM_GBS = 8000.0         # HBM3E spec
MATCH_CHUNKS = 4              # N>1 (RCCL): match launches per step, each overlapped with the previous all-gather
PEAK_FP32_TFLOPS = 157.3      # vector fp32
PEAK_FP64_TFLOPS = 78.6       # fp64 (vector and v_mfma_f64 matrix peaks are the same on MI355X)
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r1", "traffic.json")


def pmc_traffic(kind: str, frac: float = 1.0):
    """HBM bytes per step of the dominant kernel from the committed PMC passes
    (counters need their own rocprofv3 runs), scaled to this rank's share."""
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)
        return t[kind]["bytes_per_step"] * frac
    except (OSError, KeyError, ValueError):
        return None


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def timed(fn, steps, warmup, barrier):
    """W untimed steps, then K steps bracketed by barrier + synchronize; returns
    (wall seconds over K steps, per-step kernel ms from HIP events)."""
    for _ in range(warmup):
        fn(None)
    torch.cuda.synchronize()
    barrier()
    ev = []
    t0 = time.perf_counter()
    for _ in range(steps):
        ev.append(fn(True))
    torch.cuda.synchronize()
    barrier()
    wall = time.perf_counter() - t0
    kms = [a.elapsed_time(b) for a, b in ev if a is not None]
    return wall, kms


def max_over_ranks(x: float, world: int, device) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64,
                     device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def blas_threads() -> int:
    try:
        from threadpoolctl import threadpool_info
        n = [i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"]
        return int(max(n)) if n else 1
    except Exception:
        return int(os.environ.get("OMP_NUM_THREADS", "1"))


def baseline_sample(pairs, n=48):
    """Deterministic spread of pair indices used for the CPU baseline."""
    return [(i * 997) % len(pairs) for i in range(n)]


def cpu_baseline_match(qcpu, pairs, sample, budget_s=12.0):
    """Oracle (numpy GEMM-form, exact ints) on a bounded sample of the same pairs."""
    from oracle import match as om
    n_done, t_used = 0, 0.0
    for i in sample:
        if t_used >= budget_s:
            break
        a, b = (int(v) for v in pairs[i])
        t0 = time.perf_counter()
        om.bf_match_q(qcpu[a], qcpu[b], (3, 4))
        t_used += time.perf_counter() - t0
        n_done += 1
    return n_done / t_used, n_done, t_used


def voxel_and_vq_lines(sfm, syn, device, args, barrier, cpu=True):
    """V1 DDA traversal, V2+V4 fused sample/SH/composite at the plenoxel config
    (28 x 256^3 grid, 2048 rays x 192 bins per batch) and M2 vq (C3 descriptors
    as f64 vs a 200-word codebook), each with an oracle CPU baseline sample."""
    out = []
    g = torch.Generator(device=device)
    g.manual_seed(7)
    # V1: the survey's probe geometry (4096 rays, bin 1, far <= 64).  The output is
    # the reference's (N, S_max, 3) NaN-padded tensor, so its size grows with the
    # longest ray; at 1M rays it is ~89 GB of mostly padding (tools/dda_probe.py).
    nr = 4096
    o = torch.rand((nr, 3), generator=g, device=device) * 64 - 32
    dvec = torch.randn((nr, 3), generator=g, device=device)
    far = torch.rand((nr, 1), generator=g, device=device) * 64
    rays = torch.cat([o, dvec / dvec.norm(dim=1, keepdim=True), torch.zeros_like(far), far], 1).contiguous()

    def dda_step(record):
        e0 = e1 = None
        if record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        vt = sfm.voxel_traversal(rays, 1.0)
        if record:
            e1.record()
        return (e0, e1)

    wall, _ = timed(dda_step, args.steps, 1, barrier)
    ms = wall / args.steps * 1e3
    line = {"metric": "voxel_traversal rays/sec", "value": nr / (ms * 1e-3), "unit": "rays/s", "ms_per_step": ms,
            "config": {"workload": "V1 DDA (voxel_travesal.py semantics): 4096 rays, bin 1, far U(0,64) "
                                   "(count pass + host S_max + fill pass)"}}
    if cpu:
        from oracle import voxel as ov
        rr = rays.cpu().numpy()
        t0 = time.perf_counter()
        ov.voxel_traversal(rr, 1.0)
        dt = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": nr / dt, "unit": "rays/s", "cores": 1, "kind": "port",
                                "sample": f"the same {nr} rays through oracle.voxel.voxel_traversal (numpy), {dt:.2f}s"}
    out.append(line)
    # V2+V4: plenoxel N=256 grid, 16 batches of 2048 rays x 192 bins
    N, B, S, NB = 256, 2048, 192, 16
    grid = (torch.randn((28, N, N, N), generator=g, device=device) * 0.1)
    vg = sfm.VoxelGrid.plenoxel(grid, 1.5)
    vg.voxel_major()
    del grid
    ro = torch.randn((NB * B, 3), generator=g, device=device) * 0.2 + torch.tensor([0.0, 0.0, -3.0], device=device)
    rd = torch.randn((NB * B, 3), generator=g, device=device) * 0.2 + torch.tensor([0.0, 0.0, 1.0], device=device)
    rd = rd / rd.norm(dim=1, keepdim=True)
    t = torch.linspace(2.0, 6.0, S, device=device).expand(NB * B, S)
    mid = (t[:, :-1] + t[:, 1:]) / 2
    u = torch.rand((NB * B, S), generator=g, device=device)
    z = (torch.cat([t[:, :1], mid], 1) + (torch.cat([mid, t[:, -1:]], 1) - torch.cat([t[:, :1], mid], 1)) * u)
    z = z.contiguous()

    def render_step(record):
        e0 = e1 = None
        if record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        vg.render(ro, rd, z)
        if record:
            e1.record()
        return (e0, e1)

    wall, kms = timed(render_step, args.steps, 1, barrier)
    ms = wall / args.steps * 1e3
    line = {"metric": "render_rays rays/sec", "value": NB * B / (ms * 1e-3), "unit": "rays/s", "ms_per_step": ms,
            "config": {"workload": "V2+V4 plenoxel render_rays: 28x256^3 grid, 16 x (2048 rays x 192 bins)"},
            "roofline": {"bound": "hbm", "kernel": "render_kernel", "kernel_ms": float(np.mean(kms)),
                         "algorithmic_bytes_per_sample": 8 * 112}}
    if cpu:
        from oracle import voxel as ov
        gsmall = vg.grid.cpu().numpy()
        t0 = time.perf_counter()
        ov.render(gsmall, (-1.5,) * 3, (1.5,) * 3, 1, ro[:64].cpu().numpy(), rd[:64].cpu().numpy(),
                  z[:64].cpu().numpy())
        dt = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": 64 / dt, "unit": "rays/s", "cores": 1, "kind": "port",
                                "sample": f"64 rays x 192 bins through oracle.voxel.render (numpy f32), {dt:.2f}s"}
        del gsmall
    out.append(line)
    del vg
    torch.cuda.empty_cache()
    # M2: vq of all C3 descriptors (f64) against a 200-word codebook
    obs = syn.superpoint_like(N_IMG, M_KPT, 128, seed=3, device=device).reshape(-1, 128).double().contiguous()
    book = obs[torch.randperm(obs.shape[0], generator=g, device=device)[:200]].contiguous()
    codes = torch.empty(obs.shape[0], dtype=torch.int32, device=device)
    dist = torch.empty(obs.shape[0], dtype=torch.float64, device=device)
    from importlib import import_module
    abi = import_module("3d_reconstruction_amd._abi")

    def vq_step(record):
        e0 = e1 = None
        if record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        abi.call("sfmhip_vq", obs.data_ptr(), obs.shape[0], book.data_ptr(), 200, 128, codes.data_ptr(),
                 dist.data_ptr(), abi.stream_ptr())
        if record:
            e1.record()
        return (e0, e1)

    wall, kms = timed(vq_step, args.steps, 1, barrier)
    ms = wall / args.steps * 1e3
    line = {"metric": "vq obs/sec", "value": obs.shape[0] / (ms * 1e-3), "unit": "obs/s", "ms_per_step": ms,
            "config": {"workload": "M2 vq (matching.py:27): 257x4096 obs x 200 codes x 128-d, f64"},
            "roofline": {"bound": "mfma", "kernel": "vq_f32r_kernel+vq_exact_kernel", "kernel_ms": float(np.mean(kms)),
                         # GEMM form: 2 flops per (obs, codeword, dim) on v_mfma_f32_16x16x4_f32 (f32 filter
                         # with a proven error bound; undecided observations settled in f64)
                         "achieved_tflops": 2 * obs.shape[0] * 200 * 128 / (np.mean(kms) * 1e-3) / 1e12,
                         "peak_tflops": PEAK_FP32_TFLOPS,
                         "frac": 2 * obs.shape[0] * 200 * 128 / (np.mean(kms) * 1e-3) / 1e12 / PEAK_FP32_TFLOPS}}
    if cpu:
        from scipy.cluster.vq import vq as scipy_vq
        oo, bb = obs[:4096].cpu().numpy(), book.cpu().numpy()
        t0 = time.perf_counter()
        scipy_vq(oo, bb)
        dt = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": 4096 / dt, "unit": "obs/s", "cores": blas_threads(), "kind": "reference",
                                "sample": f"scipy.cluster.vq.vq (the reference's own call) on 4096 obs, {dt:.3f}s"}
    out.append(line)
    return out


def verify_line(sfm, syn, device, args, barrier, cpu=True):
    """§8f row 2: findEssentialMat (RANSAC, prob 0.999, 1 px) + recoverPose for
    256 BFS-candidate pairs x 2048 matches (30 % outliers, 0.5 px noise), one
    batched launch each; CPU baseline = the oracle restatement on 2 pairs."""
    v = sfm.verify
    s = syn.two_view_pairs(256, 2048, outlier_frac=0.3, noise_px=0.5, seed=6)
    a, b, of = v.pack_pairs(s["pts0"], s["pts1"])
    cam = torch.tensor(v._cam(s["K"]), dtype=torch.float64, device=device).expand(256, 4).contiguous()
    holder = {}

    def step(record):
        e0 = e1 = None
        if record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        r = v.find_essential_batched(a, b, of, cam)
        holder["rp"] = v.recover_pose_batched(r["E"], a, b, of, cam, mask=r["mask"])
        holder["r"] = r
        if record:
            e1.record()
        return (e0, e1)

    wall, kms = timed(step, args.steps, 1, barrier)
    ms = wall / args.steps * 1e3
    iters = holder["r"]["iters"].float().mean().item()
    line = {"metric": "geometric verification pairs/sec", "value": 256 / (ms * 1e-3), "unit": "pairs/s",
            "ms_per_step": ms,
            "config": {"workload": "findEssentialMat(RANSAC, 0.999, 1px) + recoverPose: 256 pairs x 2048 matches, "
                                   "30% outliers, 0.5 px noise (matching.py:134-139 / sfm.py:108-119)",
                       "mean_ransac_iters": iters},
            "roofline": {"bound": "fp64", "kernel": "essential_ransac_kernel+recover_pose_kernel",
                         "kernel_ms": float(np.mean(kms))}}
    if cpu:
        from oracle import ransac as orc
        t0 = time.perf_counter()
        for p in range(2):
            E, m = orc.find_essential_mat(s["pts0"][p], s["pts1"][p], s["K"])
            keep = m.ravel() > 0
            orc.recover_pose(E, s["pts0"][p][keep], s["pts1"][p][keep], s["K"])
        dt = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": 2 / dt, "unit": "pairs/s", "cores": 1, "kind": "port",
                                "sample": f"2 of the 256 pairs through oracle.ransac (numpy restatement of "
                                          f"OpenCV's findEssentialMat + recoverPose), {dt:.2f}s"}
    return line


def train_line(sfm, syn, device, args, barrier, cpu=True):
    """§8f row 4: one plenoxel training step at the reference's config
    (plenoxel.py:124-133: NerfModel(N=256), batch 2048 rays, 192 bins,
    hn=2, hf=6): fused render forward+backward (scatter into the gradient)
    + Adam over all 28 x 256^3 parameters with the gradient reset."""
    tm = importlib.import_module("3d_reconstruction_amd.train")
    N, B, S = 256, 2048, 192
    g = torch.Generator(device=device)
    g.manual_seed(11)
    grid = torch.ones((28, N, N, N), device=device) / 100        # NerfModel init (plenoxel.py:29)
    tr = tm.GridTrainer.plenoxel(grid, 1.5, lr=1e-2)
    del grid
    torch.cuda.empty_cache()
    ro = torch.randn((B, 3), generator=g, device=device) * 0.2 + torch.tensor([0.0, 0.0, -3.0], device=device)
    rd = torch.randn((B, 3), generator=g, device=device) * 0.2 + torch.tensor([0.0, 0.0, 1.0], device=device)
    rd = (rd / rd.norm(dim=1, keepdim=True)).contiguous()
    t = torch.linspace(2.0, 6.0, S, device=device).expand(B, S)
    mid = (t[:, :-1] + t[:, 1:]) / 2
    lower = torch.cat([t[:, :1], mid], 1)
    upper = torch.cat([mid, t[:, -1:]], 1)
    z = (lower + (upper - lower) * torch.rand((B, S), generator=g, device=device)).contiguous()
    gt = torch.rand((B, 3), generator=g, device=device)
    ev = {}

    def step(record):
        e0 = e1 = e2 = None
        if record:
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record()
        loss, _, nb = tr._backward(ro, rd, gt, z)
        if record:
            e1.record()
        tr.optimizer_step()
        if record:
            e2.record()
            ev.setdefault("a", []).append((e1, e2))
        float(loss.item()) / (3 * nb)              # loss.item() every step, as plenoxel.py:110
        return (e0, e2)

    wall, kms = timed(step, args.steps, 1, barrier)
    ms = wall / args.steps * 1e3
    adam_ms = float(np.mean([a.elapsed_time(b) for a, b in ev["a"]]))
    n_par = 28 * N ** 3
    tr.backward(ro, rd, gt, z)                    # the share of voxel lines one step's scatter touches
    touched = float(tr.touched.float().mean().item())
    tr.optimizer_step()
    moved = 24 + 8 * touched                      # p, m, v read + written; grad only on touched lines
    line = {"metric": "plenoxel training steps/sec", "value": 1e3 / ms, "unit": "steps/s", "ms_per_step": ms,
            "config": {"workload": "plenoxel.py train step: NerfModel(N=256) 28x256^3, 2048 rays x 192 bins, "
                                   "mse + backward + Adam(lr=1e-2)"},
            "roofline": {"bound": "hbm", "kernel": "adam_flagged_kernel", "kernel_ms": adam_ms,
                         "algorithmic_bytes_per_param": 32,
                         "achieved_gbs": n_par * 32 / (adam_ms * 1e-3) / 1e9, "peak_gbs": PEAK_HBM_GBS,
                         "frac": n_par * 32 / (adam_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                         "touched_line_frac": touched,
                         "moved_gbs": n_par * 32 / 28 * moved / (adam_ms * 1e-3) / 1e9,
                         "note": "torch Adam's 32 B/param (p, g, m, v read; p, m, v, g written) is the algorithmic "
                                 "count; the kernel skips grad lines the step's scatter did not touch (known 0), and "
                                 "moves (24 + 8 x touched) B per slot of the voxel-major 32-channel layout "
                                 "(4 pad channels): moved_gbs"}}
    if cpu:
        from oracle import train as ot
        Nc, Bc = 64, 64
        gsmall = np.full((28, Nc, Nc, Nc), 0.01, np.float32)
        zz = z[:Bc].cpu().numpy()
        t0 = time.perf_counter()
        _, _, grad = ot.render_loss_grad(gsmall, (-1.5,) * 3, (1.5,) * 3, 1, ro[:Bc].cpu().numpy(),
                                         rd[:Bc].cpu().numpy(), zz, gt[:Bc].cpu().numpy())
        t_r = (time.perf_counter() - t0) / Bc
        t0 = time.perf_counter()
        ot.adam_step(gsmall, grad, np.zeros_like(grad), np.zeros_like(grad), 1)
        t_a = (time.perf_counter() - t0) / gsmall.size
        est = t_r * B + t_a * n_par
        line["cpu_baseline"] = {"value": 1.0 / est, "unit": "steps/s", "cores": 1, "kind": "port",
                                "sample": f"oracle.train on {Bc} rays (render+backward, {t_r * 1e3:.2f} ms/ray) "
                                          f"and Adam over 28x{Nc}^3 params ({t_a * 1e9:.1f} ns/param), "
                                          f"extrapolated to 2048 rays + 28x256^3 params = {est:.1f} s/step"}
    del tr
    torch.cuda.empty_cache()
    return line


def pnp_line(sfm, syn, device, args, barrier, cpu=True):
    """sfm.py:116 solvePnPRansac batched: 256 registrations x 2000 2D-3D
    correspondences (30 % outliers, 0.5 px noise), EPnP RANSAC + LM refine."""
    from oracle import geometry as og
    v = sfm.verify
    rng = np.random.default_rng(12)
    K = np.diag([syn.FOCAL, syn.FOCAL, 1.0])
    P, n = 256, 2000
    Xs, uvs = [], []
    for _ in range(P):
        rv = rng.normal(0, 0.2, 3)
        t = np.array([rng.normal(0, 0.3), rng.normal(0, 0.3), 5.0 + rng.random()])
        X = rng.uniform(-1, 1, (n, 3))
        uv = og.project_points(X, rv, t, K) + rng.normal(0, 0.5, (n, 2))
        bad = rng.random(n) < 0.3
        uv[bad] = rng.uniform(-900, 900, (int(bad.sum()), 2))
        Xs.append(X)
        uvs.append(uv)
    Xd = torch.tensor(np.concatenate(Xs), device=device)
    ud = torch.tensor(np.concatenate(uvs), device=device)
    of = torch.tensor(np.arange(P + 1, dtype=np.int64) * n, device=device)
    cam = torch.tensor(v._cam(K), device=device).expand(P, 4).contiguous()
    holder = {}

    def step(record):
        e0 = e1 = None
        if record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        holder["r"] = v.pnp_ransac_batched(Xd, ud, of, cam)
        if record:
            e1.record()
        return (e0, e1)

    wall, kms = timed(step, args.steps, 1, barrier)
    ms = wall / args.steps * 1e3
    line = {"metric": "PnP registrations/sec", "value": P / (ms * 1e-3), "unit": "registrations/s",
            "ms_per_step": ms,
            "config": {"workload": "solvePnPRansac (sfm.py:116: 100 iters, 8 px, 0.99) + LM refine: 256 problems x "
                                   "2000 correspondences, 30% outliers",
                       "mean_ransac_iters": holder["r"]["iters"].float().mean().item()},
            "roofline": {"bound": "fp64", "kernel": "pnp_ransac_kernel", "kernel_ms": float(np.mean(kms))}}
    if cpu:
        from oracle import pnp as opnp
        t0 = time.perf_counter()
        for k in range(4):
            opnp.solve_pnp_ransac(Xs[k], uvs[k], K)
        dt = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": 4 / dt, "unit": "registrations/s", "cores": 1, "kind": "port",
                                "sample": f"4 of the 256 problems through oracle.pnp (numpy restatement of "
                                          f"OpenCV's solvePnPRansac), {dt:.2f}s"}
    return line


def ba_line(sfm, syn, device, args, barrier, cpu=True):
    """DLT + residual + FD-Jacobian over BA_PAIRS pairs x BA_OBS observations
    (pair ranges per rank)."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    sdist = importlib.import_module("3d_reconstruction_amd.dist")
    s = syn.ba_scene(BA_PAIRS, BA_OBS, seed=4)
    n = BA_PAIRS * BA_OBS
    olo, ohi = sdist.shard_range(BA_PAIRS, rank, world)
    sl = slice(olo * BA_OBS, ohi * BA_OBS)
    tt = {k: torch.from_numpy(np.ascontiguousarray(v)).to(device) for k, v in s.items()}
    x0l, x1l = tt["x0"][:, sl].contiguous(), tt["x1"][:, sl].contiguous()
    Xl, p2l, pol = tt["X"][sl].contiguous(), tt["pts2d"][sl].contiguous(), tt["pair_of_obs"][sl].contiguous()
    X4 = torch.empty((4, x0l.shape[1]), dtype=torch.float64, device=device)
    rr = torch.empty((Xl.shape[0], 2), dtype=torch.float64, device=device)
    jv = torch.empty((Xl.shape[0], 2, 9), dtype=torch.float64, device=device)

    def ba_step(record):
        e0 = e1 = None
        if record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        sfm.triangulate_batched(tt["P"], pol, x0l, x1l, out=X4)
        sfm.residual_jacobian_batched(tt["cam"], tt["K"], Xl, p2l, pol, r=rr, jv=jv)
        if record:
            e1.record()
        return (e0, e1)

    wall_b, kms_b = timed(ba_step, args.steps, args.warmup, barrier)
    wall_b = max_over_ranks(wall_b, world, device)
    b_ms = wall_b / args.steps * 1e3
    k_ms = max_over_ranks(float(np.mean(kms_b)), world, device)
    local = (ohi - olo) * BA_OBS
    gbs = local * (64 + 200) / (k_ms * 1e-3) / 1e9
    return {
        "metric": "BA obs/sec (DLT + residual + FD-Jacobian)", "value": n / (b_ms * 1e-3), "unit": "obs/s",
        "ms_per_step": b_ms, "scaling": "strong",
        "config": {"workload": f"{BA_PAIRS} pairs x {BA_OBS} obs, f64", "parallelism": f"pairs/{world}"},
        "roofline": {"bound": "hbm", "kernel": "dlt_kernel+fdjac_kernel", "kernel_ms": k_ms,
                     "algorithmic_bytes_per_obs": 64 + 200, "achieved_gbs": gbs, "peak_gbs": PEAK_HBM_GBS,
                     "frac": gbs / PEAK_HBM_GBS},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--skip-secondary", action="store_true")
    ap.add_argument("--n-img", type=int, default=N_IMG)
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL on ROCm); gloo only for rehearsal")
    ap.add_argument("--rehearse-overlap", action="store_true",
                    help="N=1 rehearsal of the N>1 RCCL path: a single-rank NCCL group + the overlapped all-gather")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("SFMHIP_BENCH_SAME_DEVICE"):  # rehearsal: every rank on device 0
        local = 0
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if args.rehearse_overlap and world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29561")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=device)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(args.dist_backend)
        barrier = lambda: dist.barrier()  # noqa: E731
    else:
        barrier = lambda: None  # noqa: E731

    sfm = importlib.import_module("3d_reconstruction_amd")
    syn = importlib.import_module("3d_reconstruction_amd.synthetic")
    sdist = importlib.import_module("3d_reconstruction_amd.dist")

    # ---------------- C3/C4: all-pairs matching ----------------------------
    n_img = args.n_img
    t0 = time.perf_counter()
    x = syn.superpoint_like(n_img, M_KPT, DIM, seed=1, device=device)
    bank = sfm.DescriptorBank.from_float(x, mode=sfm.MODE_FLOAT)
    del x
    torch.cuda.synchronize()
    log(f"[rank {rank}] descriptors ready ({time.perf_counter() - t0:.1f}s): "
        f"{n_img}x{M_KPT}x{DIM} int8 = {bank.q.numel() / 1e6:.0f} MB")
    pairs_all = sfm.all_pairs(n_img)
    P = len(pairs_all)
    num, den = 3, 4
    overlap = (world > 1 and args.dist_backend == "nccl") or args.rehearse_overlap
    if overlap:
        # chunk-major pair layout: each chunk's match launch overlaps the RCCL
        # all-gather of the previous chunk (dist.overlapped_allgather)
        pairs_dev = torch.from_numpy(pairs_all).to(device)
        mine = [(a, b) for a, b in sdist.chunk_rows(P, rank, world, MATCH_CHUNKS) if b > a]
        bufs = {a: torch.empty((b - a, bank.m_pad), dtype=torch.int32, device=device) for a, b in mine}
        lo, hi = 0, sum(b - a for a, b in mine)
    else:
        lo, hi = sdist.shard_range(P, rank, world)
        pairs_local = torch.from_numpy(pairs_all[lo:hi]).to(device)
        m0 = torch.empty((hi - lo, bank.m_pad), dtype=torch.int32, device=device)
        m16 = torch.empty((hi - lo, bank.m_pad), dtype=torch.int16, device=device)

    def compute_chunk(a, b, out):
        bank._launch(pairs_dev[a:b], num, den, bufs[a], None, None)
        out.copy_(bufs[a])

    def match_step(record):
        e0 = e1 = None
        if record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        if overlap:
            sdist.overlapped_allgather(compute_chunk, P, (bank.m_pad,), torch.int16, device, chunks=MATCH_CHUNKS,
                                       after_compute=(e1.record if record else None))
            return (e0, e1)
        bank._launch(pairs_local, num, den, m0, None, None)
        if record:
            e1.record()
        m16.copy_(m0)
        if world > 1:
            sdist.allgather_rows(m16, P)
        return (e0, e1)

    wall, kms = timed(match_step, args.steps, args.warmup, barrier)
    wall = max_over_ranks(wall, world, device)
    ms_per_step = wall / args.steps * 1e3
    kern_ms = max_over_ranks(float(np.mean(kms)), world, device)
    pairs_per_launch = hi - lo
    ops_per_launch = 2.0 * M_KPT * M_KPT * DIM * pairs_per_launch
    achieved_tops = ops_per_launch / (kern_ms * 1e-3) / 1e12
    n_matched = int(sum(int((b >= 0).sum().item()) for b in bufs.values())) if overlap else \
        int((m0 >= 0).sum().item())
    log(f"[rank {rank}] match: {ms_per_step:.2f} ms/step, kernel {kern_ms:.2f} ms, "
        f"{achieved_tops:.0f} TOPS, {n_matched} matches in shard")

    result = {
        "metric": "image-pairs matched/sec",
        "value": P / (ms_per_step * 1e-3),
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int8",
        "data": "synthetic (SuperPoint-like unit-norm descriptors, 40% cross-view overlap, seed 1)",
        "config": {"workload": f"C3/C4 all-pairs BF-L2 + ratio 0.75: {n_img} imgs x {M_KPT} kpts x {DIM}-d",
                   "pairs": P, "parallelism": f"pairs/{world}" + (
                       f" + {MATCH_CHUNKS} RCCL all-gathers (int16) overlapped with the match launches" if overlap
                       else (" + 1 all-gather (int16)" if world > 1 else ""))},
        "roofline": {"bound": "mfma", "achieved": achieved_tops, "peak": PEAK_INT8_TOPS, "unit": "TOPS",
                     "frac": achieved_tops / PEAK_INT8_TOPS,
                     "traffic": pmc_traffic("match", pairs_per_launch / P) if n_img == N_IMG else None,
                     "traffic_unit": "bytes per launch (FETCH_SIZE*2 + WRITE_SIZE, profiles/r1/traffic.json)",
                     "kernel": "match_kernel<256>", "kernel_ms": kern_ms,
                     "algorithmic": "2*M*N*d int8 ops per pair x pairs per launch"},
    }

    qcpu = {}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        for i in baseline_sample(pairs_all):
            for k in pairs_all[i]:
                if int(k) not in qcpu:
                    qcpu[int(k)] = bank.q[int(k)].cpu().numpy()

    # ---------------- C5: TSDF ------------------------------------------
    if not args.skip_secondary:
        del bank
        torch.cuda.empty_cache()
        t0 = time.perf_counter()
        depth, poses, K = syn.tsdf_scene(TSDF_F, syn.IMG_H, syn.IMG_W, device=device)
        torch.cuda.synchronize()
        log(f"[rank {rank}] depth maps ready ({time.perf_counter() - t0:.1f}s): {depth.numel() * 4 / 1e9:.2f} GB")
        R = TSDF_R
        z0, z1 = sdist.shard_range(R, rank, world)
        T = torch.zeros((R, R, R), dtype=torch.float32, device=device)
        Wt = torch.zeros_like(T)
        trunc = 3 * 2.4 / (R - 1)
        bmin, bmax = (-1.2, -1.2, -1.2), (1.2, 1.2, 1.2)

        def tsdf_step(record):
            e0 = e1 = None
            T[z0:z1].zero_()
            Wt[z0:z1].zero_()
            if record:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            if world > 1:   # each rank builds the block table of 1/N of the frames; one all-gather
                tab = sdist.shared_block_table(depth)
                sfm.tsdf_integrate(T, Wt, depth, poses, K, bmin, bmax, trunc, z0, z1, block_table=tab)
            else:
                sfm.tsdf_integrate(T, Wt, depth, poses, K, bmin, bmax, trunc, z0, z1)
            if record:
                e1.record()
            return (e0, e1)

        wall_t, kms_t = timed(tsdf_step, args.steps, args.warmup, barrier)
        wall_t = max_over_ranks(wall_t, world, device)
        t_ms = wall_t / args.steps * 1e3
        tk_ms = max_over_ranks(float(np.mean(kms_t)), world, device)
        upd = R ** 3 * TSDF_F
        local_upd = (z1 - z0) * R * R * TSDF_F
        comp_bytes = (z1 - z0) * R * R * 16 + depth.numel() * 4
        result["secondary"] = [{
            "metric": "TSDF Mvoxel/sec", "value": upd / (t_ms * 1e-3) / 1e6, "unit": "Mvoxel-updates/s",
            "ms_per_step": t_ms, "scaling": "strong",
            "config": {"workload": f"C5: {R}^3 grid x {TSDF_F} depth maps {syn.IMG_W}x{syn.IMG_H}",
                       "parallelism": f"z-slabs/{world}" + (" + 1 all-gather of the depth block table" if world > 1
                                                             else "")},
            "roofline": {"bound": "valu", "kernel": "tsdf_kernel", "kernel_ms": tk_ms,
                         "achieved_hbm_gbs": comp_bytes / (tk_ms * 1e-3) / 1e9, "peak_hbm_gbs": PEAK_HBM_GBS,
                         "achieved_tflops": 32.0 * local_upd / (tk_ms * 1e-3) / 1e12,
                         "peak_tflops": PEAK_FP32_TFLOPS,
                         "frac": (32.0 * local_upd / (tk_ms * 1e-3) / 1e12) / PEAK_FP32_TFLOPS,
                         "traffic": pmc_traffic("tsdf", (z1 - z0) / R),
                         "traffic_unit": "bytes per step (all frame-chunk launches, profiles/r1/traffic.json)"},
            "updated_voxel_frac": float((Wt[z0:z1] > 0).float().mean().item()),
        }]
        del depth, T, Wt
        torch.cuda.empty_cache()

        # ---------------- BA: DLT + residual + FD Jacobian ------------------
        result["secondary"].append(ba_line(sfm, syn, device, args, barrier))

    # ---------------- voxel anchors + vq (N=1 only; rays / obs are independent) --
    if not args.skip_secondary and world == 1:
        result["secondary"].extend(voxel_and_vq_lines(sfm, syn, device, args, barrier,
                                                      cpu=(not args.no_cpu_baseline)))
        result["secondary"].append(verify_line(sfm, syn, device, args, barrier, cpu=(not args.no_cpu_baseline)))
        result["secondary"].append(pnp_line(sfm, syn, device, args, barrier, cpu=(not args.no_cpu_baseline)))
        result["secondary"].append(train_line(sfm, syn, device, args, barrier, cpu=(not args.no_cpu_baseline)))

    # ---------------- CPU baseline (rank 0, N=1 only) ------------------------
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rate, nd, tu = cpu_baseline_match(qcpu, pairs_all, baseline_sample(pairs_all))
        result["cpu_baseline"] = {
            "value": rate, "unit": "pairs/s", "cores": blas_threads(), "kind": "port",
            "sample": f"{nd} of the {P} C3 pairs through oracle.match.bf_match_q (numpy f32 GEMM on exact "
                      f"int8 values + top-2 + exact ratio), {tu:.1f}s; linear extrapolation to all pairs "
                      f"= {P / rate:.0f}s",
        }
        if "secondary" in result:
            from oracle import voxel as ov
            dep, ps, Kk = syn.tsdf_scene(3, syn.IMG_H, syn.IMG_W, device="cpu")
            R = TSDF_R
            t0 = time.perf_counter()
            ov.tsdf_integrate(np.zeros((R, R, R), np.float32), np.zeros((R, R, R), np.float32), dep.numpy(),
                              ps.numpy(), Kk.numpy(), (-1.2,) * 3, (1.2,) * 3, np.float32(3 * 2.4 / (R - 1)))
            dt = time.perf_counter() - t0
            result["secondary"][0]["cpu_baseline"] = {
                "value": R ** 3 * 3 / dt / 1e6, "unit": "Mvoxel-updates/s", "cores": 1, "kind": "port",
                "sample": f"3 of 257 frames through oracle.voxel.tsdf_integrate (numpy f32), {dt:.1f}s"}

    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
