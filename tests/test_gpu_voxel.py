"""GPU parity: V1 DDA traversal, V2 grid sample, V4 fused render, V5 TSDF.

Bars: traversal bit-exact (NaN padding included) vs the reference's own output;
grid sample within 2e-6 abs of torch's grid_sampler_3d (sdf.py / plenoxel.py
goldens); render 1e-5 (torch reduction order / exp differ); TSDF bit-exact
vs the oracle with identical op order (tolerance 1e-4 rel per north_star)."""
import importlib

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import voxel as ov

pytestmark = pytest.mark.gpu
syn = importlib.import_module("3d_reconstruction_amd.synthetic")


@pytest.mark.parametrize("b", ["1p0", "0p5", "2p0"])
def test_voxel_traversal_golden(sfm, gpu, b):
    g = golden("voxel_traversal_golden.npz")
    out = sfm.voxel_traversal(torch.from_numpy(g["rays"]).to(gpu), float(b.replace("p", "."))).cpu().numpy()
    np.testing.assert_array_equal(out, g[f"out_{b}"])


def test_voxel_traversal_random_vs_oracle(sfm, gpu):
    rng = np.random.default_rng(0)
    N = 2048
    o = rng.uniform(-20, 20, (N, 3)).astype(np.float32)
    d = rng.standard_normal((N, 3)).astype(np.float32)
    d[::7, 0] = 0
    near = rng.uniform(0, 2, (N, 1)).astype(np.float32)
    far = near + rng.uniform(0, 30, (N, 1)).astype(np.float32)
    rays = np.concatenate([o, d, near, far], 1)
    out = sfm.voxel_traversal(torch.from_numpy(rays).to(gpu), 1.0).cpu().numpy()
    np.testing.assert_array_equal(out, ov.voxel_traversal(rays, 1.0))


@pytest.mark.parametrize("direct", ["capped", "0", "1"])
def test_voxel_traversal_padding_early_exit_vs_oracle(sfm, gpu, monkeypatch, knob, direct):
    """One long ray sets S for the whole batch, so most waves end long before S
    and store their NaN padding without walking the remaining steps; a ragged
    last wave (N = 1000) and rays inactive from the start (emitted twice).
    "capped": the one-walk form (default); "0" / "1": the two-pass form with
    either fill kernel."""
    rng = np.random.default_rng(5)
    N = 1000
    o = rng.uniform(-20, 20, (N, 3)).astype(np.float32)
    d = rng.standard_normal((N, 3)).astype(np.float32)
    near = rng.uniform(0, 2, (N, 1)).astype(np.float32)
    far = near + rng.uniform(0, 8, (N, 1)).astype(np.float32)
    far[::13] = near[::13]                         # inactive from the start
    far[131] = near[131] + 150.0                   # the longest ray, in the third wave
    rays = np.concatenate([o, d, near, far], 1)
    if direct != "capped":
        monkeypatch.setenv("SFMHIP_DDA_CAP", "0")   # the two-pass form (host-side knob) ...
        knob("DDA_DIRECT", direct)                  # ... with both fill kernels
    out = sfm.voxel_traversal(torch.from_numpy(rays).to(gpu), 1.0).cpu().numpy()
    ref = ov.voxel_traversal(rays, 1.0)
    assert out.shape == ref.shape and out.shape[1] > 100
    np.testing.assert_array_equal(out, ref)


def test_grid_sample_sdf_golden(sfm, gpu):
    g = golden("sdf_golden.npz")
    vg = sfm.VoxelGrid(torch.from_numpy(g["grid"]).to(gpu), g["bmin"], g["bmax"], sfm.MASK_SDF)
    pts = torch.from_numpy(g["pts"]).to(gpu)
    sdf = vg.get_sdf(pts).cpu().numpy()
    sdf2, sh = (t.cpu().numpy() for t in vg.get_sdf_sh(pts))
    np.testing.assert_allclose(sdf, g["sdf"], rtol=0, atol=2e-6)
    np.testing.assert_allclose(sh, g["sh"], rtol=0, atol=2e-6)
    ref = ov.grid_sample(g["grid"], g["pts"], g["bmin"], g["bmax"], 0)
    np.testing.assert_array_equal(np.c_[sdf, sh], ref)   # same op order as the restatement


def test_grid_sample_plenoxel_golden(sfm, gpu):
    """NerfModel.forward (plenoxel.py:31-43) golden: sigma AND the SH colour of
    all 27 coefficients, through VoxelGrid.sample (+ the SH restatement) and
    the fused VoxelGrid.nerf_forward kernel."""
    g = golden("plenoxel_golden.npz")
    vg = sfm.VoxelGrid.plenoxel(torch.from_numpy(g["grid"]).to(gpu), 1.5)
    s = vg.sample(torch.from_numpy(g["x"]).to(gpu)).cpu().numpy()
    np.testing.assert_allclose(np.maximum(s[:, 0], 0), g["sigma"], atol=2e-6)
    inside, _ = ov.normalise(g["x"], (-1.5,) * 3, (1.5,) * 3, 1)
    col = np.where(inside[:, None], ov.sh_colour(s[:, 1:], g["d"]), 0)
    np.testing.assert_allclose(col, g["color"], atol=5e-6)
    color, sigma = (t.cpu().numpy() for t in vg.nerf_forward(torch.from_numpy(g["x"]).to(gpu),
                                                             torch.from_numpy(g["d"]).to(gpu)))
    np.testing.assert_allclose(sigma, g["sigma"], atol=2e-6)
    np.testing.assert_allclose(color, g["color"], atol=5e-6)
    assert np.array_equal(color, col.astype(np.float32)) and (color[~inside] == 0).all()


@pytest.mark.parametrize("which", ["sdf", "plenoxel"])
def test_render_golden(sfm, gpu, which):
    g = golden(f"{which}_golden.npz")
    if which == "sdf":
        vg = sfm.VoxelGrid(torch.from_numpy(g["grid"]).to(gpu), g["bmin"], g["bmax"], sfm.MASK_SDF)
    else:
        vg = sfm.VoxelGrid.plenoxel(torch.from_numpy(g["grid"]).to(gpu), 1.5)
    rgb = vg.render(torch.from_numpy(g["rays_o"]).to(gpu), torch.from_numpy(g["rays_d"]).to(gpu),
                    torch.from_numpy(g["z"]).to(gpu)).cpu().numpy()
    np.testing.assert_allclose(rgb, g["rgb"], rtol=1e-5, atol=1e-5)


def test_render_long_rays_vs_oracle(sfm, gpu):
    """S > 64 (multi-chunk transmittance carry) on a 256-sample render."""
    rng = np.random.default_rng(2)
    grid = (rng.standard_normal((1, 28, 12, 13, 14)) * 0.3).astype(np.float32)
    B, S = 40, 200
    o = rng.normal(0, 0.1, (B, 3)).astype(np.float32) + np.array([0, 0, -3], np.float32)
    d = rng.normal(0, 0.1, (B, 3)).astype(np.float32) + np.array([0, 0, 1], np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    z = np.sort(rng.uniform(0.5, 5.5, (B, S)).astype(np.float32), 1)
    vg = sfm.VoxelGrid(torch.from_numpy(grid).to(gpu), (-1, -1, -1), (1, 1, 1), sfm.MASK_SDF)
    rgb = vg.render(torch.from_numpy(o).to(gpu), torch.from_numpy(d).to(gpu), torch.from_numpy(z).to(gpu))
    np.testing.assert_allclose(rgb.cpu().numpy(), ov.render(grid, (-1, -1, -1), (1, 1, 1), 0, o, d, z),
                               rtol=1e-5, atol=1e-5)


def test_render_ray_order_bitexact(sfm, gpu, knob):
    """Batches >= 8192 rays are rendered in a device-sorted order (sfmhip_render_rays'
    Morton key + counting sort); every ray's colour must be the same bits as the unsorted
    launch (SFMHIP_RENDER_SORT=0), incl. a ragged tail and rays that miss the grid.
    Reference semantics: plenoxel.py:71-93."""
    g = torch.Generator(device=gpu).manual_seed(5)
    N, B, S = 64, 3 * 4096 + 37, 96
    vg = sfm.VoxelGrid.plenoxel(torch.randn((28, N, N, N), generator=g, device=gpu) * 0.1, 1.5)
    ro = torch.randn((B, 3), generator=g, device=gpu) * 0.4 + torch.tensor([0.0, 0.0, -3.0], device=gpu)
    rd = torch.randn((B, 3), generator=g, device=gpu) * 0.3 + torch.tensor([0.0, 0.0, 1.0], device=gpu)
    rd = rd / rd.norm(dim=1, keepdim=True)
    z = torch.sort(torch.rand((B, S), generator=g, device=gpu) * 4 + 2, 1).values.contiguous()
    knob("RENDER_SORT", 0)
    ref = vg.render(ro, rd, z)
    knob("RENDER_SORT", 1)
    got = vg.render(ro, rd, z)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("S", [100, 300])
@pytest.mark.parametrize("sort", ["0", "1"])
def test_render_sdf_plane_skip_bitexact(sfm, gpu, knob, sort, S):
    """sfmhip_render_rays_sdf (sdf from the compact channel-0 plane, colour lines only for
    samples with alpha != 0) gives the same bits as sfmhip_render_rays on a finite grid whose
    sdf is negative for about half the samples, incl. rays that miss the grid, a ray with a
    non-finite direction (full path) and a ragged tail; a grid with a non-finite SH value
    renders through the full path (VoxelGrid.finite() False).  plenoxel.py:71-93, sdf.py:376."""
    knob("RENDER_SORT", sort)
    abi = importlib.import_module("3d_reconstruction_amd._abi")
    g = torch.Generator(device=gpu).manual_seed(9)
    N, B = 48, 8192 + 77   # S = 300: several 64-sample chunks, a ragged last one
    grid = torch.randn((28, N, N + 3, N + 5), generator=g, device=gpu) * 0.1
    vg = sfm.VoxelGrid.plenoxel(grid, 1.5)
    ro = torch.randn((B, 3), generator=g, device=gpu) * 0.6 + torch.tensor([0.0, 0.0, -3.0], device=gpu)
    rd = torch.randn((B, 3), generator=g, device=gpu) * 0.4 + torch.tensor([0.0, 0.0, 1.0], device=gpu)
    rd = rd / rd.norm(dim=1, keepdim=True)
    rd[5] = torch.tensor([float("nan"), 0.0, 1.0], device=gpu)
    z = torch.sort(torch.rand((B, S), generator=g, device=gpu) * 4 + 2, 1).values.contiguous()
    bmin, bmax = np.full(3, -1.5, np.float32), np.full(3, 1.5, np.float32)
    outs = []
    for name, extra in (("sfmhip_render_rays", ()), ("sfmhip_render_rays_sdf", (vg.grid[0].data_ptr(),))):
        rgb = torch.empty((B, 3), dtype=torch.float32, device=gpu)
        abi.call(name, vg.voxel_major().data_ptr(), *extra, N, N + 3, N + 5, bmin.ctypes.data, bmax.ctypes.data, 1,
                 ro.data_ptr(), rd.data_ptr(), z.data_ptr(), B, S, rgb.data_ptr(), torch.cuda.current_stream().cuda_stream)
        outs.append(rgb)
    assert vg.finite()

    def same(a, b):   # bit-identical, NaN positions included (torch.equal is False on any NaN)
        return torch.equal(torch.isnan(a), torch.isnan(b)) and torch.equal(a.nan_to_num(7.0), b.nan_to_num(7.0))
    assert same(outs[0], outs[1]), (outs[0] - outs[1]).abs().nan_to_num(0.0).max().item()
    assert same(vg.render(ro, rd, z), outs[0])
    assert torch.isnan(outs[0][5]).all()
    grid2 = grid.clone()
    grid2[5, 10, 10, 10] = float("inf")
    vg2 = sfm.VoxelGrid.plenoxel(grid2, 1.5)
    assert not vg2.finite()
    r2 = vg2.render(ro, rd, z)
    rgb = torch.empty((B, 3), dtype=torch.float32, device=gpu)
    abi.call("sfmhip_render_rays", vg2.voxel_major().data_ptr(), N, N + 3, N + 5, bmin.ctypes.data, bmax.ctypes.data, 1,
             ro.data_ptr(), rd.data_ptr(), z.data_ptr(), B, S, rgb.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert same(r2, rgb)


def test_render_sdf_plane_grid_faces_bitexact(sfm, gpu):
    """Samples exactly on the grid's upper faces (sdf.py's inclusive mask, mode 0): their +1 corners
    are out of range, which the sdf-plane path reads clamped with weight 0 and the full path skips;
    both must give the same bits.  Axis-aligned rays on the x = max and y = max faces, and depths
    that put the last sample on z = max."""
    abi = importlib.import_module("3d_reconstruction_amd._abi")
    g = torch.Generator(device=gpu).manual_seed(11)
    N, S = 20, 64
    grid = torch.randn((28, N, N + 1, N + 2), generator=g, device=gpu) * 0.1 + 0.05
    vg = sfm.VoxelGrid.plenoxel(grid, 1.5)
    xs = torch.tensor([1.5, 1.5, -1.5, 0.3, 1.5, 0.0], device=gpu)
    ys = torch.tensor([0.2, 1.5, 1.5, 1.5, -0.7, 0.0], device=gpu)
    B = xs.numel()
    ro = torch.stack([xs, ys, torch.full_like(xs, -3.0)], 1).contiguous()
    rd = torch.tensor([0.0, 0.0, 1.0], device=gpu).expand(B, 3).contiguous()
    z = torch.linspace(1.5, 4.5, S, device=gpu).expand(B, S).contiguous()   # last sample: z = 1.5 exactly
    assert float(z[0, -1]) == 4.5
    bmin, bmax = np.full(3, -1.5, np.float32), np.full(3, 1.5, np.float32)
    outs = []
    for name, extra in (("sfmhip_render_rays", ()), ("sfmhip_render_rays_sdf", (vg.grid[0].data_ptr(),))):
        rgb = torch.empty((B, 3), dtype=torch.float32, device=gpu)
        abi.call(name, vg.voxel_major().data_ptr(), *extra, N, N + 1, N + 2, bmin.ctypes.data, bmax.ctypes.data, 0,
                 ro.data_ptr(), rd.data_ptr(), z.data_ptr(), B, S, rgb.data_ptr(), torch.cuda.current_stream().cuda_stream)
        outs.append(rgb)
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1]), (outs[0] - outs[1]).abs().max().item()


def test_voxel_traversal_cap_boundary(sfm, gpu, monkeypatch):
    """The one-walk form at the edge of its row width: cap = S (every ray fits:
    the rows' prefix is returned) and cap = S - 1 (the longest ray does not fit:
    the two-pass fallback) both give the reference's array."""
    rng = np.random.default_rng(9)
    N = 700
    o = rng.uniform(-10, 10, (N, 3)).astype(np.float32)
    d = rng.standard_normal((N, 3)).astype(np.float32)
    near = rng.uniform(0, 1, (N, 1)).astype(np.float32)
    far = near + rng.uniform(0, 12, (N, 1)).astype(np.float32)
    far[::11] = near[::11]
    rays = np.concatenate([o, d, near, far], 1)
    ref = ov.voxel_traversal(rays, 1.0)
    S = ref.shape[1]
    for cap in (S, S - 1, 2):
        monkeypatch.setenv("SFMHIP_DDA_CAP", str(cap))
        out = sfm.voxel_traversal(torch.from_numpy(rays).to(gpu), 1.0).cpu().numpy()
        assert out.shape == ref.shape
        np.testing.assert_array_equal(out, ref)


def _tsdf_case(R=48, F=12, Hd=96, Wd=128, focal=110.0):
    depth, poses, K = syn.tsdf_scene(F, Hd, Wd, focal=focal, seed=8)
    return R, depth.numpy(), poses.numpy(), K.numpy()


# "auto": the library's choice; "0" / "1": whole-grid / latency mode; "w1" / "w3": the whole-grid
# form even on thin grids, with separate block / brick / cull / refine launches (SFMHIP_AB=1) or
# with those pre-passes fused in one persistent launch (SFMHIP_AB=3); "w31": the fused form with no
# lag and no patience (SFMHIP_AB=31), so culling tasks give up on incomplete tables and leave those
# frames undecided (the fallback: every pair projected, fused in full)
LAT_MODES = ["auto", "0", "1", "w1", "w3", "w31"]


def _set_lat(knob, lat):
    if lat in ("0", "1"):
        knob("TSDF_LATENCY", lat)
    elif lat.startswith("w"):
        knob("TSDF_LATENCY", 0)
        knob("AB", lat[1:])


def _close_to_seq(Tg, Wg, Ts, Ws):
    """The order-free fusion vs the sequential running average (oracle tsdf_integrate_seq):
    same weights, T within the accumulated roundings (|dT| <= 3e-5 + 1e-4 |T|)."""
    np.testing.assert_array_equal(Wg, Ws)
    m = Ws > 0
    np.testing.assert_allclose(Tg[m], Ts[m], rtol=1e-4, atol=3e-5)


@pytest.mark.parametrize("lat", LAT_MODES)
def test_tsdf_vs_oracle_bitexact(sfm, gpu, knob, lat):
    _set_lat(knob, lat)
    R, depth, poses, K = _tsdf_case()
    T = torch.zeros((R, R, R), dtype=torch.float32, device=gpu)
    W = torch.zeros_like(T)
    sfm.tsdf_integrate(T, W, torch.from_numpy(depth), torch.from_numpy(poses), torch.from_numpy(K),
                       (-1, -1, -1), (1, 1, 1), 3 * 2.0 / (R - 1))
    args = (depth, poses, K, (-1, -1, -1), (1, 1, 1), np.float32(3 * 2.0 / (R - 1)))
    Tr, Wr = ov.tsdf_integrate(np.zeros((R, R, R), np.float32), np.zeros((R, R, R), np.float32), *args)
    Tg, Wg = T.cpu().numpy(), W.cpu().numpy()
    np.testing.assert_array_equal(Wg, Wr)
    np.testing.assert_array_equal(Tg, Tr)
    assert (Wg > 0).mean() > 0.2
    _close_to_seq(Tg, Wg, *ov.tsdf_integrate_seq(np.zeros((R, R, R), np.float32), np.zeros((R, R, R), np.float32),
                                                 *args))


@pytest.mark.parametrize("lat", LAT_MODES)
@pytest.mark.parametrize("Wd", [96, 97])
def test_tsdf_edge_cases_bitexact(sfm, gpu, knob, Wd, lat):
    """Odd / non-cubic grid (a lane's second voxel off the grid), prior (T, W) state
    including huge, tiny, negative and non-integer values, depth holes / negative
    depth, a camera plane cutting the grid (Zc <= 0), and frames with a NaN pose, an
    infinite intrinsic and a >= 2^60 translation (skipped as a whole), unaligned depth
    rows (Wd = 97): bit-exact with the oracle."""
    _set_lat(knob, lat)
    D, H, W_ = 20, 33, 45
    F, Hd = 30, 72
    depth, poses, K = syn.tsdf_scene(F, Hd, Wd, focal=80.0, seed=11)
    depth, poses, K = depth.numpy().copy(), poses.numpy().copy(), K.numpy().copy()
    rng = np.random.default_rng(5)
    depth[rng.random(depth.shape) < 0.05] = 0.0
    depth[rng.random(depth.shape) < 0.02] = -1.0
    poses[3, 2, 3] = 0.3                      # camera plane through the grid: Zc <= 0 for part of it
    poses[5, 0, 0] = np.nan
    K[7, 2] = np.inf
    poses[9, 1, 3] = 2.0 ** 61
    T0 = rng.uniform(-1, 1, (D, H, W_)).astype(np.float32)
    W0 = rng.integers(0, 4, (D, H, W_)).astype(np.float32)
    T0[0, 0, :5] = [1e35, -3e38, 2.0 ** -120, 0.0, 7.0]
    W0[0, 1, :4] = [-2.0, 2.0 ** 25, 0.5, 1e9]
    T = torch.from_numpy(T0).to(gpu)
    Wt = torch.from_numpy(W0).to(gpu)
    args = (torch.from_numpy(depth), torch.from_numpy(poses), torch.from_numpy(K), (-1, -1.2, -0.9), (1, 1.1, 1.3),
            0.15)
    sfm.tsdf_integrate(T, Wt, *args)
    Tr, Wr = ov.tsdf_integrate(T0, W0, depth, poses, K, (-1, -1.2, -0.9), (1, 1.1, 1.3), np.float32(0.15))
    np.testing.assert_array_equal(Wt.cpu().numpy(), Wr)
    np.testing.assert_array_equal(T.cpu().numpy(), Tr)
    assert (Wr > W0).mean() > 0.1


@pytest.mark.parametrize("lat", ["auto", "w1", "w3", "w31"])
def test_tsdf_multi_step_bitexact(sfm, gpu, knob, lat):
    """More than 512 frames: the call fuses them in consecutive 512-frame integration
    steps (each finished before the next), exactly as the oracle defines it; a split
    call (frames [0, 300) then [300, F)) is a different (also exact) sequence of steps.
    w3: the fused pre-pass, its tickets and frame counters re-zeroed for every step."""
    _set_lat(knob, lat)
    R, F, Hd, Wd = 20, 530, 24, 32
    depth, poses, K = syn.tsdf_scene(F, Hd, Wd, focal=30.0, seed=13)
    depth, poses, K = depth.numpy(), poses.numpy(), K.numpy()
    rng = np.random.default_rng(7)
    T0 = rng.uniform(-1, 1, (R, R, R)).astype(np.float32)
    W0 = rng.integers(0, 3, (R, R, R)).astype(np.float32)
    bnd = ((-1, -1, -1), (1, 1, 1), np.float32(0.3))
    T, Wt = torch.from_numpy(T0).to(gpu), torch.from_numpy(W0).to(gpu)
    sfm.tsdf_integrate(T, Wt, torch.from_numpy(depth), torch.from_numpy(poses), torch.from_numpy(K), *bnd)
    Tr, Wr = ov.tsdf_integrate(T0, W0, depth, poses, K, *bnd)
    np.testing.assert_array_equal(Wt.cpu().numpy(), Wr)
    np.testing.assert_array_equal(T.cpu().numpy(), Tr)
    assert (Wr - W0).max() > 300   # voxels seen by frames of both steps
    T2, W2 = torch.from_numpy(T0).to(gpu), torch.from_numpy(W0).to(gpu)
    for a, b in ((0, 300), (300, F)):
        sfm.tsdf_integrate(T2, W2, torch.from_numpy(depth[a:b]), torch.from_numpy(poses[a:b]),
                           torch.from_numpy(K[a:b]), *bnd)
    Ta, Wa = ov.tsdf_integrate(T0, W0, depth[:300], poses[:300], K[:300], *bnd)
    Ta, Wa = ov.tsdf_integrate(Ta, Wa, depth[300:], poses[300:], K[300:], *bnd)
    np.testing.assert_array_equal(W2.cpu().numpy(), Wa)
    np.testing.assert_array_equal(T2.cpu().numpy(), Ta)


def test_tsdf_modes_and_splits_identical(sfm, gpu, knob):
    """Full-resolution frames, 96^3 grid, z-slab: both modes (whole-grid with brick /
    refinement / per-voxel block test, latency) and both thin-grid forms (the default: four
    projected frames per fusion stage, no brick / refinement passes; SFMHIP_AB=1 / 3: the
    whole-grid form with separate / fused pre-passes) give the same grid bit for bit, equal to
    the oracle on sampled slices, with both culling and the free-space path active
    (cull stats)."""
    depth, poses, K = syn.tsdf_scene(40, seed=3)   # two mask words per sub-tile
    bnd = ((-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / 95)
    out = []
    # AB=1 / 3: the whole-grid form (separate / fused pre-passes, two frames per stage) where the thin
    # default differs
    variants = [{}, dict(TSDF_LATENCY=0), dict(TSDF_LATENCY=1), dict(AB=1), dict(AB=1, TSDF_LATENCY=0),
                dict(AB=3, TSDF_LATENCY=0)]
    for v in variants:
        knob("TSDF_LATENCY", -1)
        knob("AB", 0)
        for k, x in v.items():
            knob(k, x)
        T = torch.zeros((96, 96, 96), dtype=torch.float32, device=gpu)
        W = torch.zeros_like(T)
        sfm.tsdf_integrate(T, W, depth, poses, K, *bnd, z0=5, z1=90)
        out.append((T.cpu(), W.cpu()))
    for i in range(1, len(variants)):
        assert torch.equal(out[0][0], out[i][0]) and torch.equal(out[0][1], out[i][1]), variants[i]
    assert (out[0][1] > 0).float().mean() > 0.3
    st = sfm.tsdf_cull_stats((96, 96, 96), depth, poses, K, *bnd, z0=5, z1=90)
    assert st["culled"] > 0.2 * st["tested"] and st["free"] > 0.05 * st["tested"]
    dc, pc, kc = depth.numpy(), poses.numpy(), K.numpy()
    zeros = np.zeros((96, 96, 96), np.float32)
    for z0 in (5, 47, 88):
        Tr, Wr = ov.tsdf_integrate(zeros, zeros, dc, pc, kc, *bnd[:2], np.float32(bnd[2]), z0, z0 + 2)
        np.testing.assert_array_equal(out[0][1][z0:z0 + 2].numpy(), Wr[z0:z0 + 2])
        np.testing.assert_array_equal(out[0][0][z0:z0 + 2].numpy(), Tr[z0:z0 + 2])


def test_tsdf_fused_prepass_hand_off_repeated_scenes(sfm, gpu, knob):
    """The fused whole-grid pre-pass (SFMHIP_AB=3: the block pass and the culling in one
    persistent launch, the table handed from stream tasks to culling tasks inside the launch)
    against the separate launches (SFMHIP_AB=1), call after call on different scenes and
    carried grid state, so a culling task that read a stale table line (left by the previous
    call's scene at the same scratch address) would cull differently: the grids must match
    bit for bit every call.  Full-resolution depth maps, a 160^3 grid, uneven frame costs."""
    bnd = ((-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / 159)
    grids = {}
    for ab in (1, 3):
        knob("AB", ab)
        knob("TSDF_LATENCY", 0)
        T = torch.zeros((160, 160, 160), dtype=torch.float32, device=gpu)
        W = torch.zeros_like(T)
        outs = []
        for seed in (3, 11, 3, 29):
            depth, poses, K = syn.tsdf_scene(24 + seed, seed=seed, device=gpu)
            sfm.tsdf_integrate(T, W, depth, poses, K, *bnd)
            outs.append((T.cpu(), W.cpu()))
        grids[ab] = outs
    for i, ((t1, w1), (t3, w3)) in enumerate(zip(grids[1], grids[3])):
        assert torch.equal(w1, w3) and torch.equal(t1, t3), i
    assert (grids[3][-1][1] > 0).float().mean() > 0.3


@pytest.mark.parametrize("lat", LAT_MODES)
@pytest.mark.parametrize("trunc", [0.1, 0.3, 3 * 2.0 / 31, 0.0625])
def test_tsdf_free_space_near_trunc_bitexact(sfm, gpu, knob, trunc, lat):
    """Frontal planes placed so that whole tiles sit just in front of depth - mu
    (the free-space proof's boundary), several truncation distances, prior
    (T, W) state: bit-exact with the oracle."""
    _set_lat(knob, lat)
    R, F, Hd, Wd = 32, 6, 64, 80
    rng = np.random.default_rng(int(trunc * 1000))
    zs = (np.float32(-1) + np.arange(R, dtype=np.float32) * (np.float32(2) / np.float32(R - 1)))
    depth = np.empty((F, Hd, Wd), np.float32)
    poses = np.zeros((F, 3, 4), np.float32)
    poses[:, 0, 0] = poses[:, 1, 1] = poses[:, 2, 2] = 1.0
    poses[:, 2, 3] = 4.0
    for f in range(F):
        # plane at the Zc of a voxel layer + mu (+ a few ulps either way)
        zl = zs[rng.integers(4, R - 4)] + np.float32(4.0)
        depth[f] = np.nextafter(zl + np.float32(trunc), np.float32(np.inf if f % 2 else -np.inf))
        depth[f, :, : Wd // 3] += np.float32(0.5 * trunc)
    K = np.tile(np.array([[60.0, 60.0, Wd / 2, Hd / 2]], np.float32), (F, 1))
    T0 = rng.uniform(-1, 1, (R, R, R)).astype(np.float32)
    W0 = rng.integers(0, 3, (R, R, R)).astype(np.float32)
    T = torch.from_numpy(T0).to(gpu)
    Wt = torch.from_numpy(W0).to(gpu)
    sfm.tsdf_integrate(T, Wt, torch.from_numpy(depth), torch.from_numpy(poses), torch.from_numpy(K),
                       (-1, -1, -1), (1, 1, 1), trunc)
    Tr, Wr = ov.tsdf_integrate(T0, W0, depth, poses, K, (-1, -1, -1), (1, 1, 1), np.float32(trunc))
    np.testing.assert_array_equal(Wt.cpu().numpy(), Wr)
    np.testing.assert_array_equal(T.cpu().numpy(), Tr)


@pytest.mark.parametrize("lat", LAT_MODES)
def test_tsdf_camera_inside_large_grid_near_trunc_bitexact(sfm, gpu, knob, lat):
    """Cameras at the centre of a grid with a large |bmin| (translation ~0, voxels near
    the origin: the f32 voxel coordinate's error is set by |bmin|, not |v|), slightly
    rotated, with planes a few ulps either side of the f32 Zc of a voxel layer + mu (the
    free-space proof's boundary) and of Zc - mu (the skip boundary): bit-exact."""
    _set_lat(knob, lat)
    R, F, Hd, Wd = 48, 8, 64, 80
    lo, hi = np.float32(-100.0), np.float32(100.0)
    trunc = np.float32(3.0) * (hi - lo) / np.float32(R - 1)
    s = (hi - lo) / np.float32(R - 1)
    zs = lo + np.arange(R, dtype=np.float32) * s            # the kernel's f32 voxel coordinates
    rng = np.random.default_rng(21)
    depth = np.empty((F, Hd, Wd), np.float32)
    poses = np.zeros((F, 3, 4), np.float32)
    for f in range(F):
        a = np.float32(0.02 * (f - F / 2))
        c, sn = np.cos(a), np.sin(a)
        poses[f, :3, :3] = np.array([[c, 0, sn], [0, 1, 0], [-sn, 0, c]], np.float32)
        poses[f, :, 3] = rng.uniform(-1e-3, 1e-3, 3).astype(np.float32)
        zl = zs[R // 2 + 2 + f % 4]
        edge = zl + trunc if f % 2 == 0 else zl - trunc
        k = int(rng.integers(-3, 4))
        depth[f] = edge
        for _ in range(abs(k)):
            depth[f] = np.nextafter(depth[f], np.float32(np.inf if k > 0 else -np.inf))
        depth[f, :, : Wd // 4] = np.nextafter(edge, np.float32(np.inf))
    K = np.tile(np.array([[40.0, 40.0, Wd / 2, Hd / 2]], np.float32), (F, 1))
    T0 = rng.uniform(-1, 1, (R, R, R)).astype(np.float32)
    W0 = rng.integers(0, 3, (R, R, R)).astype(np.float32)
    T = torch.from_numpy(T0).to(gpu)
    Wt = torch.from_numpy(W0).to(gpu)
    bnd = ((lo,) * 3, (hi,) * 3)
    sfm.tsdf_integrate(T, Wt, torch.from_numpy(depth), torch.from_numpy(poses), torch.from_numpy(K), *bnd,
                       float(trunc))
    Tr, Wr = ov.tsdf_integrate(T0, W0, depth, poses, K, *bnd, trunc)
    np.testing.assert_array_equal(Wt.cpu().numpy(), Wr)
    np.testing.assert_array_equal(T.cpu().numpy(), Tr)
    assert (Wr > W0).mean() > 0.005


@pytest.mark.parametrize("Wd", [96, 97])
def test_tsdf_block_table_vs_oracle(sfm, gpu, Wd):
    """The pre-pass table ({min, max} per 16x16 block, NaN rules) built in two
    frame ranges equals the oracle; ragged last block row/column."""
    rng = np.random.default_rng(9)
    depth = (rng.random((5, 41, Wd), dtype=np.float32) * 4 - 1).astype(np.float32)
    depth[1, 3, 4] = np.nan
    depth[2, 32:, 80:] = np.nan      # a block of NaN only
    depth[3, 0, 0] = np.inf
    d = torch.from_numpy(depth).to(gpu)
    tab = sfm.tsdf_block_table(d, 0, 2)
    sfm.tsdf_block_table(d, 2, 5, out=tab)
    np.testing.assert_array_equal(tab.cpu().numpy(), ov.block_table(depth))


def test_tsdf_with_shared_table_bitexact(sfm, gpu):
    """tsdf_integrate with a caller-supplied block table (what the z-slab ranks
    share by all-gather) is bit-identical to the call's own pre-pass, per slab."""
    depth, poses, K = syn.tsdf_scene(20, seed=4)
    d = depth.to(gpu)
    tab = sfm.tsdf_block_table(d, 0, 9)
    sfm.tsdf_block_table(d, 9, 20, out=tab)
    args = (d, poses, K, (-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / 79)
    T1 = torch.zeros((80, 80, 80), dtype=torch.float32, device=gpu)
    W1 = torch.zeros_like(T1)
    sfm.tsdf_integrate(T1, W1, *args)
    T2, W2 = torch.zeros_like(T1), torch.zeros_like(T1)
    for z0, z1 in ((0, 10), (10, 47), (47, 80)):
        sfm.tsdf_integrate(T2, W2, *args, z0=z0, z1=z1, block_table=tab)
    assert torch.equal(T1, T2) and torch.equal(W1, W2)
    assert (W1 > 0).float().mean() > 0.3


def test_tsdf_c5_full_size_slabs_bitexact(sfm, gpu, knob):
    """The bench workload itself (C5: 256^3 grid, 257 depth maps 1936x1296, every
    pre-pass and fast path at its default): three 2-slice z-slabs of the fused grid
    equal the oracle bit for bit and the sequential running average within 1e-4 rel /
    3e-5 abs; the latency mode gives the same grid."""
    depth, poses, K = syn.tsdf_scene(257, syn.IMG_H, syn.IMG_W, device=gpu)
    R = 256
    args = (depth, poses, K, (-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / (R - 1))
    T = torch.zeros((R, R, R), dtype=torch.float32, device=gpu)
    W = torch.zeros_like(T)
    sfm.tsdf_integrate(T, W, *args)
    dc, pc, kc = depth.cpu().numpy(), poses.cpu().numpy(), K.cpu().numpy()
    zeros = np.zeros((R, R, R), np.float32)
    for z0 in (0, 127, 254):
        oargs = (dc, pc, kc, (-1.2,) * 3, (1.2,) * 3, np.float32(3 * 2.4 / (R - 1)), z0, z0 + 2)
        Tr, Wr = ov.tsdf_integrate(zeros, zeros, *oargs)
        Tg, Wg = T[z0:z0 + 2].cpu().numpy(), W[z0:z0 + 2].cpu().numpy()
        np.testing.assert_array_equal(Wg, Wr[z0:z0 + 2])
        np.testing.assert_array_equal(Tg, Tr[z0:z0 + 2])
        Ts, Ws = ov.tsdf_integrate_seq(zeros, zeros, *oargs)
        _close_to_seq(Tg, Wg, Ts[z0:z0 + 2], Ws[z0:z0 + 2])
    assert (W > 0).float().mean() > 0.5
    T2, W2 = torch.zeros_like(T), torch.zeros_like(T)
    knob("TSDF_LATENCY", 1)
    T2.zero_()
    W2.zero_()
    sfm.tsdf_integrate(T2, W2, *args)
    assert torch.equal(T, T2) and torch.equal(W, W2)


def test_tsdf_zslab_split_equals_whole(sfm, gpu):
    R, depth, poses, K = _tsdf_case(R=40, F=6)
    args = (torch.from_numpy(depth), torch.from_numpy(poses), torch.from_numpy(K), (-1, -1, -1), (1, 1, 1), 0.12)
    T1 = torch.zeros((R, R, R), dtype=torch.float32, device=gpu)
    W1 = torch.zeros_like(T1)
    sfm.tsdf_integrate(T1, W1, *args)
    T2, W2 = torch.zeros_like(T1), torch.zeros_like(T1)
    for z0, z1 in ((0, 7), (7, 21), (21, 40)):
        sfm.tsdf_integrate(T2, W2, *args, z0=z0, z1=z1)
    assert torch.equal(T1, T2) and torch.equal(W1, W2)


def test_tsdf_planar_known_answer(sfm, gpu):
    R = 24
    T = torch.zeros((R, R, R), dtype=torch.float32, device=gpu)
    W = torch.zeros_like(T)
    Hd, Wd = 64, 80
    depth = torch.full((2, Hd, Wd), 5.0)
    pose = torch.tensor([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 5.0]]).repeat(2, 1, 1)
    K = torch.tensor([[40.0, 40.0, Wd / 2, Hd / 2]]).repeat(2, 1)
    sfm.tsdf_integrate(T, W, depth, pose, K, (-1, -1, -1), (1, 1, 1), 0.2)
    zc = (np.float32(-1) + np.arange(R, dtype=np.float32) * (np.float32(2) / np.float32(R - 1))) + np.float32(5)
    exp = np.minimum(1, (5.0 - zc) / 0.2)
    col = T[:, R // 2, R // 2].cpu().numpy()
    upd = W[:, R // 2, R // 2].cpu().numpy()
    np.testing.assert_allclose(col[upd == 2], exp[upd == 2], rtol=1e-6, atol=1e-6)


def test_sdf_sampler_and_forward_match_reference(sfm, gpu):
    """V3 + V4: ray/AABB, stratified samples (bit-exact vs the reference's
    sampler incl. torch.linspace) and SDFGrid.forward's colour."""
    g = golden("sdf_sampler_golden.npz")
    vox = importlib.import_module("3d_reconstruction_amd.voxel")
    tn, tf, va = vox.ray_aabb(torch.tensor(g["rays_o"]), torch.tensor(g["rays_d"]), g["bmin"], g["bmax"])
    va = va.cpu().numpy()
    assert np.array_equal(va, g["valid"])
    assert np.array_equal(tn.cpu().numpy()[va], g["t_near"][va])
    assert np.array_equal(tf.cpu().numpy()[va], g["t_far"][va])
    vg = sfm.VoxelGrid(torch.tensor(g["grid"]), g["bmin"], g["bmax"], sfm.MASK_SDF)
    rgb, pts, valid = vg.sdf_forward(torch.tensor(g["rays_o"]), torch.tensor(g["rays_d"]), 160,
                                     torch.tensor(g["t_rand"]))
    assert np.array_equal(valid.cpu().numpy(), g["valid"])
    assert np.array_equal(pts.cpu().numpy(), g["pts"])
    np.testing.assert_allclose(rgb.cpu().numpy(), g["rgb"], rtol=1e-5, atol=1e-5)
    with pytest.raises(ValueError):
        vg.sdf_forward(torch.tensor([[50.0, 50, 50]]), torch.tensor([[1.0, 0, 0]]), 160)


def test_tsdf_integrate_rejects_bad_arguments(sfm, gpu):
    """Shape / device checks before the call: mismatched W grid,
    host grids, poses or K rows that do not match the depth frames, bad slab."""
    R, depth, poses, K = _tsdf_case(R=16, F=3)
    T = torch.zeros((R, R, R), dtype=torch.float32, device=gpu)
    W = torch.zeros_like(T)
    args = ((-1, -1, -1), (1, 1, 1), 0.2)
    with pytest.raises(ValueError, match="one shape"):
        sfm.tsdf_integrate(T, torch.zeros((R, R, R - 1), dtype=torch.float32, device=gpu), depth, poses, K, *args)
    with pytest.raises(ValueError, match="HIP device"):
        sfm.tsdf_integrate(T.cpu(), W.cpu(), depth, poses, K, *args)
    with pytest.raises(ValueError, match="poses"):
        sfm.tsdf_integrate(T, W, depth, poses[:2], K, *args)
    with pytest.raises(ValueError, match="K must"):
        sfm.tsdf_integrate(T, W, depth, poses, K[:2], *args)
    with pytest.raises(ValueError, match="z-slab"):
        sfm.tsdf_integrate(T, W, depth, poses, K, *args, 4, R + 1)
    assert float(W.abs().sum()) == 0.0                        # nothing ran


def test_tsdf_planned_uneven_slabs_bitexact(sfm, gpu):
    """Cost-planned z-slabs (tsdf_layer_stats -> plan_slabs) fused one by one
    with the shared block table equal the single-call grid bit for bit."""
    sdist = importlib.import_module("3d_reconstruction_amd.dist")
    R, depth, poses, K = _tsdf_case(R=64, F=10, Hd=96, Wd=128, focal=110.0)
    args = ((-1, -1, -1), (1, 1, 1), 0.1)
    st = sfm.tsdf_layer_stats((R, R, R), depth, poses, K, *args)
    assert st.shape == (R // 8, 3) and (st[:, 0] > 0).all() and (st[:, 1] + st[:, 2] <= st[:, 0]).all()
    tot = sfm.tsdf_cull_stats((R, R, R), torch.from_numpy(depth), torch.from_numpy(poses), torch.from_numpy(K), *args)
    assert st[:, 0].sum() == tot["tested"] and st[:, 1].sum() == tot["culled"] and st[:, 2].sum() == tot["free"]
    slabs = sdist.plan_slabs(sfm.tsdf_layer_cost(st), 3, layer=8, depth=R)
    # three contiguous slabs covering the grid, cut on the 8-layer tile boundaries
    assert len(slabs) == 3 and slabs[0][0] == 0 and slabs[-1][1] == R
    assert all(a < b and a % 8 == 0 for a, b in slabs) and all(slabs[i][1] == slabs[i + 1][0] for i in range(2))
    T0 = torch.zeros((R, R, R), dtype=torch.float32, device=gpu)
    W0 = torch.zeros_like(T0)
    sfm.tsdf_integrate(T0, W0, depth, poses, K, *args)
    tab = sfm.tsdf_block_table(torch.from_numpy(depth).to(gpu))
    T1 = torch.zeros_like(T0)
    W1 = torch.zeros_like(T0)
    for z0, z1 in slabs:
        sfm.tsdf_integrate(T1, W1, depth, poses, K, *args, z0, z1, block_table=tab)
    assert torch.equal(T0, T1) and torch.equal(W0, W1)


@pytest.mark.parametrize("lat", LAT_MODES)
def test_tsdf_degenerate_calls(sfm, gpu, knob, lat):
    """Valid but degenerate calls: zero frames and an empty z-slab leave the grids untouched;
    one frame into the smallest grid (2^3) and into a 1-voxel-thick slab equal the oracle."""
    _set_lat(knob, lat)
    R, depth, poses, K = _tsdf_case(R=16, F=4)
    dt, pt, kt = torch.from_numpy(depth), torch.from_numpy(poses), torch.from_numpy(K)
    rng = np.random.default_rng(5)
    T0 = rng.uniform(-1, 1, (R, R, R)).astype(np.float32)
    W0 = rng.integers(0, 3, (R, R, R)).astype(np.float32)
    args = ((-1, -1, -1), (1, 1, 1), 0.3)
    T, W = torch.from_numpy(T0).to(gpu), torch.from_numpy(W0).to(gpu)
    sfm.tsdf_integrate(T, W, dt[:0], pt[:0], kt[:0], *args)                   # no frames
    sfm.tsdf_integrate(T, W, dt, pt, kt, *args, 7, 7)                        # empty slab
    assert np.array_equal(T.cpu().numpy(), T0) and np.array_equal(W.cpu().numpy(), W0)
    sfm.tsdf_integrate(T, W, dt[:1], pt[:1], kt[:1], *args, 7, 8)            # one frame, one z layer
    Tr, Wr = ov.tsdf_integrate(T0, W0, depth[:1], poses[:1], K[:1], *args[:2], np.float32(args[2]), 7, 8)
    np.testing.assert_array_equal(W.cpu().numpy(), Wr)
    np.testing.assert_array_equal(T.cpu().numpy(), Tr)
    t2, w2 = torch.zeros((2, 2, 2), device=gpu), torch.zeros((2, 2, 2), device=gpu)   # the smallest grid
    sfm.tsdf_integrate(t2, w2, dt, pt, kt, (-0.5,) * 3, (0.5,) * 3, 0.3)
    Tr2, Wr2 = ov.tsdf_integrate(np.zeros((2, 2, 2), np.float32), np.zeros((2, 2, 2), np.float32), depth, poses, K,
                                 (-0.5,) * 3, (0.5,) * 3, np.float32(0.3))
    np.testing.assert_array_equal(w2.cpu().numpy(), Wr2)
    np.testing.assert_array_equal(t2.cpu().numpy(), Tr2)
