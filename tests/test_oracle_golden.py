"""CPU: pin the oracle against fixtures generated from the reference code
(tests/golden/make_golden.py).  No GPU needed."""
import numpy as np
import pytest

from conftest import golden
from oracle import geometry as og
from oracle import match as om
from oracle import voxel as ov


# --- M2: vq -----------------------------------------------------------------
def test_vq_oracle_is_scipy_integer_ties():
    g = golden("vq_golden.npz")
    codes, dist = om.vq(g["obs"], g["code"])
    assert np.array_equal(codes, g["codes"]) and np.array_equal(dist, g["dist"])
    # tie rule: obs equal to the duplicated codeword 3 (= 7 = 20) -> 3
    assert (g["codes"][30:40] == 3).all()


def test_bf_top1_equals_vq_argmin_on_integer_data():
    """Anchor M1's best-index rule to scipy vq (matching.py:27): lowest index on ties."""
    g = golden("vq_golden.npz")
    qa = (g["obs"] - 128).astype(np.int8)
    qb = (g["code"] - 128).astype(np.int8)
    D = om.sq_dist(qa, qb)
    j1, d1, _ = om.top2(D)
    assert np.array_equal(j1, g["codes"])
    assert np.array_equal(np.sqrt(d1.astype(np.float64)), g["dist"])


# --- M1: mutual rule == lightglue filter_matches ------------------------------
def test_bf_mutual_equals_filter_matches():
    g = golden("filter_matches_golden.npz")
    # ratio 1 (accept iff d1 < d2; tie-free data) + mutual = filter_matches(th=None)
    m0, m1 = om.bf_match_mutual_pair(g["qa"], g["qb"], ratio=(1, 1))
    assert np.array_equal(m0, g["m0"])
    assert np.array_equal(m1, g["m1"])


def test_bf_ratio_semantics_small():
    qa = np.array([[0, 0], [10, 10], [5, 5]], np.int8)
    qb = np.array([[0, 1], [0, 3], [10, 10], [10, 10]], np.int8)
    m0, d1, d2 = om.bf_match_q(qa, qb, (3, 4), return_dist=True)
    # row0: d=[1,9,200,200]: 16*1 < 9*9 -> j=0 ; row1: tie at 2,3 -> j1=2, d2=0 -> reject
    assert m0.tolist() == [0, -1, -1] or m0[0] == 0
    assert d1[1] == 0 and d2[1] == 0 and m0[1] == -1
    assert om.bf_match_q(qa, qb[:1]).tolist() == [-1, -1, -1]


# --- M1 exact float mode: anchored to the same goldens on integer-valued data -------
def test_exact_float_oracle_equals_vq_argmin_and_filter_matches():
    """The exact-float oracle's top-1 is scipy vq's (lowest index on ties) and,
    with ratio 1 + mutual, the reference's filter_matches golden; on integer
    data it equals the quantised oracle."""
    g = golden("vq_golden.npz")
    D = om.sq_dist_exact(g["obs"].astype(np.float32), g["code"].astype(np.float32))
    j1, d1, _ = om.top2_f(D)
    assert np.array_equal(j1, g["codes"]) and np.array_equal(np.sqrt(d1), g["dist"])
    f = golden("filter_matches_golden.npz")
    m0, m1 = om.bf_match_exact_mutual_pair(f["qa"].astype(np.float32) / 127, f["qb"].astype(np.float32) / 127, (1, 1))
    assert np.array_equal(m0, f["m0"]) and np.array_equal(m1, f["m1"])
    rng = np.random.default_rng(1)
    qa, qb = rng.integers(-60, 60, (80, 64)), rng.integers(-60, 60, (90, 64))
    qb[5] = qa[2]
    qb[8] = qa[2]
    assert np.array_equal(om.bf_match_exact(qa.astype(np.float32), qb.astype(np.float32), (3, 4)),
                          om.bf_match_q(qa.astype(np.int8), qb.astype(np.int8), (3, 4)))


def test_exact_ratio_is_exact_at_the_boundary():
    d1 = np.array([9 * 2.0 ** -20, 9 * 2.0 ** -20, 0.0])
    d2 = np.array([16 * 2.0 ** -20, np.nextafter(16 * 2.0 ** -20, 1), 0.0])
    assert om.ratio_accept_exact(d1, d2, 3, 4).tolist() == [False, True, False]


# --- S4/S5: ba_sparse + FD Jacobian -----------------------------------------
def test_ba_sparse_matches_reference():
    g = golden("ba_golden.npz")
    for n in (3, 50):
        assert np.array_equal(og.ba_sparse(n, 6 + 3 * n).toarray(), g[f"A{n}"])


def test_fd_jacobian_direct_matches_scipy_grouped():
    g = golden("ba_golden.npz")
    assert int(g["n_groups"]) == 9
    J = og.fd_jacobian(g["x"], g["K"], g["pts"]).toarray()
    assert np.array_equal(J, g["J"])
    Jd = og.fd_jacobian_direct(g["x"], g["K"], g["pts"])
    n = len(g["pts"])
    dense = np.zeros_like(g["J"])
    for p in range(n):
        cols = list(range(6)) + [6 + 3 * p + c for c in range(3)]
        dense[2 * p, cols] = Jd[p, 0]
        dense[2 * p + 1, cols] = Jd[p, 1]
    assert np.array_equal(dense, g["J"])  # grouping does not change any value


def test_dlt_known_answer():
    rng = np.random.default_rng(0)
    f = 2378.98305085
    K = np.array([[f, 0, 0], [0, f, 0], [0, 0, 1]])
    R = og.rodrigues([0.1, -0.2, 0.05])
    t = np.array([[1.0], [0.1], [0.2]])
    P0 = K @ np.hstack([np.eye(3), np.zeros((3, 1))])
    P1 = K @ np.hstack([R, t])
    X = rng.uniform([-2, -2, 5], [2, 2, 10], (200, 3))
    Xh = np.hstack([X, np.ones((200, 1))]).T
    x0 = P0 @ Xh
    x1 = P1 @ Xh
    X4 = og.triangulate_points(P0, P1, x0[:2] / x0[2], x1[:2] / x1[2])
    np.testing.assert_allclose((X4[:3] / X4[3]).T, X, rtol=1e-9, atol=1e-9)


# --- V1: voxel traversal ------------------------------------------------------
@pytest.mark.parametrize("b", ["1p0", "0p5", "2p0"])
def test_voxel_traversal_oracle_matches_reference(b):
    g = golden("voxel_traversal_golden.npz")
    out = ov.voxel_traversal(g["rays"], float(b.replace("p", ".")))
    np.testing.assert_array_equal(out, g[f"out_{b}"])


# --- V2/V4: grid sample, SH colour, composite --------------------------------
def test_grid_sample_oracle_matches_sdf_py():
    g = golden("sdf_golden.npz")
    s = ov.grid_sample(g["grid"], g["pts"], g["bmin"], g["bmax"], 0)
    np.testing.assert_allclose(s[:, 0], g["sdf"], rtol=0, atol=2e-6)
    np.testing.assert_allclose(s[:, 1:], g["sh"], rtol=0, atol=2e-6)
    exact = (s[:, 0] == g["sdf"]).mean()
    assert exact > 0.95, exact


def test_plenoxel_forward_oracle():
    g = golden("plenoxel_golden.npz")
    s = ov.grid_sample(g["grid"], g["x"], (-1.5,) * 3, (1.5,) * 3, 1)
    sigma = np.maximum(s[:, 0], 0)
    inside, _ = ov.normalise(g["x"], (-1.5,) * 3, (1.5,) * 3, 1)
    col = np.where(inside[:, None], ov.sh_colour(s[:, 1:], g["d"]), 0)
    np.testing.assert_allclose(sigma, g["sigma"], atol=2e-6)
    np.testing.assert_allclose(col, g["color"], atol=5e-6)


def test_sh_colour_oracle_bitexact():
    g = golden("plenoxel_golden.npz")
    out = ov.sh_colour(g["sh_k"], g["sh_d"])
    np.testing.assert_allclose(out, g["sh_out"], rtol=0, atol=1e-6)


def test_render_oracle_matches_sdf_forward_and_plenoxel():
    g = golden("sdf_golden.npz")
    rgb = ov.render(g["grid"], g["bmin"], g["bmax"], 0, g["rays_o"], g["rays_d"], g["z"])
    np.testing.assert_allclose(rgb, g["rgb"], rtol=1e-5, atol=1e-5)
    p = golden("plenoxel_golden.npz")
    rgb = ov.render(p["grid"], (-1.5,) * 3, (1.5,) * 3, 1, p["rays_o"], p["rays_d"], p["z"])
    np.testing.assert_allclose(rgb, p["rgb"], rtol=1e-5, atol=1e-5)


# --- V5: TSDF known answer ----------------------------------------------------
def test_tsdf_oracle_planar_known_answer():
    """A fronto-parallel plane at depth Zp: every voxel in front of it within mu
    gets tsdf = min(1, (Zp - Zc)/mu) after one frame."""
    R = 24
    T = np.zeros((R, R, R), np.float32)
    W = np.zeros_like(T)
    Hd, Wd = 64, 80
    depth = np.full((1, Hd, Wd), 5.0, np.float32)
    pose = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 5.0]], np.float32)[None]
    K = np.array([[40.0, 40.0, Wd / 2, Hd / 2]], np.float32)
    Tn, Wn = ov.tsdf_integrate(T, W, depth, pose, K, (-1, -1, -1), (1, 1, 1), 0.2)
    zc = (np.float32(-1) + np.arange(R, dtype=np.float32) * (np.float32(2) / np.float32(R - 1))) + np.float32(5)
    exp = np.minimum(1, (5.0 - zc) / 0.2)
    upd = Wn[:, R // 2, R // 2] > 0
    np.testing.assert_allclose(Tn[upd, R // 2, R // 2], exp[upd], rtol=1e-6, atol=1e-6)
    assert (~upd == (exp * 0.2 < -0.2)).all()


def test_tsdf_oracle_order_free_vs_sequential():
    """The order-free fixed-point fusion (the definition the HIP path computes) against
    the sequential running average: same weights, T within 1e-4 rel / 3e-5 abs, from a
    prior state; the integration step (512 frames) is the unit of fusion."""
    import importlib
    syn = importlib.import_module("3d_reconstruction_amd.synthetic")
    R, F = 24, 20
    depth, poses, K = (a.numpy() for a in syn.tsdf_scene(F, 48, 64, focal=60.0, seed=4))
    rng = np.random.default_rng(2)
    T0 = rng.uniform(-1, 1, (R, R, R)).astype(np.float32)
    W0 = rng.integers(0, 5, (R, R, R)).astype(np.float32)
    args = (depth, poses, K, (-1, -1, -1), (1, 1, 1), np.float32(0.2))
    Tn, Wn = ov.tsdf_integrate(T0, W0, *args)
    Ts, Ws = ov.tsdf_integrate_seq(T0, W0, *args)
    np.testing.assert_array_equal(Wn, Ws)
    assert (Wn > W0).mean() > 0.2
    np.testing.assert_allclose(Tn, Ts, rtol=1e-4, atol=3e-5)
    # slab arrays (grid_depth) give the same slices
    Tz, Wz = ov.tsdf_integrate(T0[5:11], W0[5:11], *args, z0=5, z1=11, grid_depth=R)
    assert np.array_equal(Tz, Tn[5:11]) and np.array_equal(Wz, Wn[5:11])
    # one step vs two calls: a different (but equally close) sequence of steps
    Ta, Wa = ov.tsdf_integrate(T0, W0, depth[:9], poses[:9], K[:9], *args[3:])
    Ta, Wa = ov.tsdf_integrate(Ta, Wa, depth[9:], poses[9:], K[9:], *args[3:])
    np.testing.assert_array_equal(Wa, Ws)
    np.testing.assert_allclose(Ta, Ts, rtol=1e-4, atol=3e-5)


# --- BoW retrieval (§8f row 3) -------------------------------------------------
def test_bow_oracle_matches_reference():
    from oracle import bow as ob
    g = golden("bow_golden.npz")
    desc = list(g["desc"])
    assert np.array_equal(ob.stack_descriptors(desc).sum(1), g["stacked_rowsum"])   # bow.py:14-18 order
    book, dist = ob.codebook(desc, 200, 1, seed=123)
    assert np.array_equal(book, g["codebook"]) and dist == float(g["variance"])
    r = ob.retrieval(desc, g["codebook"])
    assert np.array_equal(np.stack(r["words"]), g["words"])
    assert np.array_equal(r["freq"], g["freq"]) and np.array_equal(r["tfidf"], g["tfidf"])
    assert np.array_equal(np.stack(r["idx"]), g["all_idx"])
    flat = [j for c in r["conn"] for j in c]
    assert flat == g["conn_flat"].tolist() and [len(c) for c in r["conn"]] == g["conn_len"].tolist()
    assert r["start"] == int(g["start"])


# --- §8f row 4: grid training step ------------------------------------------------
def test_train_oracle_matches_reference_torch():
    """plenoxel.py's training-loop body (render_rays + mse + autograd + Adam) on
    CPU torch vs the analytic-backward + Adam restatement."""
    from oracle import train as ot
    g = golden("train_golden.npz")
    grid = g["grid0"][0]
    m = np.zeros_like(grid)
    v = np.zeros_like(grid)
    for step in (1, 2):
        loss, rgb, grad = ot.render_loss_grad(grid, (-1.5,) * 3, (1.5,) * 3, 1, g[f"ro{step}"], g[f"rd{step}"],
                                              g[f"z{step}"], g[f"gt{step}"])
        assert abs(loss - float(g[f"loss{step}"])) <= 1e-6 * float(g[f"loss{step}"])
        np.testing.assert_allclose(rgb, g[f"rgb{step}"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(grad, g[f"grad{step}"][0], rtol=1e-5, atol=1e-9)
        grid, m, v = ot.adam_step(grid, grad, m, v, step)
        np.testing.assert_allclose(grid, g[f"grid{step}"][0], rtol=0, atol=1e-5)
    # Adam alone on torch's own gradients: bit-exact moments, >= 99.9 % bit-exact params (rest 1 ulp)
    grid, m, v = g["grid0"][0], np.zeros_like(grid), np.zeros_like(grid)
    for step in (1, 2):
        grid, m, v = ot.adam_step(grid, g[f"grad{step}"][0], m, v, step)
        assert (grid == g[f"grid{step}"][0]).mean() > 0.999
        assert np.abs(grid - g[f"grid{step}"][0]).max() <= 3e-8
    assert np.array_equal(m, g["exp_avg2"][0]) and np.array_equal(v, g["exp_avg_sq2"][0])


# --- V3: the SDF sampler's effective samples -----------------------------------------
def test_sdf_sampler_oracle_matches_reference():
    g = golden("sdf_sampler_golden.npz")
    tn, tf, va = ov.ray_aabb(g["rays_o"], g["rays_d"], g["bmin"], g["bmax"])
    assert np.array_equal(va, g["valid"])
    assert np.array_equal(tn[va], g["t_near"][va]) and np.array_equal(tf[va], g["t_far"][va])
    z = ov.sample_uniform(tn[va], tf[va], 160, g["t_rand"])
    pts = g["rays_o"][va][:, None, :] + g["rays_d"][va][:, None, :] * z[:, :, None]
    assert np.array_equal(pts, g["pts"])                                    # bit-exact incl. torch.linspace
    rgb = ov.render(g["grid"], g["bmin"], g["bmax"], 0, g["rays_o"][va], g["rays_d"][va], z)
    np.testing.assert_allclose(rgb, g["rgb"], rtol=1e-5, atol=1e-5)


def test_sdf_train_oracle_matches_reference_torch():
    """sdf.py's training-loop body (SDFGrid forward with its sampler + mse on the
    valid rays + autograd + Adam, sdf.py:427-438) on CPU torch vs the restated
    sampler, analytic backward and Adam."""
    from oracle import train as ot
    g = golden("sdf_train_golden.npz")
    grid = g["grid0"][0]
    m = np.zeros_like(grid)
    v = np.zeros_like(grid)
    for step in (1, 2):
        tn, tf, va = ov.ray_aabb(g[f"ro{step}"], g[f"rd{step}"], g["bmin"], g["bmax"])
        assert np.array_equal(va, g[f"valid{step}"])
        z = ov.sample_uniform(tn[va], tf[va], 160, g[f"t_rand{step}"])
        loss, rgb, grad = ot.render_loss_grad(grid, g["bmin"], g["bmax"], 0, g[f"ro{step}"][va], g[f"rd{step}"][va],
                                              z, g[f"gt{step}"][va])
        assert abs(loss - float(g[f"loss{step}"])) <= 1e-6 * float(g[f"loss{step}"])
        np.testing.assert_allclose(rgb, g[f"rgb{step}"], rtol=0, atol=1e-6)
        # f32 sums of up to 160 samples x 8 corners in another order: 1e-6 of the largest entry
        np.testing.assert_allclose(grad, g[f"grad{step}"][0], rtol=1e-5, atol=1e-6 * np.abs(g[f"grad{step}"]).max())
        grid, m, v = ot.adam_step(grid, grad, m, v, step)
        # Adam's step g / (sqrt(v) + 1e-8) is ill-conditioned where |g| is near eps: there
        # only its bound (lr per step) is checked
        well = np.ones(grid.shape, bool)
        for s_ in range(1, step + 1):
            well &= np.abs(g[f"grad{s_}"][0]) > 1e-7
        np.testing.assert_allclose(grid[well], g[f"grid{step}"][0][well], rtol=0, atol=1e-5)
        assert np.abs(grid - g[f"grid{step}"][0]).max() <= 2e-2 * step
