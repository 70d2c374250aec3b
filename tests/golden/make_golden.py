"""Generate the golden fixtures in tests/golden/ from the REFERENCE code.

Run once in the build container (needs /root/reference; never on the GPU box):
    python tests/golden/make_golden.py

Only numeric inputs/outputs are written (.npz).  The reference modules are
loaded by file path at run time:
  * voxel_travesal.py   (torch injected: the file has no `import torch`)
  * sdf.py              (stub `cv2` module: cv2 is only used by SceneHelper)
  * plenoxel.py         (main guarded)
  * lightglue/lightglue.py  (loaded standalone; filter_matches only — no weights)
  * sfm.py              ba_sparse extracted with `ast` (the module body needs cv2
                        and output/*.npy)
and scipy.cluster.vq.vq / scipy.optimize._numdiff.approx_derivative, the
third-party functions the reference calls (matching.py:27, sfm.py:38).
"""
from __future__ import annotations

import ast
import importlib.util
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(OUT, "..", "..")))


def load(name, path, inject=None):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    for k, v in (inject or {}).items():
        setattr(m, k, v)
    spec.loader.exec_module(m)
    return m


def save(name, **arrays):
    np.savez_compressed(os.path.join(OUT, name), **arrays)
    print("wrote", name, {k: v.shape for k, v in arrays.items()})


def gen_vq():
    from scipy.cluster.vq import vq
    rng = np.random.default_rng(10)
    code = rng.integers(0, 256, (40, 128)).astype(np.float64)
    code[7] = code[3]            # duplicate codewords: tie -> lowest index
    code[20] = code[3]
    obs = rng.integers(0, 256, (300, 128)).astype(np.float64)
    obs[:30] = code[rng.integers(0, 40, 30)]     # exact hits (distance 0)
    obs[30:40] = code[3]                          # hits on the tied codeword
    codes, dist = vq(obs, code)
    of = rng.standard_normal((257, 128))
    cf = rng.standard_normal((33, 128))
    codes_f, dist_f = vq(of, cf)
    save("vq_golden.npz", obs=obs, code=code, codes=codes, dist=dist,
         obs_f=of, code_f=cf, codes_f=codes_f, dist_f=dist_f)


def gen_filter_matches():
    lg = load("ref_lightglue", os.path.join(REF, "lightglue", "lightglue.py"))
    from oracle.match import sq_dist
    rng = np.random.default_rng(11)
    for _ in range(100):
        qa = rng.integers(-127, 128, (200, 64)).astype(np.int8)
        qb = rng.integers(-127, 128, (180, 64)).astype(np.int8)
        qb[:60] = np.clip(qa[:60].astype(np.int32) + rng.integers(-3, 4, (60, 64)), -127, 127)
        D = sq_dist(qa, qb)
        s = np.sort(D, 1)
        t = np.sort(D, 0)
        if (s[:, 0] < s[:, 1]).all() and (t[0] < t[1]).all():
            break
    else:
        raise RuntimeError("could not draw tie-free descriptors")
    M, N = D.shape
    scores = torch.zeros((1, M + 1, N + 1), dtype=torch.float64)
    scores[0, :M, :N] = torch.from_numpy(-D.astype(np.float64))
    m0, m1, _, _ = lg.filter_matches(scores, None)
    save("filter_matches_golden.npz", qa=qa, qb=qb, m0=m0[0].numpy(), m1=m1[0].numpy())


def gen_voxel_traversal():
    vt = load("ref_voxel_traversal", os.path.join(REF, "voxel_travesal.py"), {"torch": torch})
    rng = np.random.default_rng(12)
    N = 96
    o = rng.uniform(-6, 6, (N, 3)).astype(np.float32)
    d = rng.standard_normal((N, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d[0] = [1, 0, 0]            # axis-aligned
    d[1] = [0, -1, 0]           # negative axis
    d[2] = [0, 0, 0]            # zero direction (never active)
    d[3] = [0.6, 0.8, 0.0]      # zero component
    d[4] = [-0.6, 0.0, -0.8]
    o[5] = [0.5, 0.5, 0.5]
    d[5] = [1 / np.sqrt(3)] * 3  # diagonal: tie-breaking between axes
    near = np.zeros((N, 1), np.float32)
    far = rng.uniform(0.5, 9.0, (N, 1)).astype(np.float32)
    far[6] = 0.0                # degenerate segment
    rays = np.concatenate([o, d, near, far], 1).astype(np.float32)
    out = {}
    for b in (1.0, 0.5, 2.0):
        out[f"out_{str(b).replace('.', 'p')}"] = vt.voxel_traversal(torch.from_numpy(rays), b).numpy()
    save("voxel_traversal_golden.npz", rays=rays, **out)


def gen_sdf():
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    sd = load("ref_sdf", os.path.join(REF, "sdf.py"))
    torch.manual_seed(13)
    res = (9, 10, 11)
    mn, mx = (-2, -1, -3), (3, 2, 1)
    model = sd.SDFGrid(res, mn, mx, "cpu")
    with torch.no_grad():
        model.grid.copy_(torch.randn_like(model.grid) * 0.5)
    rng = np.random.default_rng(13)
    pts = rng.uniform(-3.5, 3.5, (600, 3)).astype(np.float32)
    pts[:8] = [[-2, -1, -3], [3, 2, 1], [3, -1, 1], [0, 0, 0], [-2, 2, -3], [3, 2, -3], [-2.0001, 0, 0], [0, 2.0001, 0]]
    with torch.no_grad():
        sdf = model.get_sdf(torch.from_numpy(pts)).numpy()
        sdf2, sh = model.get_sdf_sh(torch.from_numpy(pts))
    # forward with a deterministic sample set (perturb off); z from the sampler itself
    ro = np.tile(np.array([[0.5, 0.2, 6.0]], np.float32), (64, 1)) + rng.normal(0, 0.3, (64, 3)).astype(np.float32)
    tgt = rng.uniform([-2, -1, -3], [3, 2, 1], (64, 3)).astype(np.float32)
    rd = tgt - ro
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    model.sampler.perturb = False
    ro_t, rd_t = torch.from_numpy(ro), torch.from_numpy(rd)
    _, _, _, z_vals, valid = model.sampler(model, ro_t, rd_t)
    c, pts_out, valid2 = model(ro_t, rd_t)
    save("sdf_golden.npz", grid=model.grid.detach().numpy(), bmin=np.array(mn, np.float32),
         bmax=np.array(mx, np.float32), pts=pts, sdf=sdf, sdf2=sdf2.numpy(), sh=sh.numpy(),
         rays_o=ro[valid.numpy()], rays_d=rd[valid.numpy()], z=z_vals.detach().numpy(),
         rgb=c.detach().numpy())


def gen_plenoxel():
    pl = load("ref_plenoxel", os.path.join(REF, "plenoxel.py"))
    torch.manual_seed(14)
    model = pl.NerfModel(N=16, scale=1.5)
    with torch.no_grad():
        model.voxel_grid.copy_(torch.randn_like(model.voxel_grid) * 0.5)
    rng = np.random.default_rng(14)
    x = rng.uniform(-1.8, 1.8, (500, 3)).astype(np.float32)
    d = rng.standard_normal((500, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    with torch.no_grad():
        color, sigma = model(torch.from_numpy(x), torch.from_numpy(d))
    # render_rays draws u with torch.rand: capture it with the same seed.
    B, nb, hn, hf = 48, 40, 0.5, 4.5
    ro = rng.normal(0, 0.2, (B, 3)).astype(np.float32) + np.array([0, 0, -3.0], np.float32)
    rdir = rng.normal(0, 0.2, (B, 3)).astype(np.float32) + np.array([0, 0, 1.0], np.float32)
    rdir /= np.linalg.norm(rdir, axis=1, keepdims=True)
    torch.manual_seed(15)
    with torch.no_grad():
        rgb = pl.render_rays(model, torch.from_numpy(ro), torch.from_numpy(rdir), hn=hn, hf=hf, nb_bins=nb)
    torch.manual_seed(15)
    t = torch.linspace(hn, hf, nb).expand(B, nb)
    mid = (t[:, :-1] + t[:, 1:]) / 2.
    lower = torch.cat((t[:, :1], mid), -1)
    upper = torch.cat((mid, t[:, -1:]), -1)
    u = torch.rand(t.shape)
    z = lower + (upper - lower) * u
    k = rng.standard_normal((300, 27)).astype(np.float32)
    dd = rng.standard_normal((300, 3)).astype(np.float32)
    shc = pl.eval_spherical_function(torch.from_numpy(k).reshape(-1, 3, 9), torch.from_numpy(dd)).numpy()
    save("plenoxel_golden.npz", grid=model.voxel_grid.detach().numpy(), x=x, d=d, color=color.numpy(),
         sigma=sigma.numpy(), rays_o=ro, rays_d=rdir, z=z.numpy(), rgb=rgb.numpy(), sh_k=k, sh_d=dd,
         sh_out=shc)


def gen_ba_sparse_and_jacobian():
    src = open(os.path.join(REF, "sfm.py")).read()
    tree = ast.parse(src)
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "ba_sparse")
    ns = {"np": np}
    from scipy.sparse import lil_matrix
    ns["lil_matrix"] = lil_matrix
    exec(compile(ast.Module(body=[fn], type_ignores=[]), "sfm.py:ba_sparse", "exec"), ns)
    out = {}
    for n in (3, 50):
        out[f"A{n}"] = ns["ba_sparse"](n, 6 + 3 * n, 6).toarray().astype(np.int8)
    # scipy's grouped FD Jacobian (least_squares' own path) on the restated residual
    from oracle.geometry import ba_sparse, reprojection_error
    from scipy.optimize._numdiff import approx_derivative
    from scipy.optimize._numdiff import group_columns
    rng = np.random.default_rng(16)
    n = 40
    f = 2378.98305085
    K = np.array([[f, 0, 0], [0, f, 0], [0, 0, 1]])
    X = rng.uniform([-1, -1, 4], [1, 1, 8], (n, 3))
    rvec = np.array([0.05, -0.1, 0.02])
    t = np.array([0.3, -0.05, 0.1])
    x = np.concatenate([rvec, t, X.ravel()])
    pts = rng.normal(0, 200, (n, 2))
    A = ba_sparse(n, len(x), 6)
    f0 = reprojection_error(x, K, pts)
    J = approx_derivative(reprojection_error, x, method="2-point", f0=f0, sparsity=A, args=(K, pts))
    groups = group_columns(A)
    out.update(x=x, K=K, pts=pts, f0=f0, J=J.toarray(), n_groups=np.array(groups.max() + 1))
    save("ba_golden.npz", **out)


def _stmts(path, first, last):
    """Module-level statements of a reference script whose lines lie in [first, last]."""
    tree = ast.parse(open(path).read())
    body = [n for n in tree.body if first <= n.lineno and n.end_lineno <= last]
    return compile(ast.Module(body=body, type_ignores=[]), f"{os.path.basename(path)}:{first}-{last}", "exec")


def gen_bow():
    """bow.py:14-23 (stack + kmeans k=200, iter=1) and matching.py:24-82 (vq ->
    histograms -> tf-idf -> cosine top-k -> connection graph -> start node),
    executed from the reference files on synthetic DISK-like descriptors."""
    from numpy.linalg import norm
    from scipy.cluster.vq import kmeans, vq
    rng = np.random.default_rng(17)
    n_img, m, d = 10, 200, 128
    groups = [rng.standard_normal((m, d)) for _ in range(4)]   # images 3g..3g+2 view "scene part" g
    descs = []
    for i in range(n_img):
        own = rng.standard_normal((m, d))
        share = rng.random(m) < (0.9 if i % 3 else 0.6)
        own[share] = groups[(i // 3) % 4][share] + 0.02 * rng.standard_normal((share.sum(), d))
        own /= np.linalg.norm(own, axis=1, keepdims=True)
        descs.append(own.astype(np.float32))
    all_descriptors = np.empty(n_img, dtype=object)
    for i in range(n_img):
        all_descriptors[i] = descs[i]
    ns = {"np": np, "kmeans": kmeans, "vq": vq, "norm": norm, "print": lambda *a, **k: None,
          "all_descriptors": all_descriptors}
    ns_bow = dict(ns)
    ns_bow.update(k=200, iters=1)
    np.random.seed(123)
    exec(_stmts(os.path.join(REF, "bow.py"), 14, 23), ns_bow)
    codebook, variance = ns_bow["codebook"], ns_bow["variance"]
    np.random.seed(123)
    stacked = ns_bow["all_descriptors_"]
    init_idx = np.random.choice(stacked.shape[0], size=200, replace=False)
    ns_m = dict(ns)
    ns_m.update(k=len(codebook), codebook=codebook)
    exec(_stmts(os.path.join(REF, "matching.py"), 24, 82), ns_m)
    conn = ns_m["connection"]
    save("bow_golden.npz", desc=np.stack(descs), stacked=stacked, init_idx=init_idx, codebook=codebook,
         variance=np.array(variance), words=np.stack(ns_m["visual_words"]),
         freq=ns_m["frequency_vectors"], tfidf=ns_m["tfidf"], all_idx=np.stack(ns_m["all_idx"]),
         all_score=np.stack(ns_m["all_score"]),
         conn_flat=np.array([j for c in conn for j in c], dtype=np.int64),
         conn_len=np.array([len(c) for c in conn], dtype=np.int64), start=np.array(ns_m["start"]))


if __name__ == "__main__":
    gen_vq()
    gen_filter_matches()
    gen_voxel_traversal()
    gen_sdf()
    gen_plenoxel()
    gen_ba_sparse_and_jacobian()
    gen_bow()
