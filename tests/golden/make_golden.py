"""Generate the golden fixtures in tests/golden/ from the REFERENCE code.

Run once in the build container (needs /root/reference; never on the GPU box):
    python tests/golden/make_golden.py

Only numeric inputs/outputs are written (.npz).  The reference modules are
loaded by file path at run time:
  * voxel_travesal.py   (torch injected: the file has no `import torch`)
  * sdf.py              (stub `cv2` module: cv2 is only used by SceneHelper)
  * plenoxel.py         (main guarded; also its training-loop body with
                        torch autograd + torch.optim.Adam, see gen_train)
  * lightglue/lightglue.py  (loaded standalone; filter_matches only — no weights)
  * sfm.py              ba_sparse extracted with `ast` (the module body needs cv2
                        and output/*.npy)
  * bow.py:14-23, matching.py:24-82 and matching.py:84-185 executed with `ast`
                        from the reference files (cv2 / matcher / tqdm stubbed
                        where the BFS calls them; see gen_bfs)
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
    save("bow_golden.npz", desc=np.stack(descs), stacked_rowsum=stacked.sum(1), init_idx=init_idx, codebook=codebook,
         variance=np.array(variance), words=np.stack(ns_m["visual_words"]),
         freq=ns_m["frequency_vectors"], tfidf=ns_m["tfidf"], all_idx=np.stack(ns_m["all_idx"]),
         all_score=np.stack(ns_m["all_score"]),
         conn_flat=np.array([j for c in conn for j in c], dtype=np.int64),
         conn_len=np.array([len(c) for c in conn], dtype=np.int64), start=np.array(ns_m["start"]))


def bfs_scene(n_img=12, k=800, stride=150, seed=18):
    """Synthetic tracks: image i sees global points [i*stride, i*stride + k) under a
    random keypoint permutation; matches of (ref, id) = shared points (ordered by
    ref keypoint) plus a few spurious pairs."""
    rng = np.random.default_rng(seed)
    perm = [rng.permutation(k) for _ in range(n_img)]          # global local-slot -> keypoint idx
    def kp_of(img, g):
        return perm[img][g - img * stride]
    table = {}
    for a in range(n_img):
        for b in range(n_img):
            if a == b:
                continue
            lo, hi = max(a, b) * stride, min(a, b) * stride + k
            g = np.arange(lo, hi) if hi > lo else np.zeros(0, np.int64)
            i0 = np.array([kp_of(a, x) for x in g], np.int64)
            i1 = np.array([kp_of(b, x) for x in g], np.int64)
            if len(i0):
                extra = rng.integers(0, k, (5, 2))
                i0 = np.concatenate([i0, extra[:, 0]])
                i1 = np.concatenate([i1, extra[:, 1]])
                _, first = np.unique(i0, return_index=True)   # one match per ref keypoint
                i0, i1 = i0[first], i1[first]
            table[(a, b)] = (i0, i1)
    conn = [[] for _ in range(n_img)]
    for a in range(n_img):
        for b in (a + 1, a + 2, a + 4):
            if b < n_img:
                conn[a].append(b)
                conn[b].append(a)
    return table, conn


def gen_bfs():
    """matching.py:84-185 (BFS pair selection + track merge) executed from the
    reference file with stubs: a table-driven matcher (LightGlue's output dict),
    cv2 RANSAC stubs that accept every match, rbd, tqdm."""
    n_img, k = 12, 800
    table, conn = bfs_scene(n_img, k)
    all_points = np.empty(n_img, dtype=object)
    img_size = np.empty(n_img, dtype=object)
    for i in range(n_img):
        all_points[i] = np.random.default_rng(i).uniform(-500, 500, (k, 2)).astype(np.float32)
        img_size[i] = np.array([1936.0, 1296.0], np.float32)
    ns = {}

    def matcher(data):
        i0, i1 = table[(ns["reference_id"], ns["id"])]
        return {"matches": [torch.from_numpy(np.stack([i0, i1], 1)).long()]}

    def rbd(d):
        return {kk: v[0] if isinstance(v, (torch.Tensor, np.ndarray, list)) else v for kk, v in d.items()}

    cv2 = types.SimpleNamespace(
        RANSAC=8,
        findEssentialMat=lambda p0, p1, K, method=None, prob=None, threshold=None: (np.eye(3), np.ones((len(p0), 1), np.uint8)),
        recoverPose=lambda E, p0, p1, K: (len(p0), np.eye(3), np.zeros((3, 1)), np.ones((len(p0), 1), np.uint8)))

    class _Bar:
        def __init__(self, total=None): pass
        def __enter__(self): return self
        def __exit__(self, *a): return False
        def update(self, n=1): pass

    degrees = [len(c) for c in conn]
    start = int(np.argmax(degrees))
    ns.update(np=np, torch=torch, cv2=cv2, rbd=rbd, matcher=matcher, tqdm=_Bar, print=lambda *a, **kw: None,
              all_points=all_points, img_size=img_size, all_descriptors=all_points, connection=conn,
              start=start, N=n_img, device=torch.device("cpu"))
    exec(_stmts(os.path.join(REF, "matching.py"), 84, 185), ns)
    queue, all_matches = ns["queue"], ns["all_matches"]
    tab_keys = np.array(sorted(table), np.int64)
    save("bfs_golden.npz", conn_flat=np.array([j for c in conn for j in c], np.int64),
         conn_len=np.array([len(c) for c in conn], np.int64), start=np.array(start), k=np.array(k),
         tab_keys=tab_keys,
         tab_len=np.array([len(table[tuple(t)][0]) for t in tab_keys], np.int64),
         tab_i0=np.concatenate([table[tuple(t)][0] for t in tab_keys]),
         tab_i1=np.concatenate([table[tuple(t)][1] for t in tab_keys]),
         img_pairs=np.array(queue[1:], np.int64),
         m_len=np.array([len(m[0]) for m in all_matches], np.int64),
         m_idx0=np.concatenate([m[0] for m in all_matches]),
         m_idx1=np.concatenate([m[1] for m in all_matches]),
         m_tracks=np.concatenate([m[2] for m in all_matches]).astype(np.int64))


def gen_sfm_triangulate():
    """sfm.py:26-52 triangulate() + ba_sparse + calculate_reprojection_error
    executed from the reference file, with cv2 replaced by the oracle's numpy
    restatements of triangulatePoints / convertPointsFromHomogeneous /
    Rodrigues / projectPoints (cv2 is not installed; parity at the OpenCV
    boundary is unpinned, the wrapper logic around it is what this pins)."""
    from scipy.optimize import least_squares
    from scipy.sparse import lil_matrix
    from oracle import geometry as og
    tree = ast.parse(open(os.path.join(REF, "sfm.py")).read())
    fns = [n for n in tree.body if isinstance(n, ast.FunctionDef)
           and n.name in ("triangulate", "ba_sparse", "calculate_reprojection_error")]

    def _rod(src):
        a = np.asarray(src, np.float64)
        return (og.rodrigues(a), None) if a.size == 3 else (og.rodrigues_inverse(a), None)

    cv2 = types.SimpleNamespace(
        triangulatePoints=lambda P0, P1, x0, x1: og.triangulate_points(P0, P1, x0, x1),
        convertPointsFromHomogeneous=lambda X: (X[:, :3] / X[:, 3:4])[:, None, :],
        Rodrigues=_rod,
        projectPoints=lambda X, r, t, K, distCoeffs=None: (og.project_points(X, r, t, K)[:, None, :], None))
    rng = np.random.default_rng(19)
    n_pts, n_img = 120, 3
    f = 2378.98305085
    K = np.array([[f, 0, 0], [0, f, 0], [0, 0, 1.0]])
    R1 = og.rodrigues([0.02, -0.15, 0.01])
    cameras = [np.hstack([np.eye(3), np.zeros((3, 1))]), np.hstack([R1, np.array([[0.8], [0.05], [0.1]])]), None]
    X = rng.uniform([-1, -1, 4], [1, 1, 7], (n_pts, 3))
    Xh = np.hstack([X, np.ones((n_pts, 1))]).T
    p0 = (K @ cameras[0] @ Xh)
    p1 = (K @ cameras[1] @ Xh)
    pts0 = (p0[:2] / p0[2]).T + rng.normal(0, 0.5, (n_pts, 2))
    pts1 = (p1[:2] / p1[2]).T + rng.normal(0, 0.5, (n_pts, 2))
    cam_in = [c.copy() if c is not None else None for c in cameras]
    # BA init pose of camera j is perturbed (as after PnP): the solve has work to do
    cameras[1] = np.hstack([og.rodrigues([0.025, -0.14, 0.012]), np.array([[0.78], [0.06], [0.11]])])
    cam_in[1] = cameras[1].copy()
    idx0 = rng.permutation(400)[:n_pts]
    idx1 = rng.permutation(400)[:n_pts]
    idx3d = np.arange(n_pts) * 2 + 1
    idx3d[5] = idx3d[4]           # a duplicated track id (possible in the reference's merge)
    n_tracks = 2 * n_pts + 5
    all_point3ds = [[None] * n_tracks, [None] * n_tracks]
    all_colors = np.empty(n_img, dtype=object)
    for i in range(n_img):
        all_colors[i] = rng.integers(0, 256, (400, 3)).astype(np.uint8)
    ns = {"np": np, "cv2": cv2, "least_squares": least_squares, "lil_matrix": lil_matrix,
          "cameras": cameras, "all_point3ds": all_point3ds, "all_colors": all_colors}
    exec(compile(ast.Module(body=fns, type_ignores=[]), "sfm.py:functions", "exec"), ns)
    focal = ns["triangulate"](0, 1, pts0, pts1, idx0, idx1, idx3d, K)
    P3 = np.array([p if p is not None else np.full(3, np.nan) for p in all_point3ds[0]])
    C3 = np.array([c if c is not None else np.full(3, -1) for c in all_point3ds[1]]).astype(np.int64)
    save("sfm_triangulate_golden.npz", K=K, cam0=cam_in[0], cam1=cam_in[1], pts0=pts0, pts1=pts1, idx0=idx0,
         idx1=idx1, idx3d=idx3d, n_tracks=np.array(n_tracks), colors=np.stack(list(all_colors)),
         focal=np.array(focal), cam1_out=cameras[1], points=P3, point_colors=C3)


def gen_train():
    """Two steps of plenoxel.py's training loop body (plenoxel.py:100-111):
    render_rays -> mse_loss -> zero_grad/backward -> Adam(lr=1e-2).step(), on
    CPU torch with the reference's NerfModel / render_rays.  The stratified
    jitter u of each step is captured by re-seeding (render_rays draws it with
    torch.rand)."""
    pl = load("ref_plenoxel_train", os.path.join(REF, "plenoxel.py"))
    torch.manual_seed(21)
    model = pl.NerfModel(N=8, scale=1.5)
    with torch.no_grad():
        model.voxel_grid.copy_(torch.randn_like(model.voxel_grid) * 0.3 + 0.2)
    grid0 = model.voxel_grid.detach().numpy().copy()
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    rng = np.random.default_rng(21)
    B, nb, hn, hf = 32, 24, 2.0, 6.0
    out = dict(grid0=grid0)
    for step in (1, 2):
        ro = (rng.normal(0, 0.3, (B, 3)) + np.array([0, 0, -4.0])).astype(np.float32)
        rdir = (rng.normal(0, 0.15, (B, 3)) + np.array([0, 0, 1.0])).astype(np.float32)
        rdir /= np.linalg.norm(rdir, axis=1, keepdims=True)
        gt = rng.uniform(0, 1, (B, 3)).astype(np.float32)
        seed = 100 + step
        torch.manual_seed(seed)
        rgb = pl.render_rays(model, torch.from_numpy(ro), torch.from_numpy(rdir), hn=hn, hf=hf, nb_bins=nb)
        loss = torch.nn.functional.mse_loss(torch.from_numpy(gt), rgb)
        opt.zero_grad()
        loss.backward()
        grad = model.voxel_grid.grad.detach().numpy().copy()
        opt.step()
        torch.manual_seed(seed)
        t = torch.linspace(hn, hf, nb).expand(B, nb)
        mid = (t[:, :-1] + t[:, 1:]) / 2.
        lower = torch.cat((t[:, :1], mid), -1)
        upper = torch.cat((mid, t[:, -1:]), -1)
        z = lower + (upper - lower) * torch.rand(t.shape)
        st = opt.state[model.voxel_grid]
        out.update({f"ro{step}": ro, f"rd{step}": rdir, f"gt{step}": gt, f"z{step}": z.numpy(),
                    f"rgb{step}": rgb.detach().numpy(), f"loss{step}": np.array(loss.item()),
                    f"grad{step}": grad, f"grid{step}": model.voxel_grid.detach().numpy().copy()})
    out.update(exp_avg2=st["exp_avg"].numpy().copy(), exp_avg_sq2=st["exp_avg_sq"].numpy().copy())
    save("train_golden.npz", **out)


def gen_sdf_sampler():
    """SDFGrid.forward (sdf.py:391-406) with the GradientBasedSampler's perturbed
    stratified samples (sdf.py:220-256): rays that miss the box, start inside it
    or have a zero direction component; the jitter t_rand (torch.rand_like at
    sdf.py:176) is captured by re-seeding."""
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    sd = load("ref_sdf_sampler", os.path.join(REF, "sdf.py"))
    torch.manual_seed(33)
    res = (9, 10, 11)
    mn, mx = (-2, -1, -3), (3, 2, 1)
    model = sd.SDFGrid(res, mn, mx, "cpu")
    with torch.no_grad():
        model.grid.copy_(torch.randn_like(model.grid) * 0.5)
    rng = np.random.default_rng(33)
    B = 48
    ro = (np.array([0.5, 0.2, 6.0]) + rng.normal(0, 1.5, (B, 3))).astype(np.float32)
    tgt = rng.uniform([-2.5, -1.5, -3.5], [3.5, 2.5, 1.5], (B, 3)).astype(np.float32)
    ro[:4] = rng.uniform([-1, 0, -2], [2, 1, 0], (4, 3))          # origins inside the box
    rd = tgt - ro
    rd[4, 0] = 0.0                                                  # zero direction components
    rd[5, 1] = 0.0
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    ro_t, rd_t = torch.from_numpy(ro), torch.from_numpy(rd)
    t_near, t_far, valid = model.sampler.ray_aabb_intersection(ro_t, rd_t, model.min_bound, model.max_bound)
    torch.manual_seed(34)
    c, pts, valid2 = model(ro_t, rd_t)
    torch.manual_seed(34)
    t_rand = torch.rand((int(valid.sum()), model.sampler.num_samples))
    save("sdf_sampler_golden.npz", grid=model.grid.detach().numpy(), bmin=np.array(mn, np.float32),
         bmax=np.array(mx, np.float32), rays_o=ro, rays_d=rd, t_near=t_near.numpy(), t_far=t_far.numpy(),
         valid=valid.numpy(), t_rand=t_rand.numpy(), pts=pts.detach().numpy(), rgb=c.detach().numpy())


def gen_sdf_train():
    """Two steps of sdf.py's training loop body (sdf.py:427-438): SDFGrid forward
    (GradientBasedSampler, 160 perturbed stratified samples) -> mse_loss on the
    valid rays -> zero_grad / backward -> Adam(lr=1e-2).step(), CPU torch, the
    reference's own SDFGrid (stub cv2).  The jitter t_rand of each step
    (torch.rand_like at sdf.py:176, the sampler's first draw) is captured by
    re-seeding; Adam also holds SDFGrid's alpha / beta, which get no gradient."""
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    sd = load("ref_sdf_train", os.path.join(REF, "sdf.py"))
    torch.manual_seed(41)
    res = (8, 9, 10)
    mn, mx = (-1.0, -1.2, -0.9), (1.1, 1.0, 1.2)
    model = sd.SDFGrid(res, mn, mx, "cpu")
    with torch.no_grad():
        model.grid.copy_(torch.randn_like(model.grid) * 0.3 + 0.15)
    grid0 = model.grid.detach().numpy().copy()
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    rng = np.random.default_rng(41)
    B = 40
    out = dict(grid0=grid0, bmin=np.array(mn, np.float32), bmax=np.array(mx, np.float32))
    for step in (1, 2):
        ro = (rng.normal(0, 0.4, (B, 3)) + np.array([0, 0, -3.5])).astype(np.float32)
        rd = (rng.normal(0, 0.25, (B, 3)) + np.array([0, 0, 1.0])).astype(np.float32)
        rd[:3] = rng.normal(0, 1, (3, 3))                          # a few rays that may miss the box
        rd /= np.linalg.norm(rd, axis=1, keepdims=True)
        gt = rng.uniform(0, 1, (B, 3)).astype(np.float32)
        seed = 400 + step
        ro_t, rd_t, gt_t = torch.from_numpy(ro), torch.from_numpy(rd), torch.from_numpy(gt)
        torch.manual_seed(seed)
        rgb, pts, valid = model(ro_t, rd_t)
        loss = torch.nn.functional.mse_loss(gt_t[valid], rgb)
        opt.zero_grad()
        loss.backward()
        grad = model.grid.grad.detach().numpy().copy()
        opt.step()
        torch.manual_seed(seed)
        t_rand = torch.rand((int(valid.sum()), model.sampler.num_samples))
        out.update({f"ro{step}": ro, f"rd{step}": rd, f"gt{step}": gt, f"t_rand{step}": t_rand.numpy(),
                    f"valid{step}": valid.numpy(), f"rgb{step}": rgb.detach().numpy(),
                    f"loss{step}": np.array(loss.item()), f"grad{step}": grad,
                    f"grid{step}": model.grid.detach().numpy().copy()})
    st = opt.state[model.grid]
    out.update(exp_avg2=st["exp_avg"].numpy().copy(), exp_avg_sq2=st["exp_avg_sq"].numpy().copy())
    save("sdf_train_golden.npz", **out)


if __name__ == "__main__":
    gen_vq()
    gen_filter_matches()
    gen_voxel_traversal()
    gen_sdf()
    gen_plenoxel()
    gen_ba_sparse_and_jacobian()
    gen_bow()
    gen_bfs()
    gen_sfm_triangulate()
    gen_train()
    gen_sdf_sampler()
    gen_sdf_train()
