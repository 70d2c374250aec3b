"""Phase profile of pnp_ransac_kernel on bench.py's PnP workload (256 x 2000).
Needs the library built with: make -C 3d_reconstruction_amd/csrc clean all EXTRA=-DSFMHIP_PNP_PROF"""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
from oracle import geometry as og   # noqa: E402  (workload generation only)

dev = torch.device("cuda", 0)
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
Xd = torch.tensor(np.concatenate(Xs), device=dev)
ud = torch.tensor(np.concatenate(uvs), device=dev)
of = torch.tensor(np.arange(P + 1, dtype=np.int64) * n, device=dev)
cam = torch.tensor(v._cam(K), device=dev).expand(P, 4).contiguous()
r = v.pnp_ransac_batched(Xd, ud, of, cam)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 16)()
sfm.lib.sfmhip_debug_pnp_prof(buf)
r = v.pnp_ransac_batched(Xd, ud, of, cam)
torch.cuda.synchronize()
sfm.lib.sfmhip_debug_pnp_prof(buf)
names = ["sample draw", "EPnP solve", "score", "replay", "inlier mask", "LM refine"]
tot = sum(buf[:6])
print("per-problem mean (us, wall clock 100 MHz):", {nm: round(buf[i] / P / 100, 1) for i, nm in enumerate(names)})
print("fractions:", {nm: round(buf[i] / max(tot, 1), 3) for i, nm in enumerate(names)})
sub = ["load+prepare", "MtM", "Jacobi", "signs+L/rho", "betas+GN+R_t", "select+rodrigues_inv"]
print("EPnP sub-phases of group 0 (us per problem):", {nm: round(buf[6 + i] / P / 100, 1) for i, nm in enumerate(sub)})
esub = ["householder", "trisection", "inverse iteration", "back-transform"]
print("eig sub-phases of group 0 (us per problem):", {nm: round(buf[12 + i] / P / 100, 1) for i, nm in enumerate(esub)})
wg = (ctypes.c_ulonglong * 4096)()
sfm.lib.sfmhip_debug_pnp_wg(wg)
w = np.array(wg[:4 * P], dtype=np.int64).reshape(P, 4)
st = (w[:, 0] - w[:, 0].min()) / 100.0
dur = (w[:, 1] - w[:, 0]) / 100.0
print("workgroup start offsets (us): min/median/max", st.min(), np.median(st), st.max(), " n started > 50 us late:", int((st > 50).sum()))
print("workgroup durations (us): min/median/mean/max", dur.min(), np.median(dur), dur.mean().round(1), dur.max())
print("span first start -> last end (us):", (w[:, 1].max() - w[:, 0].min()) / 100.0)
it = r["iters"].cpu().numpy()
ep = (w[:, 2] - w[:, 0]) / 100.0
rs = (w[:, 3] - w[:, 2]) / 100.0
lm = (w[:, 1] - w[:, 3]) / 100.0
print("per workgroup (us) mean / max: to first EPnP end %.1f / %.1f, rest of RANSAC %.1f / %.1f, LM %.1f / %.1f" % (
    ep.mean(), ep.max(), rs.mean(), rs.max(), lm.mean(), lm.max()))
print("slowest 8 problems (total, to EPnP end, RANSAC rest, LM us; iters):")
for i in np.argsort(dur)[-8:]:
    print("  %.1f  %.1f  %.1f  %.1f  %d" % (dur[i], ep[i], rs[i], lm[i], it[i]))
print("mean ransac iters", r["iters"].float().mean().item())
