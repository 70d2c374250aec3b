"""PnP A/B on bench.py's workload (256 x 2000, 30 % outliers): median time of the batched
solvePnPRansac call and a checksum of every output, interleaved over SFMHIP_AB values in one
process: python tools/ab_pnp.py [ab values, default 0]."""
import hashlib
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
from oracle import geometry as og   # noqa: E402  (workload generation only, as bench.py)

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
abs_ = [int(a) for a in sys.argv[1:]] or [0]
ts = {a: [] for a in abs_}
sha = {}
for rnd in range(3):
    for a in abs_:
        os.environ["SFMHIP_AB"] = str(a)
        sfm.knobs_reload()
        r = v.pnp_ransac_batched(Xd, ud, of, cam)
        for _ in range(5):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = v.pnp_ransac_batched(Xd, ud, of, cam)
            e1.record()
            torch.cuda.synchronize()
            ts[a].append(e0.elapsed_time(e1))
        h = hashlib.sha256()
        for k in sorted(r):
            if isinstance(r[k], torch.Tensor):
                h.update(r[k].cpu().numpy().tobytes())
        sha[a] = h.hexdigest()[:16]
for a in abs_:
    print(f"ab {a}: pnp {np.median(ts[a]):.3f} ms (min {min(ts[a]):.3f}) sha {sha[a]}", flush=True)
