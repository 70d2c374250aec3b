"""Phase profile of ba_trf_kernel on bench.py's BA workload (256 pairs x 4096 obs): per pair the
wall-clock time of each phase (thread 0, 100 MHz), the mean over pairs and the slowest pairs.
Needs the library built with: make -C 3d_reconstruction_amd/csrc clean all EXTRA=-DSFMHIP_BA_PROF"""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
dev = torch.device("cuda", 0)
P, N = 256, 4096
s = syn.ba_scene(P, N, seed=4)
tt = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in s.items()}
off = torch.arange(P + 1, dtype=torch.int64, device=dev) * N
for _ in range(2):
    cam, X = tt["cam"].clone(), tt["X"].clone()
    r = sfm.ba_solve_batched(cam, tt["K"], X, tt["pts2d"], off, validate=False)
    torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (P * 10))()
assert sfm.lib.sfmhip_ba_prof_read(buf, P) == 0
t = np.array(buf[:], dtype=np.float64).reshape(P, 10) / 100.0   # us
names = ["jacobian", "regularize", "ridge", "gauss-newton", "subspace", "2-D subproblem", "trial", "accept"]
tot = t[:, :8].sum(1)
nfev = r["nfev"].cpu().numpy()
njev = r["njev"].cpu().numpy()
print("per pair (us) mean / max total:", round(tot.mean(), 1), round(tot.max(), 1))
print("phase means (us):", {nm: round(t[:, i].mean(), 1) for i, nm in enumerate(names)})
print("mean nfev / njev:", nfev.mean(), njev.mean())
per_j = t[:, 0] / np.maximum(njev, 1)
print("jacobian pass per evaluation (us): mean %.1f" % per_j.mean())
print("slowest 8 pairs: total, nfev, njev, phases")
for i in np.argsort(tot)[-8:]:
    print("  %.1f  %d  %d  %s" % (tot[i], nfev[i], njev[i], " ".join("%.1f" % v for v in t[i, :8])))
t0, t1 = t[:, 8] - t[:, 8].min(), t[:, 9] - t[:, 8].min()
print("pair start spread (us): max %.1f; end: min %.1f median %.1f max %.1f" % (t0.max(), t1.min(), np.median(t1), t1.max()))
alive = [(int(((t0 <= x) & (t1 > x)).sum())) for x in np.arange(0, t1.max(), 50.0)]
print("pairs alive every 50 us:", alive)
hist = np.bincount(nfev.astype(int))
print("nfev histogram:", {k: int(v) for k, v in enumerate(hist) if v})
