"""A/B of two library builds (separate processes) on bench.py's geometric-verification workload
(findEssentialMat RANSAC + recoverPose, 256 pairs x 2048 matches): median time and a checksum of
every output."""
import hashlib
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
dev = torch.device("cuda", 0)
v = sfm.verify
s = syn.two_view_pairs(256, 2048, outlier_frac=0.3, noise_px=0.5, seed=6)
a, b, of = v.pack_pairs(s["pts0"], s["pts1"])
cam = torch.tensor(v._cam(s["K"]), dtype=torch.float64, device=dev).expand(256, 4).contiguous()


def step():
    r = v.find_essential_batched(a, b, of, cam)
    return r, v.recover_pose_batched(r["E"], a, b, of, cam, mask=r["mask"])


step()
ts = []
for _ in range(10):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r, rp = step()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
h = hashlib.sha256()
for d in (r, rp):
    for k in sorted(d):
        if isinstance(d[k], torch.Tensor):
            h.update(d[k].cpu().numpy().tobytes())
print(f"verify {np.median(ts):.3f} ms sha {h.hexdigest()[:16]}", flush=True)
