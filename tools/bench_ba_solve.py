"""Time the on-device BA solve on C3's 256 pairs x 4096 obs: python tools/bench_ba_solve.py"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
dev = torch.device("cuda", 0)
s = syn.ba_scene(256, 4096, seed=4)
tt = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in s.items()}
off = torch.arange(257, dtype=torch.int64, device=dev) * 4096
ts = []
for rep in range(6):
    cam, X = tt["cam"].clone(), tt["X"].clone()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = sfm.ba_solve_batched(cam, tt["K"], X, tt["pts2d"], off, validate=False)
    e1.record()
    torch.cuda.synchronize()
    if rep:
        ts.append(e0.elapsed_time(e1))
print(f"BA solve 256 x 4096: {np.median(ts):.3f} ms, nfev mean {r['nfev'].float().mean().item():.2f}, "
      f"status>0 {(r['status'] > 0).sum().item()}/256", flush=True)
