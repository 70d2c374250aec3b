"""Launch the on-device BA solve (C3: 256 pairs x 4096 obs) a few times, for rocprofv3 --pmc passes."""
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
for _ in range(int(os.environ.get("REPS", "2"))):
    cam, X = tt["cam"].clone(), tt["X"].clone()
    r = sfm.ba_solve_batched(cam, tt["K"], X, tt["pts2d"], off, validate=False)
torch.cuda.synchronize()
print("nfev", r["nfev"].float().mean().item())
