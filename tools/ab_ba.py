"""BA solve timing + result checksum on C3's 256 pairs x 4096 obs, interleaved over
SFMHIP_AB values in one process: python tools/ab_ba.py [ab values, default 0 1]."""
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
s = syn.ba_scene(256, 4096, seed=4)
tt = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in s.items()}
off = torch.arange(257, dtype=torch.int64, device=dev) * 4096
abs_ = [int(a) for a in sys.argv[1:]] or [0, 1]
ts = {a: [] for a in abs_}
sha = {}
for rnd in range(3):
    for a in abs_:
        os.environ["SFMHIP_AB"] = str(a)
        sfm.knobs_reload()
        for rep in range(4):
            cam, X = tt["cam"].clone(), tt["X"].clone()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = sfm.ba_solve_batched(cam, tt["K"], X, tt["pts2d"], off, validate=False)
            e1.record()
            torch.cuda.synchronize()
            if rep:
                ts[a].append(e0.elapsed_time(e1))
        h = hashlib.sha256()
        for t in (cam, X, r["nfev"], r["njev"], r["cost"]):
            h.update(t.cpu().numpy().tobytes())
        sha[a] = (h.hexdigest()[:16], r["nfev"].float().mean().item(), r["njev"].float().mean().item())
for a in abs_:
    print(f"ab {a}: ba {np.median(ts[a]):.3f} ms (min {min(ts[a]):.3f} max {max(ts[a]):.3f}) sha {sha[a][0]} "
          f"nfev {sha[a][1]:.4f} njev {sha[a][2]:.4f}", flush=True)
