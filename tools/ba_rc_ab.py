"""A/B of the BA solve variants (SFMHIP_BA_VARIANT: 2 records, 4/5/6 recompute at 512/256/1024
threads) on C3's 256 pairs x 4096 obs, interleaved; each variant's nfev / x compared with
variant 2's.  python tools/ba_rc_ab.py [variants...]"""
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
variants = [int(a) for a in sys.argv[1:]] or [2, 4, 5, 6]


def solve(v):
    os.environ["SFMHIP_BA_VARIANT"] = str(v)
    cam, X = tt["cam"].clone(), tt["X"].clone()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = sfm.ba_solve_batched(cam, tt["K"], X, tt["pts2d"], off, validate=False)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1), cam, X, r


_, cam0, X0, r0 = solve(2)
times = {v: [] for v in variants}
for rep in range(4):
    for v in variants:
        t, cam, X, r = solve(v)
        if rep:
            times[v].append(t)
        if rep == 1:
            dx = max((cam - cam0).abs().max().item(), (X - X0).abs().max().item())
            same_nfev = int((r["nfev"] == r0["nfev"]).sum().item())
            same_njev = int((r["njev"] == r0["njev"]).sum().item())
            print(f"variant {v}: nfev equal {same_nfev}/256, njev equal {same_njev}/256, max |dx| {dx:.3g}, "
                  f"nfev mean {r['nfev'].float().mean().item():.3f}", flush=True)
for v in variants:
    print(f"variant {v}: {np.median(times[v]):.3f} ms (min {min(times[v]):.3f})", flush=True)
