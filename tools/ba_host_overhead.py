"""Host cost vs GPU time of the BA-obs step calls (bench.py ba_line): N back-to-back calls, host
perf_counter around the enqueue loop (no sync inside) and HIP events around the same loop."""
import importlib
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
dev = torch.device("cuda", 0)
s = syn.ba_scene(256, 4096, seed=4)
tt = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in s.items()}
X4 = torch.empty((4, tt["x0"].shape[1]), dtype=torch.float64, device=dev)
rr = torch.empty((tt["X"].shape[0], 2), dtype=torch.float64, device=dev)
jv = torch.empty((tt["X"].shape[0], 2, 9), dtype=torch.float64, device=dev)
fns = {
    "dlt": lambda: sfm.triangulate_batched(tt["P"], tt["pair_of_obs"], tt["x0"], tt["x1"], out=X4),
    "fdj": lambda: sfm.residual_jacobian_batched(tt["cam"], tt["K"], tt["X"], tt["pts2d"], tt["pair_of_obs"], r=rr, jv=jv),
}
fns["step"] = lambda: (fns["dlt"](), fns["fdj"]())
for name, fn in fns.items():
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    for reps in (1, 50):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        print(f"{name:5s} x{reps:3d}: host enqueue {(t1 - t0) / reps * 1e6:7.1f} us/call, GPU {e0.elapsed_time(e1) / reps * 1e3:7.1f} us/call",
              flush=True)
