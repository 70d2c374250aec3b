"""A/B the TSDF kernel knobs (SFMHIP_TSDF_MAP / _U / _CHUNK) on the C5 workload
in one process, interleaved rounds; every config must give identical grids."""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
dev = torch.device("cuda", 0)
cfgs = [tuple(int(v) for v in c.split(":")) for c in sys.argv[1].split(",")]  # map:u:chunk:swz
depth, poses, K = syn.tsdf_scene(257, syn.IMG_H, syn.IMG_W, device=dev)
R = 256
res = {}
times = {c: [] for c in cfgs}
for rnd in range(3):
    for c in cfgs:
        os.environ["SFMHIP_TSDF_MAP"], os.environ["SFMHIP_TSDF_U"], os.environ["SFMHIP_TSDF_CHUNK"], os.environ["SFMHIP_TSDF_SWZ"] = map(str, c)
        T = torch.zeros((R, R, R), dtype=torch.float32, device=dev)
        W = torch.zeros_like(T)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        sfm.tsdf_integrate(T, W, depth, poses, K, (-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / (R - 1))
        e1.record()
        torch.cuda.synchronize()
        times[c].append(e0.elapsed_time(e1))
        res[c] = (T, W)
ref = res[cfgs[0]]
for c in cfgs:
    ms = float(np.median(times[c]))
    same = torch.equal(res[c][0], ref[0]) and torch.equal(res[c][1], ref[1])
    print(f"map {c[0]} U {c[1]} chunk {c[2]:3d} swz {c[3]}: {ms:7.2f} ms  {R**3 * 257 / ms / 1e3:9.0f} Mvox/s  identical={same}",
          flush=True)
