"""A/B the TSDF kernel configurations on the C5 workload in one process,
interleaved rounds; every config must give the same grids as the first.
usage: python tools/bench_tsdf_variants.py "U=4,CHUNK=24;U=2,SBX=4;..."
(keys are SFMHIP_TSDF_<KEY> environment knobs read per call)"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
dev = torch.device("cuda", 0)
cfgs = [dict(kv.split("=") for kv in c.split(",")) for c in sys.argv[1].split(";")]
depth, poses, K = syn.tsdf_scene(257, syn.IMG_H, syn.IMG_W, device=dev)
R = 256
keys = sorted({k for c in cfgs for k in c})
res, times = {}, {i: [] for i in range(len(cfgs))}
for rnd in range(3):
    for i, c in enumerate(cfgs):
        for k in keys:
            os.environ.pop("SFMHIP_TSDF_" + k, None)
        for k, v in c.items():
            os.environ["SFMHIP_TSDF_" + k] = v
        T = torch.zeros((R, R, R), dtype=torch.float32, device=dev)
        W = torch.zeros_like(T)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        sfm.tsdf_integrate(T, W, depth, poses, K, (-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / (R - 1))
        e1.record()
        torch.cuda.synchronize()
        times[i].append(e0.elapsed_time(e1))
        res[i] = (T, W)
for i, c in enumerate(cfgs):
    ms = float(np.median(times[i]))
    same = torch.equal(res[i][0], res[0][0]) and torch.equal(res[i][1], res[0][1])
    print(f"{c}: {ms:7.2f} ms  {R**3 * 257 / ms / 1e3:9.0f} Mvox/s  identical={same}", flush=True)
