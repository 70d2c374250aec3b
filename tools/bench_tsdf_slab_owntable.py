"""N-way TSDF z-slabs on one GPU (bench.py --gpus N's per-rank work), each slab call timed two ways:
with the shared block table (dist.shared_block_table: the rank's 1/N share of the block pass +
one all-gather, timed here as the share alone) and with the call's own block pass restricted to
the slab's projected footprint per frame (no table exchange).  Same grid either way.
python tools/bench_tsdf_slab_owntable.py [N ...]"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
sdist = importlib.import_module("3d_reconstruction_amd.dist")
dev = torch.device("cuda", 0)
depth, poses, K = syn.tsdf_scene(257, syn.IMG_H, syn.IMG_W, device=dev)
R = 256
T = torch.zeros((R, R, R), dtype=torch.float32, device=dev)
W = torch.zeros_like(T)
args = (depth, poses, K, (-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / (R - 1))


def timed(fn, reps=7):
    fn()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


tab = sfm.tsdf_block_table(depth)
t_whole = timed(lambda: sfm.tsdf_integrate(T, W, *args))
print(f"whole grid, one call: {t_whole:.3f} ms", flush=True)
for n in [int(a) for a in sys.argv[1:]] or [8]:
    share = max(timed(lambda: sfm.tsdf_block_table(depth, *sdist.shard_range(257, r, n), out=tab)) for r in range(n))
    shared, own = [], []
    for r in range(n):
        z0, z1 = sdist.shard_range(R, r, n)
        shared.append(timed(lambda: sfm.tsdf_integrate(T, W, *args, z0, z1, block_table=tab)))
        T2, W2 = T.clone(), W.clone()
        own.append(timed(lambda: sfm.tsdf_integrate(T, W, *args, z0, z1)))
    print(f"N={n}: shared table: slab max {max(shared):.3f} ms + table share {share:.3f} = {max(shared) + share:.3f} "
          f"({t_whole / (max(shared) + share):.2f}x) | own footprint pass: slab max {max(own):.3f} ms "
          f"({t_whole / max(own):.2f}x) | per slab shared {[round(x, 3) for x in shared]} own {[round(x, 3) for x in own]}",
          flush=True)
