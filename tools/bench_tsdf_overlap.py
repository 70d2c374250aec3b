"""A/B: the C5 TSDF call as one launch chunk vs frames split in two with the
second chunk's block table built on a side stream while the first chunk fuses
(tsdf_block_table + tsdf_integrate(block_table=...), bit-identical grids).
usage: python tools/bench_tsdf_overlap.py [split ...]   (default 32 64 96 129)"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
vox = importlib.import_module("3d_reconstruction_amd.voxel")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
dev = torch.device("cuda", 0)
depth, poses, K = syn.tsdf_scene(257, syn.IMG_H, syn.IMG_W, device=dev)
F = depth.shape[0]
R = 256
args = (-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / (R - 1)
splits = [int(a) for a in sys.argv[1:]] or [32, 64, 96, 129]
side = torch.cuda.Stream(device=dev)
tab = torch.empty(vox.block_table_shape(*depth.shape), dtype=torch.float32, device=dev)


def run(split, T, W):
    main = torch.cuda.current_stream()
    if split is None:
        sfm.tsdf_integrate(T, W, depth, poses, K, *args)
        return
    e0 = torch.cuda.Event()
    e0.record(main)
    side.wait_event(e0)
    ev = []
    with torch.cuda.stream(side):
        for a, b in ((0, split), (split, F)):
            vox.tsdf_block_table(depth, a, b, out=tab)
            e = torch.cuda.Event()
            e.record(side)
            ev.append(e)
    for (a, b), e in zip(((0, split), (split, F)), ev):
        main.wait_event(e)
        sfm.tsdf_integrate(T, W, depth[a:b], poses[a:b], K[a:b], *args, block_table=tab[a:b])


cfgs = [None] + splits
times = {c: [] for c in cfgs}
res = {}
for rnd in range(4):
    for c in cfgs:
        T = torch.zeros((R, R, R), dtype=torch.float32, device=dev)
        W = torch.zeros_like(T)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(c, T, W)
        e1.record()
        torch.cuda.synchronize()
        if rnd:
            times[c].append(e0.elapsed_time(e1))
        res[c] = (T, W)
for c in cfgs:
    same = torch.equal(res[c][0], res[None][0]) and torch.equal(res[c][1], res[None][1])
    print(f"split {c}: {np.median(times[c]):.3f} ms (min {min(times[c]):.3f})  identical={same}", flush=True)
