"""Time the C5 fusion of each z-slab of an N-way split on one GPU (what each rank of
`bench.py --gpus N` fuses), equal-thickness slabs vs cost-planned slabs
(voxel.tsdf_layer_stats -> dist.plan_slabs): python tools/bench_tsdf_slabs.py 2 4 8"""
import importlib
import os
import sys
import time

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


def timed(fn, reps=5):
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


args = (depth, poses, K, (-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / (R - 1))
full_tab = sfm.tsdf_block_table(depth)
t_whole = timed(lambda: sfm.tsdf_integrate(T, W, *args))
print(f"whole grid, one call: {t_whole:.3f} ms", flush=True)
t0 = time.perf_counter()
stats = sfm.tsdf_layer_stats((R, R, R), *args)
print(f"layer stats (all frames): {(time.perf_counter() - t0) * 1e3:.2f} ms wall; "
      f"t_stats_kernel {timed(lambda: sfm.tsdf_layer_stats((R, R, R), *args)):.3f} ms", flush=True)
cost = sfm.tsdf_layer_cost(stats)
print("layer cost (proj-equivalent units):", [int(c) for c in cost], flush=True)
for n in [int(a) for a in sys.argv[1:]] or [8]:
    f_parts = [sdist.shard_range(depth.shape[0], r, n) for r in range(n)]
    t_tab = max(timed(lambda: sfm.tsdf_block_table(depth, f0, f1, out=full_tab)) for f0, f1 in f_parts)
    # per-rank layer stats over its 1/n of the frames (what a rank computes before planning)
    t_st = max(timed(lambda: sfm.tsdf_layer_stats((R, R, R), depth[f0:f1], poses[f0:f1], K[f0:f1], *args[3:]),
                     reps=3) for f0, f1 in f_parts)
    plans = {"equal": [sdist.shard_range(R, r, n) for r in range(n)],
             "planned": sdist.plan_slabs(cost, n, layer=8, depth=R)}
    def slab_times(slabs):
        return [timed(lambda: sfm.tsdf_integrate(T, W, *args, z0, z1, block_table=full_tab)) if z1 > z0 else 0.0
                for z0, z1 in slabs]

    for name, slabs in plans.items():
        ts = slab_times(slabs)
        print(f"N={n} {name:8s}: fusion max {max(ts):.3f} ms mean {np.mean(ts):.3f} (+ table {t_tab:.3f}, "
              f"+ stats/rank {t_st:.3f}) slabs {slabs} ms {[round(t, 3) for t in ts]}", flush=True)
    # feedback balancing as bench.py --gpus N does it (dist.rebalance_slabs on measured times, 3 rounds)
    slabs = plans["equal"]
    ts = slab_times(slabs)
    for rnd in range(1, 4):
        slabs = sdist.rebalance_slabs(slabs, ts, R)
        ts = slab_times(slabs)
        print(f"N={n} rebal {rnd} : fusion max {max(ts):.3f} ms mean {np.mean(ts):.3f} slabs {slabs} "
              f"ms {[round(t, 3) for t in ts]}", flush=True)
