"""A/B of the heavy sub-tile path (tsdf_heavy_kernel) on C5: the whole-grid call and the
N-way z-slab calls (shared block table, what each rank of bench.py --gpus N fuses), for
several SFMHIP_TSDF_HEAVY thresholds (0 = off), interleaved; every variant's grid is checked
against the default call.  python tools/tsdf_heavy_ab.py [N ...]"""
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
tab = sfm.tsdf_block_table(depth)


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


def setenv(**kw):
    for k in ("HEAVY", "HEAVY_WG", "LATENCY", "HEAVY_MODE", "PREPIPE"):
        os.environ.pop("SFMHIP_TSDF_" + k, None)
    for k, v in kw.items():
        os.environ["SFMHIP_TSDF_" + k] = str(v)


def run_whole():
    T.zero_()
    W.zero_()
    sfm.tsdf_integrate(T, W, *args)


setenv()
run_whole()
Tref, Wref = T.clone(), W.clone()
whole_variants = [dict(), dict(PREPIPE=2), dict(PREPIPE=3), dict(PREPIPE=4), dict(PREPIPE=6), dict(PREPIPE=8)]
for rep in range(2):
    for v in whole_variants:
        setenv(**v)
        t = timed(run_whole)
        same = torch.equal(T, Tref) and torch.equal(W, Wref)
        print(f"whole grid {v or 'default'}: {t:.3f} ms  identical={same}", flush=True)
slab_variants = [dict(HEAVY=0), dict(HEAVY=96, HEAVY_MODE=0), dict(HEAVY=96, HEAVY_MODE=1), dict(HEAVY=96, HEAVY_MODE=2),
                 dict(HEAVY=160, HEAVY_MODE=1), dict(HEAVY=160, HEAVY_MODE=2), dict(HEAVY=64, HEAVY_MODE=2)]
for n in [int(a) for a in sys.argv[1:]]:
    slabs = [sdist.shard_range(R, r, n) for r in range(n)]
    f_parts = [sdist.shard_range(depth.shape[0], r, n) for r in range(n)]
    t_tab = max(timed(lambda: sfm.tsdf_block_table(depth, f0, f1, out=tab)) for f0, f1 in f_parts)
    for rep in range(2):
        for v in slab_variants:
            setenv(**v)
            ts = [timed(lambda: sfm.tsdf_integrate(T, W, *args, z0, z1, block_table=tab)) for z0, z1 in slabs]
            T.zero_()
            W.zero_()
            for z0, z1 in slabs:
                sfm.tsdf_integrate(T, W, *args, z0, z1, block_table=tab)
            same = torch.equal(T, Tref) and torch.equal(W, Wref)
            print(f"N={n} {str(v):36s} slab max {max(ts):.3f} ms mean {np.mean(ts):.3f} + table {t_tab:.3f} "
                  f"identical={same} [{' '.join(f'{t:.3f}' for t in ts)}]", flush=True)
