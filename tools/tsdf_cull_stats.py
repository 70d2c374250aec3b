"""C5 pre-pass statistics: fraction of (wave sub-tile, frame) pairs culled,
fused as free space and fused with gathers, for whole-tile and per-wave tests
and a few z-slab splits.  python tools/tsdf_cull_stats.py"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
sdist = importlib.import_module("3d_reconstruction_amd.dist")
dev = torch.device("cuda", 0)
depth, poses, K = syn.tsdf_scene(257, syn.IMG_H, syn.IMG_W, device=dev)
R = 256
for sub, ref in (("1", "0"), ("1", "1"), ("4", "0")):
    os.environ["SFMHIP_TSDF_CULLSUB"] = sub
    os.environ["SFMHIP_TSDF_REFINE"] = ref
    for n in (1, 8):
        z0, z1 = sdist.shard_range(R, 0, n)
        s = sfm.tsdf_cull_stats((R, R, R), depth, poses, K, (-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / (R - 1), z0, z1)
        print(f"CULLSUB={sub} REFINE={ref} slab 0/{n}: culled {s['culled_frac']:.3f} free {s['free_frac']:.3f} "
              f"full {s['full_frac']:.3f}", flush=True)
