"""One C5 z-slab of an N-way split, fused repeatedly with the shared block table
(what rank r of bench.py --gpus N runs), for rocprofv3 kernel traces:
python tools/run_tsdf_slab.py N r [reps]"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
sdist = importlib.import_module("3d_reconstruction_amd.dist")
n, r = int(sys.argv[1]), int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
dev = torch.device("cuda", 0)
depth, poses, K = syn.tsdf_scene(257, syn.IMG_H, syn.IMG_W, device=dev)
R = 256
T = torch.zeros((R, R, R), dtype=torch.float32, device=dev)
W = torch.zeros_like(T)
tab = sfm.tsdf_block_table(depth)
z0, z1 = sdist.shard_range(R, r, n)
args = (depth, poses, K, (-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / (R - 1))
for _ in range(reps):
    sfm.tsdf_integrate(T, W, *args, z0, z1, block_table=tab)
torch.cuda.synchronize()
print("slab", z0, z1, "done")
