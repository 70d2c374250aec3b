"""One N=8 centre slab of C5 (shared block table) called 3 times with the heavy path in the
mode given by the environment; run under rocprofv3 --kernel-trace to see the fusion kernels'
start / end on the timeline (tools/trace_tail.py style analysis)."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
dev = torch.device("cuda", 0)
depth, poses, K = syn.tsdf_scene(257, syn.IMG_H, syn.IMG_W, device=dev)
R = 256
T = torch.zeros((R, R, R), dtype=torch.float32, device=dev)
W = torch.zeros_like(T)
args = (depth, poses, K, (-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / (R - 1))
tab = sfm.tsdf_block_table(depth)
for _ in range(3):
    sfm.tsdf_integrate(T, W, *args, 64, 96, block_table=tab)
torch.cuda.synchronize()
print("done")
