"""Run the C5 TSDF fusion a couple of times (for rocprofv3 --pmc passes)."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
dev = torch.device("cuda", 0)
depth, poses, K = syn.tsdf_scene(int(os.environ.get("NF", "257")), syn.IMG_H, syn.IMG_W, device=dev)
R = 256
T = torch.zeros((R, R, R), dtype=torch.float32, device=dev)
W = torch.zeros_like(T)
for _ in range(int(os.environ.get("REPS", "2"))):
    T.zero_()
    W.zero_()
    sfm.tsdf_integrate(T, W, depth, poses, K, (-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / (R - 1))
torch.cuda.synchronize()
print("updated", float((W > 0).float().mean()))
