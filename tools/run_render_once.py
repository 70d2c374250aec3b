"""bench.py's V2+V4 render workload (plenoxel 28x256^3, 16 x 2048 rays x 192
stratified bins, one launch), run REPS times — for rocprofv3 --pmc passes.
SORT=1 renders the rays in direction-sorted order."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
N, B, S, NB = 256, 2048, 192, 16
vg = sfm.VoxelGrid.plenoxel(torch.randn((28, N, N, N), generator=g, device=dev) * 0.1, 1.5)
vg.voxel_major()
ro = torch.randn((NB * B, 3), generator=g, device=dev) * 0.2 + torch.tensor([0.0, 0.0, -3.0], device=dev)
rd = torch.randn((NB * B, 3), generator=g, device=dev) * 0.2 + torch.tensor([0.0, 0.0, 1.0], device=dev)
rd = rd / rd.norm(dim=1, keepdim=True)
t = torch.linspace(2.0, 6.0, S, device=dev).expand(NB * B, S)
mid = (t[:, :-1] + t[:, 1:]) / 2
u = torch.rand((NB * B, S), generator=g, device=dev)
z = (torch.cat([t[:, :1], mid], 1) + (torch.cat([mid, t[:, -1:]], 1) - torch.cat([t[:, :1], mid], 1)) * u).contiguous()
if os.environ.get("SORT") == "1":
    # rays through nearby voxels next to each other: key = quantised exit point at z = +1.5
    p = ro + rd * ((1.5 - ro[:, 2:3]) / rd[:, 2:3])
    q = ((p[:, :2] + 3) * 32).clamp(0, 255).long()
    key = q[:, 1] * 256 + q[:, 0]
    perm = torch.argsort(key)
    ro, rd, z = ro[perm].contiguous(), rd[perm].contiguous(), z[perm].contiguous()
for _ in range(int(os.environ.get("REPS", "3"))):
    vg.render(ro, rd, z)
torch.cuda.synchronize()
print("done")
