"""A/B of the render with and without the compact sdf plane (sfmhip_render_rays_sdf vs
sfmhip_render_rays) on the bench's plenoxel workload (28 x 256^3, 16 x 2048 rays x 192 bins),
interleaved, identical colours checked.  python tools/render_sdf_ab.py"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
abi = importlib.import_module("3d_reconstruction_amd._abi")
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(7)
N, B, S, NB = 256, 2048, 192, 16
vg = sfm.VoxelGrid.plenoxel(torch.randn((28, N, N, N), generator=g, device=dev) * 0.1, 1.5)
vm = vg.voxel_major()
ro = torch.randn((NB * B, 3), generator=g, device=dev) * 0.2 + torch.tensor([0.0, 0.0, -3.0], device=dev)
rd = torch.randn((NB * B, 3), generator=g, device=dev) * 0.2 + torch.tensor([0.0, 0.0, 1.0], device=dev)
rd = rd / rd.norm(dim=1, keepdim=True)
t = torch.linspace(2.0, 6.0, S, device=dev).expand(NB * B, S)
mid = (t[:, :-1] + t[:, 1:]) / 2
u = torch.rand((NB * B, S), generator=g, device=dev)
z = (torch.cat([t[:, :1], mid], 1) + (torch.cat([mid, t[:, -1:]], 1) - torch.cat([t[:, :1], mid], 1)) * u).contiguous()
bmin, bmax = np.full(3, -1.5, np.float32), np.full(3, 1.5, np.float32)


def run(sdf):
    rgb = torch.empty((NB * B, 3), dtype=torch.float32, device=dev)
    args = (vm.data_ptr(),) + ((vg.grid[0].data_ptr(),) if sdf else ()) + (N, N, N, bmin.ctypes.data, bmax.ctypes.data,
                                                                         1, ro.data_ptr(), rd.data_ptr(), z.data_ptr(),
                                                                         NB * B, S, rgb.data_ptr(),
                                                                         torch.cuda.current_stream().cuda_stream)
    abi.call("sfmhip_render_rays_sdf" if sdf else "sfmhip_render_rays", *args)
    return rgb


ref = run(False)
for rep in range(3):
    for sdf, occ, two in ((False, "0", "0"), (True, "4", "0"), (True, "0", "0"), (True, "0", "3"), (True, "4", "3"),
                          (True, "4", "4"), (True, "0", "4")):
        os.environ["SFMHIP_RENDER_OCC"] = occ
        os.environ["SFMHIP_RENDER_2PH"] = two
        ts = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = run(sdf)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(f"sdf_plane={sdf} occ={occ} 2ph={two}: {np.median(ts):.3f} ms (min {min(ts):.3f})  identical={torch.equal(out, ref)}",
              flush=True)
