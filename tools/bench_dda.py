"""Time bench.py's V1 workload (4096 rays, bin 1, far U(0,64)): the whole sfm.voxel_traversal call
(count pass, host S, fill pass), median of 20, plus a checksum of the output."""
import hashlib
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(11)
nr = 4096
o = torch.rand((nr, 3), generator=g, device=dev) * 64 - 32
dvec = torch.randn((nr, 3), generator=g, device=dev)
far = torch.rand((nr, 1), generator=g, device=dev) * 64
rays = torch.cat([o, dvec / dvec.norm(dim=1, keepdim=True), torch.zeros_like(far), far], 1).contiguous()
out = sfm.voxel_traversal(rays, 1.0)
ts = []
for _ in range(20):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = sfm.voxel_traversal(rays, 1.0)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
h = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
print(f"dda {np.median(ts):.3f} ms (min {min(ts):.3f}) S={out.shape[1]} sha {h}", flush=True)
