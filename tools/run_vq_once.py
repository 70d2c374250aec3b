"""Launch bench.py's M2 vq (257 x 4096 obs x 200 codes x 128-d) a few times, for rocprofv3 --pmc passes."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
abi = importlib.import_module("3d_reconstruction_amd._abi")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
dev = torch.device("cuda", 0)
obs = syn.superpoint_like(257, 4096, 128, seed=3, device=dev).reshape(-1, 128).double().contiguous()
book = obs[torch.randperm(obs.shape[0], device=dev)[:200]].contiguous()
codes = torch.empty(obs.shape[0], dtype=torch.int32, device=dev)
dist = torch.empty(obs.shape[0], dtype=torch.float64, device=dev)
for _ in range(int(os.environ.get("REPS", "2"))):
    abi.call("sfmhip_vq", obs.data_ptr(), obs.shape[0], book.data_ptr(), 200, 128, codes.data_ptr(),
             dist.data_ptr(), abi.stream_ptr())
torch.cuda.synchronize()
print("codes", int(codes.max().item()))
