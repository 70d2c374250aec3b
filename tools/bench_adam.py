"""Adam kernel bandwidth at the plenoxel N=256 size (32-channel voxel-major): min/median of 10."""
import importlib, os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
abi = importlib.import_module("3d_reconstruction_amd._abi")
import ctypes
n = 256 ** 3 * 32
t = [torch.zeros(n, device="cuda") for _ in range(4)]
ts = []
for k in range(12):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    abi.call("sfmhip_adam_step", *(x.data_ptr() for x in t), n, 1e-2, 0.9, 0.999, 1e-8, k + 1, 1, abi.stream_ptr())
    e1.record(); torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
ts = sorted(ts[2:])
print(f"adam n={n}: min {ts[0]:.3f} ms median {ts[len(ts)//2]:.3f} ms -> {32*n/ts[0]/1e6:.0f} GB/s (actual bytes incl pads)")
