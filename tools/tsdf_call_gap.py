"""Wall time of back-to-back C5 integrations vs the sum of their in-stream event
times (host / allocation gaps), before and after raising the HIP default memory
pool's release threshold (hipMallocAsync scratch kept cached)."""
import ctypes
import importlib
import os
import sys
import time

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


def run(tag):
    for _ in range(2):
        sfm.tsdf_integrate(T, W, *args)
    torch.cuda.synchronize()
    evs = []
    t0 = time.perf_counter()
    for _ in range(10):
        T.zero_()
        W.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        sfm.tsdf_integrate(T, W, *args)
        e1.record()
        evs.append((e0, e1))
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / 10 * 1e3
    ev = sum(a.elapsed_time(b) for a, b in evs) / 10
    print(f"{tag}: wall {wall:.3f} ms/call, events {ev:.3f} ms/call", flush=True)


run("default pool")
hip = ctypes.CDLL("libamdhip64.so")
pool = ctypes.c_void_p()
assert hip.hipDeviceGetDefaultMemPool(ctypes.byref(pool), 0) == 0
thr = ctypes.c_uint64(2 ** 63)
assert hip.hipMemPoolSetAttribute(pool, 4, ctypes.byref(thr)) == 0   # hipMemPoolAttrReleaseThreshold
run("release threshold raised")
