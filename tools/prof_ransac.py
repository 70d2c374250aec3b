"""Phase profile of essential_ransac_kernel (256 pairs x 2048 matches).
Needs the library built with: make -C 3d_reconstruction_amd/csrc clean all EXTRA=-DSFMHIP_RANSAC_PROF
"""
import ctypes, importlib, sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
v = sfm.verify
s = syn.two_view_pairs(256, 2048, seed=6)
a, b, of = v.pack_pairs(s["pts0"], s["pts1"])
cam = v._cam(s["K"])
r = v.find_essential_batched(a, b, of, cam); torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 16)()
sfm.lib.sfmhip_debug_ransac_prof(buf)
t0 = time.perf_counter(); r = v.find_essential_batched(a, b, of, cam); torch.cuda.synchronize(); dt = time.perf_counter() - t0
sfm.lib.sfmhip_debug_ransac_prof(buf)
tot = sum(buf[:3])
print("ms", dt*1e3, "phase fractions (gen, solve, score):", [round(buf[i]/tot, 3) for i in range(3)], "per-block avg ticks(100MHz):", [buf[i]/256 for i in range(3)])
print("iters", r["iters"].float().mean().item())
names = ["basis", "rows", "GJ", "B+det", "roots", "backsub"]
sub = [buf[i] for i in range(3, 9)]
print("solver sub-phases (fraction of group-0 time):", {nm: round(v / max(1, sum(sub)), 3) for nm, v in zip(names, sub)})

print("aberth: group-0 solves", buf[13], "mean iterations", buf[12] / max(1, buf[13]))
