"""Phase profile of the load-balanced essential-matrix chunk kernel (ess_chunk_kernel) on bench.py's
verification workload: per work item, the solve (samples -> 16-lane five-point groups -> model list)
and the scoring, plus the five-point solver's sub-phases of group 0.
Needs the library built with: make -C 3d_reconstruction_amd/csrc clean all EXTRA=-DSFMHIP_RANSAC_PROF"""
import ctypes
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
v = sfm.verify
s = syn.two_view_pairs(256, 2048, outlier_frac=0.3, noise_px=0.5, seed=6)
a, b, of = v.pack_pairs(s["pts0"], s["pts1"])
cam = v._cam(s["K"])
v.find_essential_batched(a, b, of, cam)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 16)()
sfm.lib.sfmhip_debug_ransac_prof(buf)
v.find_essential_batched(a, b, of, cam)
torch.cuda.synchronize()
sfm.lib.sfmhip_debug_ransac_prof(buf)
items = max(1, buf[14])
print("work items", items, "per item (us, 100 MHz): solve", round(buf[9] / items / 100, 1), "score",
      round(buf[10] / items / 100, 1))
names = ["basis", "rows", "GJ", "B+det", "roots", "backsub"]
print("solver sub-phases of group 0 (us per item):", {nm: round(buf[3 + i] / items / 100, 1) for i, nm in enumerate(names)})
print("aberth: group-0 solves", buf[13], "mean iterations", buf[12] / max(1, buf[13]))
