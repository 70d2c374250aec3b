"""Candidate statistics of the exact-mode resolve on the C3 bench workload (one call): rows, mean and
max candidates per row, rows over the cap (every candidate evaluated), a histogram by 64.
Needs the library built with: make -C 3d_reconstruction_amd/csrc clean all EXTRA=-DSFMHIP_RESOLVE_PROF"""
import ctypes
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
dev = torch.device("cuda", 0)
x = syn.superpoint_like(257, 4096, 256, seed=1, device=dev)
bank = sfm.DescriptorBank.from_float(x, mode=sfm.MODE_FLOAT)
del x
pairs = torch.from_numpy(sfm.all_pairs(257)).to(dev)
out = torch.empty((pairs.shape[0], bank.m_pad), dtype=torch.int32, device=dev)
bank.match(pairs, ratio=0.75, out=out, exact=True)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 16)()
sfm.lib.sfmhip_debug_resolve_prof(buf)   # reset is not needed: one call measured below minus the first
first = list(buf)
bank.match(pairs, ratio=0.75, out=out, exact=True)
torch.cuda.synchronize()
sfm.lib.sfmhip_debug_resolve_prof(buf)
d = [b - a for a, b in zip(first, buf)]
rows = max(d[0], 1)
print("rows", d[0], "mean candidates %.1f" % (d[1] / rows), "rows over the cap", d[2], "max", buf[3])
print("histogram by 64 candidates:", d[4:16])
