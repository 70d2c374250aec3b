"""A/B of the C3 all-pairs match launch writing the int32 graph vs the int16 graph (the same
kernels, OutT = int32_t / int16_t), interleaved in one process: median HIP-event time of each and
a check that the two graphs hold the same values.  EXACT=0: the int8 mode."""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
dev = torch.device("cuda", 0)
x = syn.superpoint_like(257, 4096, 256, seed=1, device=dev)
bank = sfm.DescriptorBank.from_float(x, mode=sfm.MODE_FLOAT)
del x
pairs = torch.from_numpy(sfm.all_pairs(257)).to(dev)
exact = os.environ.get("EXACT", "1") != "0"
outs = {dt: torch.empty((pairs.shape[0], bank.m_pad), dtype=dt, device=dev) for dt in (torch.int32, torch.int16)}
ts = {dt: [] for dt in outs}
for rnd in range(3):
    for dt, out in outs.items():
        for _ in range(2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            bank.match(pairs, ratio=0.75, out=out, exact=exact)
            e1.record()
            torch.cuda.synchronize()
            ts[dt].append(e0.elapsed_time(e1))
same = torch.equal(outs[torch.int32], outs[torch.int16].to(torch.int32))
for dt in outs:
    print(f"{'exact' if exact else 'int8'} graph {str(dt):12s}: median {np.median(ts[dt]):.2f} ms  "
          f"({', '.join(f'{t:.1f}' for t in ts[dt])})", flush=True)
print("same values:", same, flush=True)
