"""Cost of the exact float matching mode vs the int8 path on C3-shaped descriptors
(and C2 SIFT-128): python tools/bench_match_exact.py [n_pairs]"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
n_pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 4096


def timed(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


x = syn.superpoint_like(257, 4096, 256, seed=1, device=dev)
bank = sfm.DescriptorBank.from_float(x, mode=sfm.MODE_FLOAT, exact=True)
pairs = torch.from_numpy(sfm.all_pairs(257)).to(dev)
sel = pairs[torch.linspace(0, pairs.shape[0] - 1, n_pairs, device=dev).long()].contiguous()
out = torch.empty((n_pairs, bank.m_pad), dtype=torch.int32, device=dev)
t_q = timed(lambda: bank.match(sel, out=out, exact=False))
mq = out.clone()
t_x = timed(lambda: bank.match(sel, out=out, exact=True))
res = int(bank.last_resolved.item()) if bank.last_resolved is not None else -1
diff = float((out != mq).float().mean().item())
print(f"C3 {n_pairs} pairs: int8 {t_q:.2f} ms, exact {t_x:.2f} ms ({t_x / t_q:.2f}x); rows re-scored "
      f"{res} of {n_pairs * 4096} ({res / (n_pairs * 4096):.4%}); exact vs int8 indices differ on {diff:.4%}",
      flush=True)
del bank, x
torch.cuda.empty_cache()
xs = syn.sift_like(64, 2048, 128, seed=0, device=dev)
b2 = sfm.DescriptorBank.from_float(xs, mode=sfm.MODE_SIFT)
p2 = torch.from_numpy(sfm.all_pairs(64)).to(dev)
o2 = torch.empty((p2.shape[0], b2.m_pad), dtype=torch.int32, device=dev)
print(f"C2 2016 pairs (shift {b2.shift}): {timed(lambda: b2.match(p2, out=o2), reps=10):.3f} ms", flush=True)
