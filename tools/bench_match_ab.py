"""C3 (257 x 4096 x 256, float mode, operand shift) and C2 (64 x 2048 x 128, SIFT mode)
all-pairs match launches timed with HIP events (median of 5) and a checksum of each match
graph, for A/B runs of two library builds in separate processes: python tools/bench_match_ab.py"""
import hashlib
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
dev = torch.device("cuda", 0)
for name, n_img, m, d, mode, seed in (("C3", 257, 4096, 256, sfm.MODE_FLOAT, 1), ("C2", 64, 2048, 128, sfm.MODE_SIFT, 0)):
    x = (syn.superpoint_like if mode == sfm.MODE_FLOAT else syn.sift_like)(n_img, m, d, seed=seed, device=dev)
    bank = sfm.DescriptorBank.from_float(x, mode=mode)
    del x
    pairs = sfm.all_pairs(n_img)
    out = bank.match(pairs)
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = bank.match(pairs)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    P = len(pairs)
    ops = 2.0 * m * m * d * P
    h = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"{name}: {np.median(ts):.3f} ms ({ops / (np.median(ts) * 1e-3) / 1e12:.0f} TOPS) graph sha {h}", flush=True)
    del bank, out
    torch.cuda.empty_cache()
