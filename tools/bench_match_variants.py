"""A/B the match kernel variants (SFMHIP_MATCH_VARIANT) on the C3 workload in
one process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24), and
check every variant's output is identical to variant 0 (the tested default)."""
import importlib
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")

variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3").split(",")]
n_img = int(os.environ.get("N_IMG", "257"))
d = int(os.environ.get("DIM", "256"))
m = int(os.environ.get("MKPT", "4096"))
dev = torch.device("cuda", 0)
sift = os.environ.get("DATA", "float") == "sift"   # DATA=sift: bench.py's C2 operands (MODE_SIFT)
x = (syn.sift_like if sift else syn.superpoint_like)(n_img, m, d, seed=0 if sift else 1, device=dev)
bank = sfm.DescriptorBank.from_float(x, mode=sfm.MODE_SIFT if sift else sfm.MODE_FLOAT)
del x
pairs = torch.from_numpy(sfm.all_pairs(n_img)).to(dev)
P = pairs.shape[0]
outs = {v: torch.empty((P, bank.m_pad), dtype=torch.int32, device=dev) for v in variants}
times = {v: [] for v in variants}
for rnd in range(4):
    for v in variants:
        os.environ["SFMHIP_MATCH_VARIANT"] = str(v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        bank._launch(pairs, 3, 4, outs[v], None, None)
        e1.record()
        torch.cuda.synchronize()
        if rnd > 0:
            times[v].append(e0.elapsed_time(e1))
ref = outs[0] if 0 in outs else outs[variants[0]]
ops = 2.0 * m * m * d * P
for v in variants:
    ms = float(np.median(times[v]))
    same = bool(torch.equal(outs[v], ref))
    print(f"variant {v}: {ms:8.2f} ms  {ops / ms / 1e9:7.0f} TOPS  ({ops / ms / 1e9 / 5000:.1%} of int8 peak)  identical={same}",
          flush=True)
