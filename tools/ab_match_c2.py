"""C2 all-pairs match (64 x 2048 x 128 SIFT, MODE_SIFT) timed with HIP events, interleaved over
SFMHIP_AB values in one process, with a checksum of each match graph:
python tools/ab_match_c2.py [ab values, default 0]"""
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
x = syn.sift_like(64, 2048, 128, seed=0, device=dev)
bank = sfm.DescriptorBank.from_float(x, mode=sfm.MODE_SIFT)
del x
pairs = torch.from_numpy(sfm.all_pairs(64)).to(dev)
abs_ = [int(a) for a in sys.argv[1:]] or [0]
ts = {a: [] for a in abs_}
sha = {}
for rnd in range(3):
    for a in abs_:
        os.environ["SFMHIP_AB"] = str(a)
        sfm.knobs_reload()
        out = bank.match(pairs)
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = bank.match(pairs)
            e1.record()
            torch.cuda.synchronize()
            ts[a].append(e0.elapsed_time(e1))
        sha[a] = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
ops = 2.0 * 2048 * 2048 * 128 * pairs.shape[0]
for a in abs_:
    t = np.median(ts[a])
    print(f"ab {a}: C2 {t:.3f} ms ({ops / (t * 1e-3) / 1e12:.0f} TOPS, frac {ops / (t * 1e-3) / 5e15:.3f}) "
          f"sha {sha[a]}", flush=True)
