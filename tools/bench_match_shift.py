"""A/B the matcher's operand shift (SFMHIP_MATCH_SHIFT) on the C3 workload in one
process, interleaved rounds; both banks must give identical matches."""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")

n_img = int(os.environ.get("N_IMG", "257"))
d, m = 256, 4096
dev = torch.device("cuda", 0)
x = syn.superpoint_like(n_img, m, d, seed=1, device=dev)
banks = {}
for sh in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "1"]):
    os.environ["SFMHIP_MATCH_SHIFT"] = sh
    banks[sh] = sfm.DescriptorBank.from_float(x, mode=sfm.MODE_FLOAT)
del x
pairs = torch.from_numpy(sfm.all_pairs(n_img)).to(dev)
P = pairs.shape[0]
outs = {k: torch.empty((P, banks[k].m_pad), dtype=torch.int32, device=dev) for k in banks}
times = {k: [] for k in banks}
for rnd in range(4):
    for k, bank in banks.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        bank._launch(pairs, 3, 4, outs[k], None, None)
        e1.record()
        torch.cuda.synchronize()
        if rnd > 0:
            times[k].append(e0.elapsed_time(e1))
ops = 2.0 * m * m * d * P
for k in banks:
    ms = float(np.median(times[k]))
    print(f"shift={k}: {ms:8.2f} ms  {ops / ms / 1e9:7.0f} TOPS  ({ops / ms / 1e9 / 5000:.1%} of int8 peak)  "
          f"identical={bool(torch.equal(outs[k], outs['0']))}", flush=True)
