"""Interleaved A/B of the TSDF step forms on the C5 call (257 frames into a 256^3 grid), one
process: SFMHIP_AB=1 the serial step, 2 pipelined culling + one fusion launch, 0 the default
(pipelined culling + the two-part fusion).  Every form's (T, W) must be the same bits; prints the
median ms of each form over ROUNDS interleaved rounds of 5 timed calls."""
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
depth, poses, K = syn.tsdf_scene(257, syn.IMG_H, syn.IMG_W, device=dev)
R = 256
T = torch.zeros((R, R, R), dtype=torch.float32, device=dev)
W = torch.zeros_like(T)
FORMS = os.environ.get("FORMS", "1,2,0").split(",")
ROUNDS = int(os.environ.get("ROUNDS", "4"))
times = {f: [] for f in FORMS}
digest = {}
for rnd in range(ROUNDS):
    for f in FORMS:
        os.environ["SFMHIP_AB"] = f
        sfm.knobs_reload()
        for i in range(7):
            T.zero_()
            W.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            sfm.tsdf_integrate(T, W, depth, poses, K, (-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / (R - 1))
            e1.record()
            torch.cuda.synchronize()
            if i >= 2:
                times[f].append(e0.elapsed_time(e1))
        h = hashlib.sha256(T.cpu().numpy().tobytes() + W.cpu().numpy().tobytes()).hexdigest()[:16]
        digest.setdefault(f, h)
        assert digest[f] == h, f"form {f} not deterministic"
os.environ["SFMHIP_AB"] = "0"
sfm.knobs_reload()
same = len(set(digest.values())) == 1
for f in FORMS:
    t = np.array(times[f])
    print(f"SFMHIP_AB={f}: median {np.median(t):.3f} ms  min {t.min():.3f}  max {t.max():.3f}  sha {digest[f]}",
          flush=True)
print(f"identical grids across forms: {same}", flush=True)
assert same
