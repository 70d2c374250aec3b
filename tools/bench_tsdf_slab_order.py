"""A/B of the fusion's workgroup order on one z-slab of an N-way split (env knobs
read per call): python tools/bench_tsdf_slab_order.py N r"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
sdist = importlib.import_module("3d_reconstruction_amd.dist")
n, r = int(sys.argv[1]), int(sys.argv[2])
dev = torch.device("cuda", 0)
depth, poses, K = syn.tsdf_scene(257, syn.IMG_H, syn.IMG_W, device=dev)
R = 256
T = torch.zeros((R, R, R), dtype=torch.float32, device=dev)
W = torch.zeros_like(T)
tab = sfm.tsdf_block_table(depth)
z0, z1 = sdist.shard_range(R, r, n)
args = (depth, poses, K, (-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / (R - 1))


def timed(reps=7):
    ts = []
    for _ in range(reps):
        T[z0:z1].zero_()
        W[z0:z1].zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        sfm.tsdf_integrate(T, W, *args, z0, z1, block_table=tab) if tab is not None else \
            sfm.tsdf_integrate(T, W, *args, z0, z1)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


ref = None
VARIANTS = [("default", {}), ("LATENCY=0", {"SFMHIP_TSDF_LATENCY": "0"}), ("LATENCY=1", {"SFMHIP_TSDF_LATENCY": "1"}),
            ("default", {}), ("LATENCY=0", {"SFMHIP_TSDF_LATENCY": "0"}), ("LATENCY=1", {"SFMHIP_TSDF_LATENCY": "1"})]
if os.environ.get("NO_TABLE"):   # the single-GPU call: the block pass inside tsdf_integrate
    tab = None
for name, env in VARIANTS:
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    sfm.knobs_reload()   # knobs are read once per process: re-read after every change
    t = timed()
    out = (T[z0:z1].clone(), W[z0:z1].clone())
    same = ref is None or (torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1]))
    ref = ref or out
    print(f"N={n} slab {r} [{z0},{z1}) {name:10s}: {t:.3f} ms  identical={same}", flush=True)
    for k, v in old.items():
        if v is None:
            os.environ.pop(k)
        else:
            os.environ[k] = v
    sfm.knobs_reload()
