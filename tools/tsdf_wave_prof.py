"""Per-wave timeline of the TSDF fusion kernel (tool-only build with -DSFMHIP_TSDF_PROF):
start / end wall clock and projected-frame count of every fusion wave, for the whole C5
grid and for N = 8 slabs 2 (heavy) and 6 (light).  Shows whether a call is bound by
throughput (waves end evenly) or by its longest waves' frame loops.
  hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -DSFMHIP_TSDF_PROF -shared \\
        -c voxel.hip -o voxel_prof.o, linked with the other objects of the Makefile into ab/libtsdf_prof.so
python tools/tsdf_wave_prof.py   (SFMHIP_TSDF_PROF_LDS=bytes: dynamic LDS per slab fusion workgroup,
                                  capping the resident waves, to tell latency- from issue-bound waves)"""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sfm = importlib.import_module("3d_reconstruction_amd")
abi = importlib.import_module("3d_reconstruction_amd._abi")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
sdist = importlib.import_module("3d_reconstruction_amd.dist")
abi.LIB_PATH = os.path.join(ROOT, "ab", "libtsdf_prof.so")
abi.lib = abi._load()
abi.lib.sfmhip_tsdf_prof_read.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
NW = 1 << 18
dev = torch.device("cuda", 0)
depth, poses, K = syn.tsdf_scene(257, syn.IMG_H, syn.IMG_W, device=dev)
R = 256
T = torch.zeros((R, R, R), dtype=torch.float32, device=dev)
W = torch.zeros_like(T)
args = (depth, poses, K, (-1.2,) * 3, (1.2,) * 3, 3 * 2.4 / (R - 1))
tab = sfm.tsdf_block_table(depth)
buf = np.zeros(3 * NW, np.uint64)


def run(label, fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    assert abi.lib.sfmhip_tsdf_prof_read(buf.ctypes.data, NW, 1) == 0   # clear
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    assert abi.lib.sfmhip_tsdf_prof_read(buf.ctypes.data, NW, 0) == 0
    b = buf.reshape(NW, 3).astype(np.float64)
    m = b[:, 0] > 0
    t0, t1, npj = b[m, 0], b[m, 1], b[m, 2]
    base = t0.min()
    st, en, du = (t0 - base) * 0.01, (t1 - base) * 0.01, (t1 - t0) * 0.01   # us
    span = en.max()
    late = np.argsort(-en)[:8]
    print(f"{label}: call {e0.elapsed_time(e1) * 1e3:.0f} us, fusion span {span:.0f} us, waves {m.sum()}, "
          f"duration p50 {np.median(du):.1f} p90 {np.percentile(du, 90):.1f} p99 {np.percentile(du, 99):.1f} "
          f"max {du.max():.1f} us; nproj p50 {np.median(npj):.0f} max {npj.max():.0f}", flush=True)
    print(f"   last-ending waves (start, duration, nproj): "
          + ", ".join(f"({st[i]:.0f}, {du[i]:.0f}, {npj[i]:.0f})" for i in late), flush=True)
    for lo, hi in ((0, 16), (16, 64), (64, 128), (128, 1000)):
        sel = (npj >= lo) & (npj < hi)
        if sel.any():
            print(f"   nproj [{lo},{hi}): {sel.sum()} waves, mean duration {du[sel].mean():.1f} us, "
                  f"max {du[sel].max():.1f}, us per projected frame {np.mean(du[sel] / np.maximum(npj[sel], 1)):.2f}",
                  flush=True)
    fin = np.sort(en)
    print(f"   waves still running at 50/75/90 % of the span: "
          + " / ".join(str(int(((st <= f * span) & (en > f * span)).sum())) for f in (0.5, 0.75, 0.9)), flush=True)


if os.environ.get("SFMHIP_TSDF_PROF_LDS", "0") == "0":
    run("whole grid", lambda: sfm.tsdf_integrate(T, W, *args))
for r in (2, 6):
    z0, z1 = sdist.shard_range(R, r, 8)
    run(f"N=8 slab {r} [{z0},{z1})", lambda: sfm.tsdf_integrate(T, W, *args, z0, z1, block_table=tab))
