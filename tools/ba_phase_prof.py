"""Phase breakdown of the BA solve kernel on C3's 256 pairs x 4096 obs (SFMHIP_BA_VARIANT as given).
Needs the tool-only build (the phase timers are compiled out of the product library):
  hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -DSFMHIP_BA_PROF -shared \
        3d_reconstruction_amd/csrc/{lib,ba}.hip -o ab/libba_prof.so
python tools/ba_phase_prof.py [variant: 0..3]"""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SFMHIP_BA_VARIANT", sys.argv[1] if len(sys.argv) > 1 else "1")
lib = ctypes.CDLL(os.path.join(root, "ab", "libba_prof.so"))
P = ctypes.c_void_p
lib.sfmhip_ba_solve.argtypes = [P, P, P, P, P, ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                ctypes.c_double, ctypes.c_int32, P, P, P, P, P]
lib.sfmhip_ba_prof_read.argtypes = [P, ctypes.c_int]
dev = torch.device("cuda", 0)
s = syn.ba_scene(256, 4096, seed=4)
tt = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in s.items()}
off = torch.arange(257, dtype=torch.int64, device=dev) * 4096
n = int(off[-1])
cost = torch.empty(256, dtype=torch.float64, device=dev)
nfev, njev, st = (torch.empty(256, dtype=torch.int32, device=dev) for _ in range(3))
names = ["jacobian (+X move)", "regularize", "ridge + chol", "gn pass", "subspace pass", "tr solve", "trial pass",
         "trial serial", "-", "-"]
for rep in range(3):
    cam, X = tt["cam"].clone(), tt["X"].clone()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    rc = lib.sfmhip_ba_solve(cam.data_ptr(), tt["K"].data_ptr(), X.data_ptr(), tt["pts2d"].data_ptr(), off.data_ptr(),
                             256, n, 1e-8, 1e-8, 1e-8, 0, cost.data_ptr(), nfev.data_ptr(), njev.data_ptr(),
                             st.data_ptr(), torch.cuda.current_stream().cuda_stream)
    e1.record()
    torch.cuda.synchronize()
    assert rc == 0
ms = e0.elapsed_time(e1)
buf = np.zeros(256 * 10, np.uint64)
assert lib.sfmhip_ba_prof_read(buf.ctypes.data, 256) == 0
t = buf.reshape(256, 10).astype(np.float64) * 10e-3   # 100 MHz ticks -> us
print(f"variant {os.environ['SFMHIP_BA_VARIANT']}: kernel {ms:.3f} ms; nfev mean {nfev.float().mean().item():.2f} "
      f"njev mean {njev.float().mean().item():.2f}; per-pair phase sums (us): mean / max over pairs")
tot = t.sum(1)
for k, nm in enumerate(names[:8]):
    print(f"  {nm:13s} {t[:, k].mean():8.1f} {t[:, k].max():8.1f}")
print(f"  {'total':13s} {tot.mean():8.1f} {tot.max():8.1f}")
