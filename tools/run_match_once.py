"""Launch the C3 all-pairs match a few times (for rocprofv3 --pmc passes): the exact float mode
of the bench headline (int8 MFMA certified filter + f64 re-score); EXACT=0 runs the int8 mode."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
n_img = int(os.environ.get("N_IMG", "257"))
dev = torch.device("cuda", 0)
x = syn.superpoint_like(n_img, 4096, 256, seed=1, device=dev)
bank = sfm.DescriptorBank.from_float(x, mode=sfm.MODE_FLOAT)
del x
pairs = torch.from_numpy(sfm.all_pairs(n_img)).to(dev)
# the bench's graph: int16 written by the kernels (GRAPH=int32: the int32 entry points)
gdt = torch.int32 if os.environ.get("GRAPH", "int16") == "int32" else torch.int16
out = torch.empty((pairs.shape[0], bank.m_pad), dtype=gdt, device=dev)
exact = os.environ.get("EXACT", "1") != "0"
for _ in range(int(os.environ.get("REPS", "2"))):
    bank.match(pairs, ratio=0.75, out=out, exact=exact)
torch.cuda.synchronize()
import hashlib   # noqa: E402
print("matches", int((out >= 0).sum().item()), "sha", hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16])
