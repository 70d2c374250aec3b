"""BA solve on the first P pairs of bench.py's scene (P from argv), printing the time and an output
checksum per size (a quick way to compare two builds run in separate processes)."""
import hashlib
import importlib
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
dev = torch.device("cuda", 0)
s = syn.ba_scene(256, 4096, seed=4)
sel = os.environ.get("PAIRS")
if sel:   # only these pairs (comma-separated), in that order
    idx = [int(x) for x in sel.split(",")]
    obs = np.concatenate([np.arange(p * 4096, (p + 1) * 4096) for p in idx])
    s = {"cam": s["cam"][idx], "K": s["K"][idx], "X": s["X"][obs], "pts2d": s["pts2d"][obs]}
for P in [int(a) for a in sys.argv[1:]]:
    n = P * 4096
    tt = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in s.items() if k in ("cam", "K", "X", "pts2d")}
    cam, X = tt["cam"][:P].clone(), tt["X"][:n].clone()
    off = torch.arange(P + 1, dtype=torch.int64, device=dev) * 4096
    torch.cuda.synchronize()
    t0 = time.time()
    mx = int(os.environ.get("MAXNFEV", "0")) or None
    r = sfm.ba_solve_batched(cam, tt["K"][:P].contiguous(), X, tt["pts2d"][:n].contiguous(), off, validate=False,
                             max_nfev=mx)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for t in (cam, X, r["nfev"], r["njev"], r["cost"]):
        h.update(t.cpu().numpy().tobytes())
    print(P, "pairs: %.1f ms" % ((time.time() - t0) * 1e3), "nfev", r["nfev"].float().mean().item(),
          "njev", r["njev"].float().mean().item(), "sha", h.hexdigest()[:16], flush=True)
    nf, nj, st, co = (r[k].cpu().numpy() for k in ("nfev", "njev", "status", "cost"))
    for i in np.nonzero(nf != nj)[0][:8]:
        print("   pair", i, "nfev", nf[i], "njev", nj[i], "status", st[i], "cost", co[i], flush=True)
