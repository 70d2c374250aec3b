"""A/B the M2 vq kernels: python tools/bench_vq.py  (SFMHIP_VQ_VARIANT: 0 f32 filter + exact decision,
register-resident observations (default), 4 the same filter tile-staged, 6 f16-split matrix-core filter, 3 f64 MFMA one block/step, 2 f64 MFMA two blocks/step, 1 FMA difference form)."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
abi = importlib.import_module("3d_reconstruction_amd._abi")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
dev = torch.device("cuda", 0)
obs = syn.superpoint_like(257, 4096, 128, seed=3, device=dev).reshape(-1, 128).double().contiguous()
book = obs[torch.randperm(obs.shape[0], device=dev)[:200]].contiguous()
out = {}
for variant in (sys.argv[1].split(",") if len(sys.argv) > 1 else ("0", "4", "3", "2", "1")):
    os.environ["SFMHIP_VQ_VARIANT"], _, probe = variant.partition(":")   # "6:1": variant 6 under timing probe 1
    os.environ["SFMHIP_VQ_PROBE"] = probe or "0"
    codes = torch.empty(obs.shape[0], dtype=torch.int32, device=dev)
    dist = torch.empty(obs.shape[0], dtype=torch.float64, device=dev)

    def run():
        abi.call("sfmhip_vq", obs.data_ptr(), obs.shape[0], book.data_ptr(), 200, 128, codes.data_ptr(),
                 dist.data_ptr(), abi.stream_ptr())
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    out[variant] = (codes.clone(), dist.clone())
    print(f"variant {variant}: {ms:.3f} ms  {obs.shape[0] / ms / 1e3:.1f} Mobs/s  "
          f"{2 * obs.shape[0] * 200 * 128 / ms / 1e9:.2f} TFLOP/s (2nkd)", flush=True)
ref = next(iter(out))
c0, d0 = out[ref]
for v in [v for v in out if v != ref]:
    c1, d1 = out[v]
    print(f"{ref} vs {v}: codes agree", (c0 == c1).float().mean().item(), "max rel dist",
          ((d0 - d1).abs() / d1.clamp_min(1e-300)).max().item())
