"""Run selected secondary bench lines alone: python tools/bench_lines.py verify train [--cpu]."""
import argparse
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

sfm = importlib.import_module("3d_reconstruction_amd")
syn = importlib.import_module("3d_reconstruction_amd.synthetic")
ap = argparse.ArgumentParser()
ap.add_argument("lines", nargs="+")
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--warmup", type=int, default=2)
ap.add_argument("--cpu", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda", 0)
for name in a.lines:
    fn = getattr(bench, f"{name}_line", None) or getattr(bench, f"{name}_lines")
    print(json.dumps(fn(sfm, syn, dev, a, lambda: None, cpu=a.cpu)), flush=True)
