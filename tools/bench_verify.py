"""Time the §8f row 2 verification line alone (bench.py's verify_line)."""
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
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--cpu", action="store_true")
a = ap.parse_args()
line = bench.verify_line(sfm, syn, torch.device("cuda", 0), a, lambda: None, cpu=a.cpu)
print(json.dumps(line))
