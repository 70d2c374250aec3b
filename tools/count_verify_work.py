"""Counts the data-dependent work terms of the geometric-verification and PnP
bench lines on their own scenes (bench.py verify_line / pnp_line), with the
oracle restatements on the host: mean 5-point models per RANSAC sample, and
CvLevMarq iterations / projection passes per PnP refinement.  bench.py turns
these into algorithmic fp64 flop counts.  Writes
profiles/r3/verify_work.json.  CPU only.

    python tools/count_verify_work.py [n_pairs]
"""
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import geometry as og  # noqa: E402
from oracle import pnp as opnp  # noqa: E402
from oracle import ransac as orc  # noqa: E402

syn = importlib.import_module("3d_reconstruction_amd.synthetic")


def essential(n_pairs):
    s = syn.two_view_pairs(256, 2048, outlier_frac=0.3, noise_px=0.5, seed=6)
    cnt = {"samples": 0, "models": 0, "iters": 0, "inliers": 0, "points": 0}
    five = orc.five_point

    def counting(q1, q2):
        out = five(q1, q2)
        cnt["samples"] += 1
        cnt["models"] += len(out)
        return out
    orc.five_point = counting
    try:
        for p in range(n_pairs):
            E, m, it = orc.find_essential_mat(s["pts0"][p], s["pts1"][p], s["K"], return_iters=True)
            cnt["iters"] += it
            cnt["inliers"] += int(m.sum())
            cnt["points"] += len(s["pts0"][p])
    finally:
        orc.five_point = five
    return {"pairs": n_pairs, "mean_iters": cnt["iters"] / n_pairs,
            "models_per_sample": cnt["models"] / max(1, cnt["samples"]),
            "inlier_frac": cnt["inliers"] / cnt["points"]}


def pnp(n_pairs):
    # the scene of bench.py pnp_line (same generator, same seed)
    rng = np.random.default_rng(12)
    K = np.diag([syn.FOCAL, syn.FOCAL, 1.0])
    P, n = 256, 2000
    probs = []
    for _ in range(P):
        rv = rng.normal(0, 0.2, 3)
        t = np.array([rng.normal(0, 0.3), rng.normal(0, 0.3), 5.0 + rng.random()])
        X = rng.uniform(-1, 1, (n, 3))
        uv = og.project_points(X, rv, t, K) + rng.normal(0, 0.5, (n, 2))
        bad = rng.random(n) < 0.3
        uv[bad] = rng.uniform(-900, 900, (int(bad.sum()), 2))
        probs.append((X, uv))
    cnt = {"lm_calls": 0, "proj": 0, "lm_points": 0, "iters": 0, "jac_proj": 0}
    pj = opnp.project_with_jacobian
    lm = opnp.lm_refine

    def counting_pj(X, param, K_):
        cnt["proj"] += 1
        return pj(X, param, K_)

    def counting_lm(X, m, K_, rvec, tvec, *a, **k):
        cnt["lm_calls"] += 1
        cnt["lm_points"] += len(np.asarray(X).reshape(-1, 3))
        return lm(X, m, K_, rvec, tvec, *a, **k)
    opnp.project_with_jacobian, opnp.lm_refine = counting_pj, counting_lm
    try:
        for p in range(n_pairs):
            r = opnp.solve_pnp_ransac(probs[p][0], probs[p][1], K, return_iters=True)
            cnt["iters"] += r[-1]
    finally:
        opnp.project_with_jacobian, opnp.lm_refine = pj, lm
    return {"problems": n_pairs, "mean_iters": cnt["iters"] / n_pairs,
            "lm_projection_passes_per_problem": cnt["proj"] / max(1, cnt["lm_calls"]),
            "lm_points_per_problem": cnt["lm_points"] / max(1, cnt["lm_calls"])}


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    out = {"essential": essential(n), "pnp": pnp(n),
           "note": "oracle restatements on the bench scenes (tools/count_verify_work.py); the GPU kernels replay "
                   "the same RANSAC samples (tests/test_gpu_verify.py, test_gpu_pnp.py)"}
    path = os.path.join(ROOT, "profiles", "r3", "verify_work.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
