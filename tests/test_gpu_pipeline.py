"""GPU: the whole matching stage (BoW graph -> all-pairs mutual BF on MFMA ->
BFS + tracks) equals the same stage driven by the oracle's matches (the stage's
default exact-float semantics: oracle.match.bf_match_exact, bit for bit)."""
import importlib

import numpy as np
import pytest

from oracle import bow as ob
from oracle import match as om

pytestmark = pytest.mark.gpu
pipe = importlib.import_module("3d_reconstruction_amd.pipeline")
tracks = importlib.import_module("3d_reconstruction_amd.tracks")


def _scene(n_img=8, w=600, stride=150, d=128, seed=5, with_points=False):
    """Global features seen through a sliding window (image i sees features
    [i*stride, i*stride + w), so tracks span 3-4 views); feature descriptors
    cluster by location so the BoW words are informative."""
    rng = np.random.default_rng(seed)
    G = stride * (n_img - 1) + w
    centers = rng.standard_normal((G // 100 + 1, d))
    base = centers[np.arange(G) // 100] + 0.4 * rng.standard_normal((G, d))
    descs, gs = [], []
    for i in range(n_img):
        g = rng.permutation(np.arange(i * stride, i * stride + w))
        x = base[g] + 0.01 * rng.standard_normal((w, d))
        x /= np.linalg.norm(x, axis=1, keepdims=True)
        descs.append(x.astype(np.float32))
        gs.append(g)
    if not with_points:
        return descs
    # geometry for the verification stage: global feature g is a 3D point,
    # image i a camera on an orbit; keypoints in centred pixels (matching.py:133 K)
    syn = importlib.import_module("3d_reconstruction_amd.synthetic")
    X = rng.uniform(-1, 1, (G, 3))
    Rs, ts = syn.orbit_cameras(4 * n_img, seed=seed)
    pts = []
    for i in range(n_img):
        Xc = X[gs[i]] @ Rs[i].T + ts[i]
        pts.append((Xc[:, :2] / Xc[:, 2:] * syn.FOCAL + 0.3 * rng.standard_normal((w, 2))).astype(np.float32))
    return descs, pts


def test_matching_stage_equals_oracle_driven(sfm, gpu):
    descs = _scene()
    book, _ = ob.codebook(descs, 40, 1, seed=1)
    out = pipe.matching_stage(descs, book, min_matches=200)
    assert len(out["img_pairs"]) >= 3
    def oracle_fn(r, i):   # the stage's default: exact-float BF (f32 descriptors, f64 distances)
        m0 = om.bf_match_exact(descs[r], descs[i], (3, 4), mutual=True)
        idx0 = np.nonzero(m0 >= 0)[0]
        return idx0.astype(np.int64), m0[idx0].astype(np.int64)

    ref = ob.retrieval(descs, book)
    assert out["connection"] == [[int(v) for v in c] for c in ref["conn"]] and out["start"] == ref["start"]
    pairs, matches = tracks.bfs_tracks(ref["conn"], ref["start"], [len(x) for x in descs], oracle_fn,
                                       min_matches=200)
    assert [tuple(p) for p in out["img_pairs"]] == [tuple(p) for p in pairs]
    for a, b in zip(out["all_matches"], matches):
        for x, y in zip(a, b):
            assert np.array_equal(x, y)


def test_matching_stage_with_essential_verification(sfm, gpu):
    """matching.py:130-144 on the GPU (speculative batch over all candidate
    pairs) == the BFS driven by oracle matches + the oracle's
    findEssentialMat/recoverPose restatement."""
    from oracle import ransac as orc
    descs, pts = _scene(with_points=True)
    book, _ = ob.codebook(descs, 40, 1, seed=1)
    out = pipe.matching_stage(descs, book, min_matches=200, verify="essential", all_points=pts)
    assert len(out["img_pairs"]) >= 3
    f = importlib.import_module("3d_reconstruction_amd.synthetic").FOCAL
    K = np.array([[f, 0, 0], [0, f, 0], [0, 0, 1.0]])

    def oracle_fn(r, i):
        m0 = om.bf_match_exact(descs[r], descs[i], (3, 4), mutual=True)
        idx0 = np.nonzero(m0 >= 0)[0]
        return idx0.astype(np.int64), m0[idx0].astype(np.int64)

    def oracle_verify(r, i, idx0, idx1):
        a, b = pts[r][idx0].astype(np.float32), pts[i][idx1].astype(np.float32)
        E, m = orc.find_essential_mat(a, b, K)
        if E is None:
            return None
        keep = m.ravel() > 0
        return orc.recover_pose(E, a[keep], b[keep], K)[0]

    ref = ob.retrieval(descs, book)
    pairs, matches = tracks.bfs_tracks(ref["conn"], ref["start"], [len(x) for x in descs], oracle_fn,
                                       verify=oracle_verify, min_matches=200)
    assert [tuple(p) for p in out["img_pairs"]] == [tuple(p) for p in pairs]
    for a, b in zip(out["all_matches"], matches):
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
