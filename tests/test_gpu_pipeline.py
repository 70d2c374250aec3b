"""GPU: the whole matching stage (BoW graph -> all-pairs mutual BF on MFMA ->
BFS + tracks) equals the same stage driven by the oracle's matches."""
import importlib

import numpy as np
import pytest

from oracle import bow as ob
from oracle import match as om

pytestmark = pytest.mark.gpu
pipe = importlib.import_module("3d_reconstruction_amd.pipeline")
tracks = importlib.import_module("3d_reconstruction_amd.tracks")


def _scene(n_img=8, w=600, stride=150, d=128, seed=5):
    """Global features seen through a sliding window (image i sees features
    [i*stride, i*stride + w), so tracks span 3-4 views); feature descriptors
    cluster by location so the BoW words are informative."""
    rng = np.random.default_rng(seed)
    G = stride * (n_img - 1) + w
    centers = rng.standard_normal((G // 100 + 1, d))
    base = centers[np.arange(G) // 100] + 0.4 * rng.standard_normal((G, d))
    descs = []
    for i in range(n_img):
        g = rng.permutation(np.arange(i * stride, i * stride + w))
        x = base[g] + 0.01 * rng.standard_normal((w, d))
        x /= np.linalg.norm(x, axis=1, keepdims=True)
        descs.append(x.astype(np.float32))
    return descs


def test_matching_stage_equals_oracle_driven(sfm, gpu):
    descs = _scene()
    book, _ = ob.codebook(descs, 40, 1, seed=1)
    out = pipe.matching_stage(descs, book, min_matches=200)
    assert len(out["img_pairs"]) >= 3
    q = [om.quantize(x, 1) for x in descs]

    def oracle_fn(r, i):
        m0 = om.bf_match_q(q[r], q[i], (3, 4), mutual=True)
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
