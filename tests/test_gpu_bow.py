"""GPU parity: BoW retrieval front end vs the reference
goldens (bow.py:14-23 and matching.py:24-82 executed from the reference files)."""
import importlib

import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
bow = importlib.import_module("3d_reconstruction_amd.bow")


def test_kmeans_matches_scipy_reference(sfm, gpu):
    g = golden("bow_golden.npz")
    from oracle.bow import stack_descriptors
    book, dist = bow.kmeans(stack_descriptors(list(g["desc"])), 200, 1, rng=np.random.RandomState(123))
    assert book.shape == g["codebook"].shape
    np.testing.assert_allclose(book, g["codebook"], rtol=1e-12, atol=1e-12)
    assert abs(dist - float(g["variance"])) < 1e-12


def test_kmeans_update_bitexact_given_codes(sfm, gpu):
    """The centroid update alone is scipy's summation order -> identical bits."""
    from scipy.cluster.vq import _vq
    rng = np.random.default_rng(3)
    obs = rng.standard_normal((5000, 96))
    codes = rng.integers(0, 37, 5000).astype(np.int32)
    codes[codes == 5] = 6            # an empty cluster
    ref, has = _vq.update_cluster_means(obs, codes, 37)
    o = torch.from_numpy(obs).to(gpu)
    c = torch.from_numpy(codes).to(gpu)
    book = torch.zeros((37, 96), dtype=torch.float64, device=gpu)
    cnt = torch.empty(37, dtype=torch.int32, device=gpu)
    sfm.lib.sfmhip_kmeans_update(o.data_ptr(), 5000, 96, c.data_ptr(), 37, book.data_ptr(), cnt.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(cnt.cpu().numpy() > 0, has)
    assert np.array_equal(book.cpu().numpy()[has], ref[has])


def test_retrieval_graph_matches_reference(sfm, gpu):
    g = golden("bow_golden.npz")
    words, conn, start = bow.retrieval_graph(list(g["desc"]), g["codebook"])
    assert np.array_equal(np.stack(words), g["words"])
    assert [j for c in conn for j in c] == g["conn_flat"].tolist()
    assert [len(c) for c in conn] == g["conn_len"].tolist()
    assert start == int(g["start"])


def test_histogram_exact(sfm, gpu):
    g = golden("bow_golden.npz")
    codes = torch.from_numpy(g["words"].astype(np.int32).ravel()).to(gpu)
    offsets = np.arange(0, g["words"].size + 1, g["words"].shape[1])
    freq = bow.frequency_vectors(codes, offsets, 200)
    assert np.array_equal(freq, g["freq"])
