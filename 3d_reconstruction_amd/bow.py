"""BoW image retrieval: the codebook of ``bow.py`` and the
pair-candidate graph of ``matching.py:24-82``.

GPU: word assignment of every descriptor of every image in ONE ``sfmhip_vq``
launch, per-image histograms (``sfmhip_word_histogram``) and the k-means
iterations of ``scipy.cluster.vq.kmeans`` (``sfmhip_vq`` +
``sfmhip_kmeans_update``, scipy's summation order -> identical centroids).
Host: the N x k tf-idf / cosine / top-k / graph bookkeeping (a few hundred
numbers per image) with the reference's numpy operations.
"""
from __future__ import annotations

from collections import deque

import numpy as np
import torch

from ._abi import call, dev, ptr, require_gpu, stream_ptr


def _vq_dev(o: torch.Tensor, book: torch.Tensor):
    n = o.shape[0]
    codes = torch.empty(n, dtype=torch.int32, device=o.device)
    dist = torch.empty(n, dtype=torch.float64, device=o.device)
    call("sfmhip_vq", ptr(o), n, ptr(book), book.shape[0], book.shape[1], ptr(codes), ptr(dist), stream_ptr())
    return codes, dist


def _kpoints(data_n: int, k: int, rng):
    """scipy.cluster.vq._kpoints: k distinct observation indices from ``rng``."""
    return rng.choice(data_n, size=int(k), replace=False)


def kmeans(obs, k_or_guess, iter: int = 20, thresh: float = 1e-5, check_finite: bool = True, *, rng=None):
    """``scipy.cluster.vq.kmeans`` (what bow.py:23 calls) with the vq and the
    centroid update on the GPU.  Returns (codebook, distortion)."""
    from scipy._lib._util import check_random_state
    require_gpu()
    o_np = np.asarray(obs, dtype=np.float64)
    if check_finite and not np.isfinite(o_np).all():
        raise ValueError("array must not contain infs or NaNs")
    if o_np.ndim == 1:
        o_np = o_np[:, None]
    o = dev(o_np, torch.float64)
    guess = np.asarray(k_or_guess)
    if iter < 1:
        raise ValueError(f"iter must be at least 1, got {iter}")
    if guess.size != 1:
        return _kmeans(o, dev(guess.reshape(-1, o.shape[1]), torch.float64), thresh)
    k = int(guess)
    if k != guess or k < 1:
        raise ValueError(f"Asked for {k_or_guess} clusters.")
    r = check_random_state(rng)
    best_book, best_dist = None, np.inf
    for _ in range(iter):
        idx = _kpoints(o.shape[0], k, r)
        book, d = _kmeans(o, o[torch.from_numpy(np.asarray(idx)).to(o.device)].contiguous(), thresh)
        if d < best_dist:
            best_book, best_dist = book, d
    return best_book, best_dist


def _kmeans(o: torch.Tensor, book: torch.Tensor, thresh: float):
    """scipy.cluster.vq._kmeans loop: assign, re-centre, drop empty clusters,
    stop when the mean distortion changes by <= thresh."""
    diff = np.inf
    prev = deque([diff], maxlen=2)
    n, d = o.shape
    while diff > thresh:
        codes, dist = _vq_dev(o, book)
        prev.append(np.mean(dist.cpu().numpy(), axis=-1))
        k = book.shape[0]
        new = torch.zeros((k, d), dtype=torch.float64, device=o.device)
        counts = torch.empty(k, dtype=torch.int32, device=o.device)
        call("sfmhip_kmeans_update", ptr(o), n, d, ptr(codes), k, ptr(new), ptr(counts), stream_ptr())
        book = new[counts > 0].contiguous()
        diff = abs(prev[0] - prev[1])
    return book.cpu().numpy(), prev[1]


def visual_words(all_descriptors, codebook):
    """matching.py:26-28: vq of every image's descriptors (one launch for all)."""
    rows = [np.asarray(x, dtype=np.float64) for x in all_descriptors]
    sizes = np.array([r.shape[0] for r in rows], dtype=np.int64)
    o = dev(np.concatenate(rows, 0), torch.float64)
    book = dev(np.asarray(codebook, np.float64), torch.float64)
    codes, _ = _vq_dev(o, book)
    offsets = np.concatenate([[0], np.cumsum(sizes)])
    c = codes.cpu().numpy()
    return [c[offsets[i]:offsets[i + 1]] for i in range(len(rows))], codes, offsets


def frequency_vectors(codes: torch.Tensor, offsets: np.ndarray, k: int) -> np.ndarray:
    """matching.py:30-37: (N, k) float64 word counts, from the device codes."""
    n_img = len(offsets) - 1
    off = dev(np.asarray(offsets, np.int64), torch.int64)
    hist = torch.empty((n_img, k), dtype=torch.int32, device=codes.device)
    call("sfmhip_word_histogram", ptr(codes), ptr(off), n_img, int(k), ptr(hist), stream_ptr())
    return hist.cpu().numpy().astype(np.float64)


def tfidf(freq: np.ndarray) -> np.ndarray:
    """matching.py:41-47: tf-idf weighting of the word counts."""
    n = freq.shape[0]
    idf = np.log(n / np.sum(freq > 0, axis=0))
    return freq * idf


def retrieval_topk(tf: np.ndarray, top_k: int = 10):
    """matching.py:49-59: per image, the top_k-1 most cosine-similar other images
    (index list and negated scores, in the reference's argsort order)."""
    norms = np.linalg.norm(tf, axis=1)
    idxs, scores = [], []
    for i in range(tf.shape[0]):
        sim = np.dot(tf[i], tf.T) / (np.linalg.norm(tf[i]) * norms)
        idxs.append(np.argsort(-sim)[1:top_k])
        scores.append(np.sort(-sim)[1:top_k])
    return idxs, scores


def connection_graph(idxs, scores, thresh: float = 0.75):
    """matching.py:61-73: undirected adjacency lists, edge iff cosine > thresh,
    neighbours in first-seen order."""
    n = len(idxs)
    conn = [None] * n
    for i in range(n):
        for j, nb in enumerate(idxs[i]):
            conn[i] = conn[i] if conn[i] else []
            conn[nb] = conn[nb] if conn[nb] else []
            if -scores[i][j] > thresh:
                if nb not in conn[i]:
                    conn[i].append(nb)
                if i not in conn[nb]:
                    conn[nb].append(i)
    return conn


def start_node(conn) -> int:
    """matching.py:77-82: the first image with the most connections."""
    best, start = 0, 0
    for i, c in enumerate(conn):
        if len(c) > best:
            best, start = len(c), i
    return start


def retrieval_graph(all_descriptors, codebook, k: int | None = None, top_k: int = 10, thresh: float = 0.75):
    """The whole matching.py:24-82 front end: (visual_words, connection, start)."""
    k = int(np.asarray(codebook).shape[0]) if k is None else int(k)
    words, codes, offsets = visual_words(all_descriptors, codebook)
    freq = frequency_vectors(codes, offsets, k)
    idxs, scores = retrieval_topk(tfidf(freq), top_k)
    conn = connection_graph(idxs, scores, thresh)
    return words, conn, start_node(conn)
