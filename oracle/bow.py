"""Oracle for the BoW retrieval front end.  TEST
INFRASTRUCTURE ONLY.

bow.py:14-23   stack all descriptors (last image first), scipy kmeans(k=200, iter=1)
matching.py:24-82  vq per image -> word histograms -> tf-idf -> per-image cosine
               top-k (argsort of the negated similarity, entries 1..top_k-1) ->
               undirected graph (cosine > 0.75) -> start = first max-degree image.
The numeric kernels ARE scipy's (vq, kmeans); the bookkeeping is restated.
"""
from __future__ import annotations

import numpy as np
from scipy.cluster.vq import kmeans as _kmeans
from scipy.cluster.vq import vq as _vq


def stack_descriptors(all_descriptors):
    """bow.py:14-18 order: image 0 last, image N-1 first."""
    return np.vstack([np.asarray(d, np.float64) for d in all_descriptors[::-1]])


def codebook(all_descriptors, k=200, iters=1, seed=None):
    if seed is not None:
        np.random.seed(seed)
    return _kmeans(stack_descriptors(all_descriptors), k, iters)


def retrieval(all_descriptors, book, top_k=10, thresh=0.75):
    words = [_vq(np.asarray(d, np.float64), book)[0] for d in all_descriptors]
    k = len(book)
    freq = np.zeros((len(words), k))
    for i, w in enumerate(words):
        np.add.at(freq[i], w, 1.0)
    n = freq.shape[0]
    tf = freq * np.log(n / (freq > 0).sum(0))
    idx, score = [], []
    for i in range(n):
        cs = np.dot(tf[i], tf.T) / (np.linalg.norm(tf[i]) * np.linalg.norm(tf, axis=1))
        idx.append(np.argsort(-cs)[1:top_k])
        score.append(np.sort(-cs)[1:top_k])
    conn = [[] for _ in range(n)]
    for i in range(n):
        for j, nb in enumerate(idx[i]):
            if -score[i][j] > thresh:
                if nb not in conn[i]:
                    conn[i].append(nb)
                if i not in conn[nb]:
                    conn[nb].append(i)
    degrees = [len(c) for c in conn]
    start = int(np.argmax(degrees)) if max(degrees) > 0 else 0
    return dict(words=words, freq=freq, tfidf=tf, idx=idx, score=score, conn=conn, start=start)
