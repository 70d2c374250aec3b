"""The matching stage of the reference (matching.py) on the sfmhip path:
BoW retrieval graph (GPU vq) -> exhaustive all-pairs BF matching (GPU, mutual
+ ratio) -> BFS pair selection + track building on the match graph (host C++)
-> the img_pairs / all_matches that sfm.py reads (matching.py:188-189).
With ``verify="essential"`` (and ``all_points``) the geometric check of
matching.py:130-144 runs on the GPU for every candidate pair in one batch
(verify.EssentialVerifier)."""
from __future__ import annotations

import numpy as np
import torch

from . import bow, tracks, verify as _verify
from .match import MODE_FLOAT, DescriptorBank, all_pairs


def matching_stage(all_descriptors, codebook, ratio=0.75, mode: int = MODE_FLOAT, top_k: int = 10,
                   verify=None, min_matches: int = 500, all_points=None, focal: float = 2378.98305085,
                   exact: bool | None = None):
    """Returns dict(img_pairs, all_matches, connection, start, matches0, matches1).
    ``exact`` (default: True for float descriptors): the matcher's distance semantics
    (match.py module docstring); False selects the quantised int8 mode."""
    descs = [np.asarray(d, np.float32) for d in all_descriptors]
    _, conn, start = bow.retrieval_graph(descs, codebook, top_k=top_k)
    bank = DescriptorBank.from_float(descs, mode=mode, exact=exact)
    pairs = all_pairs(len(descs))
    m0, m1 = bank.match(pairs, ratio=ratio, mutual=True)
    torch.cuda.synchronize()
    n_kpts = [d.shape[0] for d in descs]
    graph = tracks.MatchGraph(pairs, m0, m1, n_kpts)
    if isinstance(verify, str):
        if verify != "essential" or all_points is None:
            raise ValueError('verify must be a callable, None, or "essential" with all_points given')
        K = np.array([[focal, 0, 0], [0, focal, 0], [0, 0, 1.0]])       # matching.py:133
        verify = _verify.EssentialVerifier(conn, graph, all_points, K)
    img_pairs, all_matches = tracks.bfs_tracks(conn, start, n_kpts, graph, verify=verify,
                                               min_matches=min_matches)
    return dict(img_pairs=img_pairs, all_matches=all_matches, connection=conn, start=start,
                matches0=m0, matches1=m1)
