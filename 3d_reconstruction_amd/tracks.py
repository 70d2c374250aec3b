"""Match-graph consumer: BFS pair selection + track
building of ``matching.py:84-185``, run on the (all-gathered) BF match graph
instead of per-pair LightGlue calls.

* :class:`MatchGraph` — lookup of a pair's matches (idx0, idx1) in the device
  match graph of all pairs (a < b): forward rows from ``matches0``, reverse
  rows from the mutual ``matches1``.
* :func:`bfs_tracks` — the reference's BFS over the BoW connection graph:
  reference-image choice (matching.py:96-105), raw-match and geometric
  checks (130-144; ``verify`` stands in for cv2's findEssentialMat RANSAC +
  recoverPose, which are not part of this build yet — §8f row 2), the
  interlace test and acceptance (146-160), and the track merge (161-176) in
  host C++ (``sfmhip_track_interlace`` / ``sfmhip_track_merge``).
Output = the ``img_pairs`` / ``all_matches`` formats sfm.py reads
(matching.py:188-189).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._abi import lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _check(name, rc):
    if rc != 0:
        raise RuntimeError(f"{name} failed ({rc}): {lib.sfmhip_last_error().decode(errors='replace')}")


class MatchGraph:
    """Pair -> matches view of an all-pairs match graph.

    ``pairs`` (P,2) with a < b; ``matches0`` (P, m_pad) for rows of a and, for
    reverse lookups, ``matches1`` (P, m_pad) for rows of b (mutual matching)."""

    def __init__(self, pairs, matches0, matches1=None, n_kpts=None):
        self.pairs = np.asarray(pairs, np.int64)
        self.m0 = np.asarray(matches0.cpu() if hasattr(matches0, "cpu") else matches0)
        self.m1 = None if matches1 is None else np.asarray(matches1.cpu() if hasattr(matches1, "cpu") else matches1)
        self.index = {(int(a), int(b)): p for p, (a, b) in enumerate(self.pairs)}
        self.n_kpts = None if n_kpts is None else np.asarray(n_kpts)

    def __call__(self, ref: int, other: int):
        if (ref, other) in self.index:
            row = self.m0[self.index[(ref, other)]]
        elif (other, ref) in self.index:
            if self.m1 is None:
                raise KeyError("reverse lookup needs the mutual matches1 graph")
            row = self.m1[self.index[(other, ref)]]
        else:
            raise KeyError(f"pair ({ref}, {other}) not in the graph")
        if self.n_kpts is not None:
            row = row[: int(self.n_kpts[ref])]
        idx0 = np.nonzero(row >= 0)[0].astype(np.int64)
        return idx0, row[idx0].astype(np.int64)


def bfs_tracks(connection, start: int, n_kpts, match_fn, verify=None, min_raw: int = 8,
               min_inliers: int = 10, min_matches: int = 500, min_interlace: float = 0.3):
    """matching.py:84-185.  Returns (img_pairs (P,2) list, all_matches list of
    [idx0, idx1, track_ids]).  ``verify(ref, id, idx0, idx1)`` returns the
    number of geometric inliers, or None to skip the pair (cv2 returned no
    mask); default: every match is an inlier."""
    n = len(connection)
    tracks = [None] * n
    queue = [(start, start)]
    visited = [False] * n
    visited[start] = True
    all_matches = []
    next_id = np.zeros(1, np.int64)
    cnt = np.zeros(1, np.int64)
    i = 0
    while True:
        cur = queue[i][1]
        for nid in connection[cur]:
            if visited[nid]:
                continue
            ref = cur
            for nb in connection[nid]:
                if nb == cur:
                    break
                if visited[nb]:
                    ref = nb
                    break
            idx0, idx1 = match_fn(ref, nid)
            idx0 = np.ascontiguousarray(idx0, np.int64)
            idx1 = np.ascontiguousarray(idx1, np.int64)
            if len(idx0) <= min_raw:
                continue
            n_inl = len(idx0) if verify is None else verify(ref, nid, idx0, idx1)
            if n_inl is None or n_inl <= min_inliers:
                continue
            for img in (ref, nid):
                if tracks[img] is None:
                    tracks[img] = np.full(int(n_kpts[img]), -1, np.int32)
            tr, ti = tracks[ref], tracks[nid]
            _check("sfmhip_track_interlace",
                   lib.sfmhip_track_interlace(_ptr(tr), len(tr), _ptr(ti), len(ti), _ptr(idx0), _ptr(idx1),
                                              len(idx0), _ptr(cnt)))
            if len(idx0) >= min_matches and (cur == start or cnt[0] / len(idx0) >= min_interlace):
                pid = np.empty(len(idx0), np.int64)
                _check("sfmhip_track_merge",
                       lib.sfmhip_track_merge(_ptr(tr), len(tr), _ptr(ti), len(ti), _ptr(idx0), _ptr(idx1),
                                              len(idx0), _ptr(next_id), _ptr(pid)))
                all_matches.append([idx0, idx1, pid])
                queue.append((ref, nid))
                visited[nid] = True
        i += 1
        if i >= len(queue):
            break
    return queue[1:], all_matches


def save_outputs(out_dir: str, img_pairs, all_matches) -> None:
    """matching.py:188-189 formats: img_pairs.npy (P,2), all_matches.npy object (P,3)."""
    import os
    os.makedirs(out_dir, exist_ok=True)
    np.save(os.path.join(out_dir, "img_pairs.npy"), np.array(img_pairs))
    arr = np.empty((len(all_matches), 3), dtype=object)
    for r, m in enumerate(all_matches):
        arr[r, 0], arr[r, 1], arr[r, 2] = m
    np.save(os.path.join(out_dir, "all_matches.npy"), arr, allow_pickle=True)
