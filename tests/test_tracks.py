"""CPU: the match-graph consumer (BFS pair selection + track merge, SURVEY.md
§8f row 1) against matching.py:84-185 executed from the reference file on the
same match table (tests/golden/make_golden.py:gen_bfs).  Host C++ + Python;
no GPU needed."""
import importlib

import numpy as np

from conftest import golden

tracks = importlib.import_module("3d_reconstruction_amd.tracks")


def _unpack(g):
    conn, o = [], 0
    for L in g["conn_len"]:
        conn.append([int(v) for v in g["conn_flat"][o:o + L]])
        o += L
    table, o = {}, 0
    for (a, b), L in zip(g["tab_keys"], g["tab_len"]):
        table[(int(a), int(b))] = (g["tab_i0"][o:o + L], g["tab_i1"][o:o + L])
        o += L
    return conn, table


def test_bfs_tracks_match_reference():
    g = golden("bfs_golden.npz")
    conn, table = _unpack(g)
    k = int(g["k"])
    pairs, matches = tracks.bfs_tracks(conn, int(g["start"]), [k] * len(conn), lambda r, i: table[(r, i)])
    assert [list(p) for p in pairs] == g["img_pairs"].tolist()
    assert [len(m[0]) for m in matches] == g["m_len"].tolist()
    assert np.array_equal(np.concatenate([m[0] for m in matches]), g["m_idx0"])
    assert np.array_equal(np.concatenate([m[1] for m in matches]), g["m_idx1"])
    assert np.array_equal(np.concatenate([m[2] for m in matches]), g["m_tracks"])


def test_match_graph_lookup_both_directions():
    pairs = np.array([[0, 1], [0, 2], [1, 2]])
    m0 = np.full((3, 8), -1, np.int32)
    m1 = np.full((3, 8), -1, np.int32)
    m0[0, [1, 4]] = [3, 5]
    m1[0, [3, 5]] = [1, 4]
    mg = tracks.MatchGraph(pairs, m0, m1)
    i0, i1 = mg(0, 1)
    assert i0.tolist() == [1, 4] and i1.tolist() == [3, 5]
    i0, i1 = mg(1, 0)
    assert i0.tolist() == [3, 5] and i1.tolist() == [1, 4]


def test_track_merge_quirks():
    """matching.py:169-170 writes the reference image's track at p2 from the id
    image's track at p1, and appends the reference track at p1 (may be -1)."""
    tr = np.full(4, -1, np.int32)
    ti = np.full(4, -1, np.int32)
    ti[0] = 7                       # id image already tracked at index 0 (== p1 below)
    i0 = np.array([0, 1], np.int64)
    i1 = np.array([2, 1], np.int64)
    nid = np.array([10], np.int64)
    pid = np.empty(2, np.int64)
    lib = tracks.lib
    rc = lib.sfmhip_track_merge(tracks._ptr(tr), 4, tracks._ptr(ti), 4, tracks._ptr(i0), tracks._ptr(i1), 2,
                                tracks._ptr(nid), tracks._ptr(pid))
    assert rc == 0
    # match (0,2): ref[0]=-1, id[2]=-1 -> new id 10 for both
    # match (1,1): ref[1]=-1, id[1]=-1 -> new id 11
    assert pid.tolist() == [10, 11] and nid[0] == 12
    tr = np.full(4, -1, np.int32)
    ti = np.full(4, -1, np.int32)
    ti[2] = 5
    ti[0] = 9
    i0 = np.array([0], np.int64)
    i1 = np.array([2], np.int64)
    rc = lib.sfmhip_track_merge(tracks._ptr(tr), 4, tracks._ptr(ti), 4, tracks._ptr(i0), tracks._ptr(i1), 1,
                                tracks._ptr(nid), tracks._ptr(pid))
    # ref[0]=-1, id[2]=5 (not both -1); ref[0]==-1 -> elif id[p1=0]=9 != -1 -> ref[p2=2] = 9; append ref[0] = -1
    assert rc == 0 and tr[2] == 9 and pid[0] == -1
