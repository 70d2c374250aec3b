"""GPU parity: the exact float matching mode (int8 MFMA pass with a proven
residual bound + exact re-score of the undecided rows) vs oracle.bf_match_exact
(f64 k-ordered squared L2 of the f32 descriptors, exact rational ratio test).

Bar: bit-exact match indices.  Every test also runs with SFMHIP_MATCH_CERT=0
(no row certified: the exact pass settles every row) so both paths are checked."""
import importlib

import numpy as np
import pytest
import torch

from oracle import match as om

pytestmark = pytest.mark.gpu
syn = importlib.import_module("3d_reconstruction_amd.synthetic")


def _oracle(x, nk, pairs, ratio):
    out = np.full((len(pairs), x.shape[1]), -1, np.int64)
    for p, (a, b) in enumerate(pairs):
        out[p, :nk[a]] = om.bf_match_exact(x[a, :nk[a]], x[b, :nk[b]], ratio)
    return out


@pytest.mark.parametrize("cert", ["1", "0"])
@pytest.mark.parametrize("d,kind", [(256, "superpoint"), (128, "disk"), (64, "randn"), (128, "sift")])
def test_exact_float_ragged_pairs(sfm, gpu, knob, cert, d, kind):
    knob("MATCH_CERT", cert)
    n_img, m = 5, 600
    if kind == "randn":        # not normalised, components beyond the int8 range after rint(127 x): clipped rows
        x = torch.randn((n_img, m, d), generator=torch.Generator().manual_seed(d)).numpy() * 0.6
    elif kind == "sift":       # SIFT-like values 0..255 with fractional noise (mode 0)
        x = syn.sift_like(n_img, m, d, seed=d).numpy() + np.float32(0.37)
    else:
        x = syn.superpoint_like(n_img, m, d, seed=d + 1).numpy()
    nk = np.array([600, 513, 129, 600, 2], np.int32)
    for i in range(n_img):
        x[i, nk[i]:] = 0
    mode = 0 if kind == "sift" else 1
    pairs = np.array([[0, 1], [1, 0], [0, 2], [2, 3], [3, 0], [4, 0], [0, 4], [1, 1]], np.int32)
    bank = sfm.DescriptorBank.from_float(torch.from_numpy(x), n_kpts=nk, mode=mode, exact=True)
    m0 = bank.match(pairs, ratio=0.75).cpu().numpy()[:, :m]
    ref = _oracle(x, nk, pairs, (3, 4))
    assert np.array_equal(m0, ref)
    if cert == "0":
        assert int(bank.last_resolved.item()) == sum(int(nk[a]) for a, b in pairs if nk[b] >= 2)


@pytest.mark.parametrize("cert", ["1", "0"])
def test_exact_float_near_ties_and_ratio_boundary(sfm, gpu, knob, cert):
    """Rows whose int8 images tie or sit at the ratio boundary: exact ties
    (lowest index wins, then d1 == d2 -> reject), 1-ulp perturbations of the
    best candidate, and d1/d2 = 9/16 exactly (rejected: not strictly below)."""
    knob("MATCH_CERT", cert)
    rng = np.random.default_rng(5)
    d = 128
    a = (rng.standard_normal((64, d)) * 0.05).astype(np.float32)
    b = (rng.standard_normal((400, d)) * 0.05).astype(np.float32)
    for r in range(0, 40, 4):
        j = 10 * r
        b[j] = a[r]                                              # exact copy
        b[j + 3] = np.nextafter(a[r], np.float32(1))              # 1 ulp away, later index
        b[j + 1] = a[r + 1]                                       # duplicate pair for row r+1: exact tie
        b[j + 7] = a[r + 1]
    # d1 / d2 = 9 / 16 exactly: row 50 = 0, candidates at 3/1024 and 4/1024 along axis 0
    a[50] = 0
    b[300] = 0
    b[300, 0] = 3 / 1024
    b[301] = 0
    b[301, 0] = 4 / 1024
    b[302:400] = np.where(np.abs(b[302:400]) < 0.2, b[302:400] + 0.3, b[302:400])   # far from row 50
    # accept side of the boundary: 3/1024 vs 4/1024 + 1 ulp, around a point far from row 50's pair
    a[51] = 0
    a[51, 2] = 1.0
    b[303] = a[51]
    b[303, 1] = 3 / 1024
    b[304] = a[51]
    b[304, 1] = np.nextafter(np.float32(4 / 1024), np.float32(1))
    got = sfm.bf_match(a, b, ratio=0.75, exact=True)
    ref = om.bf_match_exact(a, b, (3, 4))
    assert np.array_equal(got, ref)
    assert ref[50] == -1 and ref[51] == 303


def test_exact_float_mutual_and_matcher_contract(sfm, gpu):
    x = syn.superpoint_like(3, 512, 128, seed=9).numpy()
    bank = sfm.DescriptorBank.from_float(torch.from_numpy(x), mode=1, exact=True)
    pairs = np.array([[0, 1], [2, 1]], np.int32)
    m0, m1 = bank.match(pairs, ratio=0.8, mutual=True)
    for p, (a, b) in enumerate(pairs):
        r0, r1 = om.bf_match_exact_mutual_pair(x[a], x[b], (4, 5))
        assert np.array_equal(m0[p].cpu().numpy(), r0) and np.array_equal(m1[p].cpu().numpy(), r1)
    data = {"image0": {"descriptors": torch.from_numpy(x[0:1]).to(gpu)},
            "image1": {"descriptors": torch.from_numpy(x[1:2, :300]).to(gpu)}}
    pred = sfm.Matcher()(data)                                   # exact by default
    r0, r1 = om.bf_match_exact_mutual_pair(x[0], x[1, :300], (3, 4))
    assert np.array_equal(pred["matches0"][0].cpu().numpy(), r0)
    assert np.array_equal(pred["matches1"][0].cpu().numpy(), r1)
    # scores: the Lowe margin 1 - sqrt(d1/d2) of the oracle's k-ordered f64 distances, bit for bit
    # (> 1 - 0.75 for every accepted match)
    sc = pred["matching_scores0"][0].cpu().numpy()
    D = om.sq_dist_exact(x[0], x[1, :300])
    for i in np.nonzero(r0 >= 0)[0]:
        d1 = D[i, r0[i]]
        d2 = np.min(np.delete(D[i], r0[i]))
        assert sc[i] == np.float32(1 - np.sqrt(d1 / d2)) and sc[i] > 0.25
    assert (sc[r0 < 0] == 0).all()


def test_exact_float_c3_full_size_sampled_rows(sfm, gpu):
    """C3 at full size on float SuperPoint-like descriptors: 32 pairs spread
    over the pair index space (near and far images), 384 rows each, bit-exact
    against the oracle; the exact pass touches a small share of the rows."""
    x = syn.superpoint_like(257, 4096, 256, seed=1, device=gpu)
    bank = sfm.DescriptorBank.from_float(x, mode=1, exact=True)
    del x
    pairs = sfm.all_pairs(257)
    m0 = bank.match(pairs)
    torch.cuda.synchronize()
    resolved = int(bank.last_resolved.item())
    assert resolved < 0.01 * len(pairs) * 4096
    rng = np.random.default_rng(7)
    near = [p for p in range(len(pairs)) if pairs[p][1] - pairs[p][0] <= 2]
    sample = list(rng.choice(near, 16, replace=False)) + list(rng.choice(len(pairs), 16, replace=False))
    for p in sample:
        a, b = pairs[p]
        rows = np.sort(rng.choice(4096, 384, replace=False))
        xa = bank.x[a, rows].cpu().numpy()
        xb = bank.x[b].cpu().numpy()
        ref = om.bf_match_exact(xa, xb, (3, 4))
        assert np.array_equal(m0[p, rows].cpu().numpy(), ref), p
    assert (m0[near[:50]] >= 0).float().mean().item() > 0.03


def _sq_dist_exact_torch(xa, xb):
    """oracle/match.py:sq_dist_exact restated with torch on the device, op for op (f32 -> f64,
    then per k: subtract, square, add — separate IEEE ops, k order): the test's fast checker
    for whole C3 pairs, pinned bit for bit to the numpy oracle below."""
    a = xa.float().double()
    bt = xb.float().double().t().contiguous()
    D = torch.zeros((a.shape[0], bt.shape[1]), dtype=torch.float64, device=a.device)
    t = torch.empty_like(D)
    for k in range(a.shape[1]):
        torch.sub(a[:, k:k + 1], bt[k][None, :], out=t)
        t.mul_(t)
        D.add_(t)
    return D


def test_exact_float_c3_whole_pairs(sfm, gpu):
    """C3 at full size, exact float mode: 24 WHOLE pairs (every one of the 4096 rows; near and
    far images) against the oracle's decision rules (top2_f, ratio_accept_exact) on the
    oracle's distance, computed by its device restatement (bit-identical to sq_dist_exact,
    checked here on a slice)."""
    x = syn.superpoint_like(257, 4096, 256, seed=1, device=gpu)
    bank = sfm.DescriptorBank.from_float(x, mode=1, exact=True)
    del x
    pairs = sfm.all_pairs(257)
    m0 = bank.match(pairs)
    torch.cuda.synchronize()
    xa, xb = bank.x[3, :48], bank.x[200, :333]
    assert np.array_equal(_sq_dist_exact_torch(xa, xb).cpu().numpy(),
                          om.sq_dist_exact(xa.cpu().numpy(), xb.cpu().numpy()))
    rng = np.random.default_rng(11)
    near = [p for p in range(len(pairs)) if pairs[p][1] - pairs[p][0] <= 2]
    sample = list(rng.choice(near, 12, replace=False)) + list(rng.choice(len(pairs), 12, replace=False))
    for p in sample:
        a, b = pairs[p]
        D = _sq_dist_exact_torch(bank.x[a], bank.x[b]).cpu().numpy()
        j1, d1, d2 = om.top2_f(D)
        ref = np.where(om.ratio_accept_exact(d1, d2, 3, 4), j1, -1)
        assert np.array_equal(m0[p, :4096].cpu().numpy(), ref), p


def test_exact_float_resolve_bucket_overflow(sfm, gpu, knob):
    """More than 4096 undecided rows against one image (the resolve's per-image bucket): the
    collected pass stands down and the graph-scanning per-row pass settles every row; the graph
    equals the certified run's and the oracle's on sampled rows."""
    n_img, m, d = 3, 4096, 64
    x = syn.superpoint_like(n_img, m, d, seed=9).numpy()
    pairs = np.array([[0, 1], [2, 1], [1, 0]], np.int32)   # image 1 receives 8192 rows
    bank = sfm.DescriptorBank.from_float(torch.from_numpy(x), mode=1, exact=True)
    knob("MATCH_CERT", "0")   # every row undecided
    forced = bank.match(pairs, ratio=0.75).cpu().numpy()
    assert int(bank.last_resolved.item()) == len(pairs) * m
    knob("MATCH_CERT", "1")
    certified = bank.match(pairs, ratio=0.75).cpu().numpy()
    assert np.array_equal(forced, certified)
    rows = np.random.default_rng(3).choice(m, 48, replace=False)
    for p, (a, b) in enumerate(pairs):
        ref = om.bf_match_exact(x[a, rows], x[b], (3, 4))
        assert np.array_equal(forced[p, rows], ref)


@pytest.mark.parametrize("cert", ["1", "0"])
def test_exact_float_resolve_many_images(sfm, gpu, knob, cert):
    """More images than the resolve's offset scan takes at once (1024 positions of the XCD-major
    order per pass): the image offsets and per-XCD ranges carried across passes, with pairs whose
    image b sits before and after position 1024 on every XCD."""
    knob("MATCH_CERT", cert)
    n_img, m, d = 1100, 128, 64
    x = syn.superpoint_like(n_img, m, d, seed=21).numpy()
    nk = np.full(n_img, m, np.int32)
    nk[1093] = 77
    rng = np.random.default_rng(8)
    bs = np.concatenate([np.arange(8), np.arange(1088, 1100), [512, 1023, 1024, 1025]])
    pairs = np.array([[int(rng.integers(n_img)), int(b)] for b in bs], np.int32)
    bank = sfm.DescriptorBank.from_float(torch.from_numpy(x), n_kpts=nk, mode=1, exact=True)
    m0 = bank.match(pairs, ratio=0.75).cpu().numpy()[:, :m]
    assert np.array_equal(m0, _oracle(x, nk, pairs, (3, 4)))
    if cert == "0":
        assert int(bank.last_resolved.item()) == sum(int(nk[a]) for a, b in pairs)


def _i16(bank, pairs, **kw):
    out = torch.empty((len(pairs), bank.m_pad), dtype=torch.int16, device=bank.device)
    bank.match(pairs, out=out, **kw)
    return out.cpu().numpy().astype(np.int64)


@pytest.mark.parametrize("cert", ["1", "0"])
@pytest.mark.parametrize("d,kind", [(256, "superpoint"), (128, "sift"), (64, "randn")])
def test_int16_graph_equals_int32_graph(sfm, gpu, knob, cert, d, kind):
    """The kernels writing the int16 graph directly (dist.match_all_pairs_sharded's form:
    sfmhip_match_pairs_exact_i16 / sfmhip_match_pairs_i16) give the int32 graph's values in
    both modes; with every row undecided (MATCH_CERT=0) each row's transient mark carries
    ceil(8 sqrt(D2)) instead of D2 and the resolve still settles every row to the oracle's
    answer (the widest distances: SIFT-range values, clipped randn rows)."""
    knob("MATCH_CERT", cert)
    n_img, m = 4, 520
    if kind == "randn":
        x = torch.randn((n_img, m, d), generator=torch.Generator().manual_seed(d)).numpy() * 0.6
    elif kind == "sift":
        x = syn.sift_like(n_img, m, d, seed=d).numpy() + np.float32(0.37)
    else:
        x = syn.superpoint_like(n_img, m, d, seed=d + 1).numpy()
    nk = np.array([520, 300, 129, 2], np.int32)
    for i in range(n_img):
        x[i, nk[i]:] = 0
    mode = 0 if kind == "sift" else 1
    pairs = np.array([[0, 1], [1, 0], [0, 2], [2, 0], [3, 0], [0, 3], [1, 1]], np.int32)
    bank = sfm.DescriptorBank.from_float(torch.from_numpy(x), n_kpts=nk, mode=mode, exact=True)
    for exact in (True, False):
        g32 = bank.match(pairs, ratio=0.75, exact=exact).cpu().numpy().astype(np.int64)
        g16 = _i16(bank, pairs, ratio=0.75, exact=exact)
        assert np.array_equal(g16, g32), exact
        if exact and cert == "0":
            assert int(bank.last_resolved.item()) == sum(int(nk[a]) for a, b in pairs if nk[b] >= 2)
    assert np.array_equal(_i16(bank, pairs, ratio=0.75)[:, :m], _oracle(x, nk, pairs, (3, 4)))


def test_int16_graph_resolve_bucket_overflow(sfm, gpu, knob):
    """int16 graph, more than 4096 undecided rows against one image: the graph-scanning
    per-row pass reads the int16 marks (the same graph as the int32 run)."""
    n_img, m, d = 3, 4096, 64
    x = syn.superpoint_like(n_img, m, d, seed=9).numpy()
    pairs = np.array([[0, 1], [2, 1], [1, 0]], np.int32)
    bank = sfm.DescriptorBank.from_float(torch.from_numpy(x), mode=1, exact=True)
    knob("MATCH_CERT", "0")
    g16 = _i16(bank, pairs, ratio=0.75)
    assert int(bank.last_resolved.item()) == len(pairs) * m
    g32 = bank.match(pairs, ratio=0.75).cpu().numpy()
    assert np.array_equal(g16, g32)


def test_int16_graph_sharded_product_api(sfm, gpu):
    """dist.match_all_pairs_sharded on one rank returns the int16 graph straight from the
    kernels, equal to the int32 graph of bank.match."""
    sdist = importlib.import_module("3d_reconstruction_amd.dist")
    x = syn.superpoint_like(6, 640, 256, seed=4).to(gpu)
    bank = sfm.DescriptorBank.from_float(x, mode=1, exact=True)
    pairs = sfm.all_pairs(6)
    g = sdist.match_all_pairs_sharded(bank, torch.from_numpy(pairs).to(gpu), exact=True)
    assert g.dtype == torch.int16 and tuple(g.shape) == (len(pairs), bank.m_pad)
    ref = bank.match(pairs)
    assert torch.equal(g.long(), ref.long())
    with pytest.raises(ValueError):
        bank.match(pairs, out=torch.empty((len(pairs), bank.m_pad), dtype=torch.int16, device=gpu), mutual=True)


def test_int16_graph_c3_full_size_equals_int32(sfm, gpu):
    """The bench headline's graph (C3 at full size: 257 x 4096 x 256 float descriptors, all
    32,896 pairs, exact float mode, dist.match_all_pairs_sharded -> int16 written by the
    kernels) equals the int32 graph of bank.match entry for entry; sampled rows of both against
    the oracle are covered by test_exact_float_c3_full_size_sampled_rows."""
    sdist = importlib.import_module("3d_reconstruction_amd.dist")
    x = syn.superpoint_like(257, 4096, 256, seed=1, device=gpu)
    bank = sfm.DescriptorBank.from_float(x, mode=1, exact=True)
    del x
    pairs = torch.from_numpy(sfm.all_pairs(257)).to(gpu)
    g16 = sdist.match_all_pairs_sharded(bank, pairs, exact=True)
    assert g16.dtype == torch.int16
    n16 = int(bank.last_resolved.item())
    g32 = bank.match(pairs)
    assert int(bank.last_resolved.item()) == n16 > 0          # the same rows went to the exact pass
    for lo in range(0, pairs.shape[0], 4096):                 # compare in slices (the int32 graph is 539 MB)
        assert torch.equal(g16[lo:lo + 4096].to(torch.int32), g32[lo:lo + 4096]), lo


@pytest.mark.parametrize("cert", ["1", "0"])
def test_exact_float_empty_and_single_keypoint_images(sfm, gpu, knob, cert):
    """Exact float mode, int32 and int16 graphs: a query image with 0 keypoints yields only
    padding rows, a candidate image with 0 or 1 keypoints (no second-best) gives -1 for every
    query row, padding rows never match; the rest equals the oracle, and an image against itself
    matches nearly every row to its own index."""
    knob("MATCH_CERT", cert)
    x = syn.superpoint_like(3, 300, 128, seed=77).numpy()
    nk = np.array([0, 1, 300], np.int32)
    for i in range(3):
        x[i, nk[i]:] = 0
    pairs = np.array([[0, 2], [2, 0], [1, 2], [2, 1], [0, 1], [2, 2]], np.int32)
    bank = sfm.DescriptorBank.from_float(torch.from_numpy(x), n_kpts=nk, mode=1, exact=True)
    g32 = bank.match(pairs, ratio=0.75).cpu().numpy().astype(np.int64)
    g16 = _i16(bank, pairs, ratio=0.75)
    assert np.array_equal(g16, g32)
    assert np.array_equal(g32[:, :300], _oracle(x, nk, pairs, (3, 4))[:, :300])
    assert (g32[1] == -1).all() and (g32[3] == -1).all()       # candidate image empty / single keypoint
    assert (g32[0] == -1).all() and (g32[4] == -1).all()       # query image empty: padding rows only
    assert (g32[:, 300:] == -1).all()
    assert (g32[5, :300] == np.arange(300)).mean() > 0.9      # self-match: nearly every row its own index
