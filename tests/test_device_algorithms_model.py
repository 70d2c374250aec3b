"""CPU models of three device algorithms whose correctness arguments are numerical or
number-theoretic rather than bit-for-bit against the oracle:

* geom_dev.h `wave_reduce_scatter`: the reduce-scatter form of the wave sums adds every value
  along the same pairwise tree as the plain xor butterfly (offset 32 first), so the per-value sums
  are the same floating-point results (the claim behind "the same bits" in pnp.hip / ba.hip).
* pnp.hip `epnp_eig4_tri`: the four smallest eigenpairs of the Householder tridiagonal by
  Sturm-count trisection (leading-minor recurrence on the power-of-two-scaled
  matrix) and inverse iteration with partial pivoting (the four vectors in lockstep, modified
  Gram-Schmidt after every step), restated step for step in numpy and checked against LAPACK
  (numpy.linalg.eigh) on EPnP-like M^T M matrices.
* geom_dev.h `cv_rng_sample_wave`: cv::RNG jump-ahead; the wave-parallel sampler gives the serial
  cv_rng_sample5 sequence and final state exactly.
"""
import math

import numpy as np


def _butterfly(vals):
    """vals: (64, K) per-lane values -> (K,) the xor-butterfly wave sums as lane 0 sees them."""
    x = vals.copy()
    for o in (32, 16, 8, 4, 2, 1):
        x = x + x[np.arange(64) ^ o]
    return x[0]


def _reduce_scatter(vals):
    """The device reduce-scatter on 64 lanes: returns {value index: sum} from the writer lanes."""
    K = vals.shape[1]
    P = 0 if K <= 1 else int(math.ceil(math.log2(K)))
    NP = 1 << P
    x = np.zeros((64, NP))
    x[:, :K] = vals
    lanes = np.arange(64)
    for st in range(P):
        o, half = 32 >> st, NP >> (st + 1)
        hi = (lanes & o) != 0
        keep = np.where(hi[:, None], x[:, half:2 * half], x[:, :half])
        send = np.where(hi[:, None], x[:, :half], x[:, half:2 * half])
        x = x.copy()
        x[:, :half] = keep + send[lanes ^ o]
    o = 32 >> P
    while o >= 1:
        x[:, 0] = x[:, 0] + x[lanes ^ o, 0]
        o >>= 1
    out = {}
    for lane in range(64):
        idx = lane >> (6 - P)
        if (lane & ((64 >> P) - 1)) == 0 and idx < K:
            out[idx] = x[lane, 0]
    return out


def test_reduce_scatter_matches_butterfly_bits():
    rng = np.random.default_rng(7)
    for K in (1, 2, 3, 6, 7, 13, 27, 28, 32):
        vals = rng.standard_normal((64, K)) * 10.0 ** rng.integers(-8, 8, (64, K))
        ref = _butterfly(vals)
        got = _reduce_scatter(vals)
        assert sorted(got) == list(range(K))
        for k in range(K):
            assert got[k] == ref[k], (K, k)   # identical floating-point sums


def _householder_tridiag(A):
    """EISPACK tred2-like reduction (the device order: column k reflected into rows k+1..)."""
    A = A.copy()
    n = A.shape[0]
    Q = np.eye(n)
    for k in range(n - 2):
        x = A[k + 1:, k].copy()
        n2 = x @ x
        x0 = x[0]
        s2 = n2 - x0 * x0
        if not (s2 > 1e-300 * n2) or not (n2 > 0):
            continue
        alpha = -math.sqrt(n2) if x0 >= 0 else math.sqrt(n2)
        v = x.copy()
        v[0] = x0 - alpha
        beta = 2.0 / (v @ v)
        H = np.eye(n)
        H[k + 1:, k + 1:] -= beta * np.outer(v, v)
        A = H @ A @ H
        Q = Q @ H
    return np.diag(A).copy(), np.diag(A, 1).copy(), Q


def _eig4_tri(d, e):
    """pnp.hip epnp_eig4_tri restated: 4 smallest eigenpairs of tridiag(d, e)."""
    n = len(d)
    r = np.abs(np.concatenate([[0.0], e])) + np.abs(np.concatenate([e, [0.0]]))
    lo, hi = np.min(d - r), np.max(d + r)
    tn = np.max(np.abs(d) + r)
    sc = math.ldexp(1.0, -(math.frexp(tn)[1] - 1) - 1) if tn > 0 else 1.0
    ds, es2 = d * sc, (e * sc) ** 2

    def count(x):
        p0, p1 = 1.0, ds[0] - x
        c = int(p1 < 0)
        for i in range(1, n):
            p2 = (ds[i] - x) * p1 - es2[i - 1] * p0
            c += int((p2 < 0) != (p1 < 0))
            p0, p1 = p1, p2
        return c

    lams = []
    for k in range(4):
        a, b = lo * sc - 2.0 ** -50, hi * sc + 2.0 ** -50
        for _ in range(30):
            w = (b - a) / 3.0
            m1, m2 = a + w, a + 2.0 * w
            if count(m1) > k:
                b = m1
            elif count(m2) > k:
                a, b = m1, m2
            else:
                a = m2
        lams.append(0.5 * (a + b) / sc)
    tol = 2.0 ** -52 * max(tn, 2.0 ** -1000)
    facts, ys = [], []
    for k in range(4):
        lk = lams[k]
        u0, u1, u2, lm, sw = np.zeros(n), np.zeros(n), np.zeros(n), np.zeros(n - 1), np.zeros(n - 1, bool)
        pd, p1, p2 = d[0] - lk, e[0], 0.0
        for i in range(n - 1):
            nd, n1, n2 = e[i], d[i + 1] - lk, (e[i + 1] if i + 1 < n - 1 else 0.0)
            sw[i] = abs(nd) > abs(pd)
            if not sw[i]:
                piv = (-tol if pd < 0 else tol) if abs(pd) < tol else pd
                m = nd / piv
                u0[i], u1[i], u2[i], lm[i] = piv, p1, p2, m
                pd, p1, p2 = n1 - m * p1, n2 - m * p2, 0.0
            else:
                m = pd / nd
                u0[i], u1[i], u2[i], lm[i] = nd, n1, n2, m
                pd, p1, p2 = p1 - m * n1, p2 - m * n2, 0.0
        u0[n - 1] = (-tol if pd < 0 else tol) if abs(pd) < tol else pd
        facts.append((u0, u1, u2, lm, sw))
        ys.append(np.array([1.0 / (1.0 + ((i * 7 + k * 5) % 12)) for i in range(n)]))
    # the four iterations in lockstep (one lane each); every step ends with modified
    # Gram-Schmidt in order 0..3 against the other lanes' current iterates
    for _ in range(3):
        for k in range(4):
            u0, u1, u2, lm, sw = facts[k]
            y = ys[k]
            for i in range(n - 1):
                if sw[i]:
                    y[i], y[i + 1] = y[i + 1], y[i]
                y[i + 1] -= lm[i] * y[i]
            y[n - 1] /= u0[n - 1]
            y[n - 2] = (y[n - 2] - u1[n - 2] * y[n - 1]) / u0[n - 2]
            for i in range(n - 3, -1, -1):
                y[i] = (y[i] - u1[i] * y[i + 1] - u2[i] * y[i + 2]) / u0[i]
        for j in range(4):
            ys[j] = ys[j] / math.sqrt(ys[j] @ ys[j])
            for k in range(j + 1, 4):
                ys[k] = ys[k] - (ys[k] @ ys[j]) * ys[j]
    Y = ys
    return np.array(lams), np.array(Y).T


def _epnp_mtm(rng, f=1500.0):
    """M^T M of a random 5-point EPnP sample (2 rows per point, 12 columns)."""
    alphas = rng.random((5, 4))
    alphas /= alphas.sum(1, keepdims=True)
    du, dv = rng.normal(0, 300, 5), rng.normal(0, 300, 5)
    M = np.zeros((10, 12))
    for p in range(5):
        for c in range(4):
            M[2 * p, 3 * c], M[2 * p, 3 * c + 2] = alphas[p, c] * f, alphas[p, c] * du[p]
            M[2 * p + 1, 3 * c + 1], M[2 * p + 1, 3 * c + 2] = alphas[p, c] * f, alphas[p, c] * dv[p]
    return M.T @ M


def test_eig4_tridiagonal_matches_lapack():
    rng = np.random.default_rng(11)
    for _ in range(60):
        A = _epnp_mtm(rng)
        d, e, Q = _householder_tridiag(A)
        lam, Yt = _eig4_tri(d, e)
        V = Q @ Yt
        w, U = np.linalg.eigh(A)
        scale = np.abs(w).max()
        assert np.all(np.diff(lam) >= -1e-12 * scale)
        assert np.allclose(lam, w[:4], atol=1e-11 * scale)
        # eigen-residuals and orthonormality of the four vectors
        assert np.linalg.norm(A @ V - V * lam, axis=0).max() <= 1e-10 * scale
        assert np.abs(V.T @ V - np.eye(4)).max() <= 1e-10
        # the two exact null vectors span LAPACK's null pair; the others match up to sign
        Pn = U[:, :2] @ U[:, :2].T
        assert np.linalg.norm(V[:, :2] - Pn @ V[:, :2]) <= 1e-7
        for k in (2, 3):
            if w[k + 1] - w[k] > 1e-6 * scale and w[k] - w[k - 1] > 1e-6 * scale:
                assert min(np.linalg.norm(V[:, k] - U[:, k]), np.linalg.norm(V[:, k] + U[:, k])) <= 1e-6


# ---------------------------------------------------------------------------------------------
# geom_dev.h cv_rng_sample_wave (pnp.hip's RANSAC chunks, ransac.hip's ess_pregen_kernel):
# cv::RNG's multiply-with-carry step s' = A lo(s) + hi(s) is
# s' = s b^-1 mod m (b = 2^32, m = A b - 1, b^-1 = A), so the state 5 L draws ahead is
# s A^(5 L) mod m, formed on the device as mwc_red^3(s C_L) with C_L = A^(5 L - 3) mod m
# (mwc_red(T) = (T >> 32) + lo32(T) A = T b^-1 mod m).  The wave's 64 lanes each draw one
# sample from their jumped state; the first lane whose five draws repeat an index redraws one at
# a time (cv_rng_sample5) and the lanes after it restart from its final state.

_A = 4164903690
_M = _A * (1 << 32) - 1


def _mwc(s):
    return (s & 0xFFFFFFFF) * _A + (s >> 32)


def _rng_mod(x, n):
    mg = (1 << 32) // n
    r = x - ((x * mg) >> 32) * n
    return r - n if r >= n else r


def _sample5(s, n):
    """geom_dev.h cv_rng_sample5 restated: (state after, five indices)"""
    d = []
    while len(d) < 5:
        s = _mwc(s)
        idx = _rng_mod(s & 0xFFFFFFFF, n)
        if idx not in d:
            d.append(idx)
    return s, d


def _mulred3(s, c):
    t = s * c
    for _ in range(3):
        t = (t >> 32) + (t & 0xFFFFFFFF) * _A
    assert t < 2 * _M
    return t - _M if t >= _M else t


def _jump_table():
    import re
    from pathlib import Path
    src = (Path(__file__).resolve().parent.parent / "3d_reconstruction_amd" / "csrc" / "geom_dev.h").read_text()
    body = src[src.index("kMwcJump5[64] = {"):]
    body = body[:body.index("};")]
    return [int(v, 16) for v in re.findall(r"0x([0-9a-f]+)ULL", body)]


def _parallel_chunk(rs, n, nh, C):
    out = [None] * nh
    base, b0 = rs, 0
    while True:
        starts, draws, dups = {}, {}, []
        for lane in range(b0, nh):
            L = lane - b0
            st = base if L == 0 else _mulred3(base, C[L])
            sv, d = st, []
            for _ in range(5):
                sv = _mwc(sv)
                d.append(_rng_mod(sv & 0xFFFFFFFF, n))
            starts[lane], draws[lane] = st, (sv, d)
            if len(set(d)) < 5:
                dups.append(lane)
        hs = dups[0] if dups else nh
        for lane in range(b0, hs):
            out[lane] = draws[lane][1]
        if hs >= nh:
            return draws[nh - 1][0], out
        s2, d2 = _sample5(starts[hs], n)
        out[hs] = d2
        base, b0 = s2, hs + 1
        if b0 >= nh:
            return base, out


def test_mwc_jump_sampler_matches_serial():
    C = _jump_table()
    assert len(C) == 64
    for L in range(1, 64):
        assert C[L] == pow(_A, 5 * L - 3, _M)
    # one step from any state is s * A mod m (the seed ~0 is >= m: its successor is not reduced)
    rs = (1 << 64) - 1
    assert _mwc(rs) % _M == rs * _A % _M
    for n in (6, 7, 9, 40, 300, 2000):
        s_ser = s_par = (1 << 64) - 1
        for chunk in range(4):
            nh = 64 if chunk < 3 else 23
            ser = []
            for _ in range(nh):
                s_ser, d = _sample5(s_ser, n)
                ser.append(d)
            s_par, par = _parallel_chunk(s_par, n, nh, C)
            assert par == ser, (n, chunk)
            assert s_par == s_ser, (n, chunk)
