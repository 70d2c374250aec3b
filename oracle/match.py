"""Oracle for M1 (BF-L2 + ratio test) and M2 (vq).  TEST INFRASTRUCTURE ONLY.

M1 has no reference implementation: the reference matches with LightGlue at
matching.py:20,122-128.  The build's semantics:
  * quantise: SIFT-like integer values q = clip(rint(x),0,255) - 128;
    float descriptors q = clip(rint(127 x), -127, 127) (float32 arithmetic).
  * d(i,j) = |q_a_i - q_b_j|^2, exact integers.
  * j1 = lowest index attaining min_j d(i,j)   (scipy vq tie rule, matching.py:27)
  * d2 = min over j != j1
  * accept iff den^2 * d1 < num^2 * d2  (Lowe ratio r = num/den, exact)
  * mutual (optional): keep i->j only if j->i is the accepted match of the
    reverse direction (lightglue/lightglue.py:241-253 mutual rule).
Distances use float32 GEMM on integer operands: every product and partial sum
is an integer below 2^24, so the GEMM is exact (|dot| <= 127^2*256 < 2^23).

Exact float mode (bf_match_exact; the matcher receives FLOAT descriptors at
matching.py:111-122 — DISK from feature_extraction.py:10, SuperPoint-256 in
config C3): the same top-2 / ratio rules on
  d(i,j) = sum_k (f64(a_ik) - f64(b_jk))^2
accumulated in k order with one IEEE f64 operation per step (subtract, square,
add: no FMA), and the ratio test den^2*d1 < num^2*d2 decided on those f64
values as exact rationals.  Build-defined (no reference BF matcher); on
integer-valued data it equals the quantised semantics above (pinned by the vq
and filter_matches goldens), parity of the float rounding rule unpinned.
"""
from __future__ import annotations

from fractions import Fraction

import numpy as np
from scipy.cluster.vq import vq as _scipy_vq

MODE_SIFT = 0
MODE_FLOAT = 1


def quantize(x, mode: int) -> np.ndarray:
    x = np.asarray(x, dtype=np.float32)
    if mode == MODE_SIFT:
        return (np.clip(np.rint(x), 0, 255).astype(np.int32) - 128).astype(np.int8)
    r = np.rint(np.float32(127.0) * x)
    return np.clip(r, -127, 127).astype(np.int8)


def sq_dist(qa: np.ndarray, qb: np.ndarray) -> np.ndarray:
    """Exact squared L2 between int8 rows, int64 (M, N)."""
    A = qa.astype(np.float32)
    B = qb.astype(np.float32)
    dot = (A @ B.T).astype(np.int64)
    na = (qa.astype(np.int64) ** 2).sum(1)
    nb = (qb.astype(np.int64) ** 2).sum(1)
    return na[:, None] + nb[None, :] - 2 * dot


def top2(D: np.ndarray):
    """(j1, d1, d2) per row; j1 lowest index on ties; d2 = min over j != j1."""
    M, N = D.shape
    if N == 0:
        return np.full(M, -1), np.full(M, -1), np.full(M, -1)
    j1 = D.argmin(1)
    d1 = D[np.arange(M), j1]
    if N < 2:
        return j1, d1, np.full(M, np.iinfo(np.int64).max)
    D2 = D.copy()
    D2[np.arange(M), j1] = np.iinfo(np.int64).max
    d2 = D2.min(1)
    return j1, d1, d2


def bf_match_q(qa, qb, ratio=(3, 4), mutual: bool = False, return_dist: bool = False):
    """Oracle matches0 (M,) int64 for int8 descriptors qa (M,d), qb (N,d)."""
    num, den = ratio
    qa = np.asarray(qa, np.int8)
    qb = np.asarray(qb, np.int8)
    M, N = qa.shape[0], qb.shape[0]
    if M == 0:
        out = np.zeros(0, np.int64)
        return (out, out, out) if return_dist else out
    if N < 2:
        out = np.full(M, -1, np.int64)
        return (out, out, out) if return_dist else out
    D = sq_dist(qa, qb)
    j1, d1, d2 = top2(D)
    ok = (den * den) * d1 < (num * num) * d2
    m0 = np.where(ok, j1, -1).astype(np.int64)
    if mutual:
        j1b, d1b, d2b = top2(D.T)
        okb = (den * den) * d1b < (num * num) * d2b
        m1 = np.where(okb, j1b, -1)
        keep = (m0 >= 0) & (m1[np.clip(m0, 0, None)] == np.arange(M))
        m0 = np.where(keep, m0, -1)
    if return_dist:
        return m0, d1, d2
    return m0


def bf_match_mutual_pair(qa, qb, ratio=(3, 4)):
    """(matches0, matches1) after the mutual filter, both directions ratio-tested."""
    m0 = bf_match_q(qa, qb, ratio, mutual=True)
    m1 = bf_match_q(qb, qa, ratio, mutual=True)
    return m0, m1


def bf_match(desc0, desc1, ratio=0.75, mutual=False, mode=MODE_FLOAT):
    from fractions import Fraction
    fr = Fraction(str(ratio)).limit_denominator(65535)
    return bf_match_q(quantize(desc0, mode), quantize(desc1, mode), (fr.numerator, fr.denominator), mutual)


def sq_dist_exact(xa, xb) -> np.ndarray:
    """Exact-float-mode distance (module docstring), f64 (M, N)."""
    A = np.asarray(xa, np.float32).astype(np.float64)
    BT = np.ascontiguousarray(np.asarray(xb, np.float32).astype(np.float64).T)
    D = np.zeros((A.shape[0], BT.shape[1]))
    rows = max(1, 65536 // max(1, BT.shape[1]))          # row blocks that stay in cache across the k loop
    t = np.empty((rows, BT.shape[1]))
    for r0 in range(0, A.shape[0], rows):
        Dr = D[r0:r0 + rows]
        tr = t[:Dr.shape[0]]
        for k in range(A.shape[1]):                     # k order, one IEEE op per step
            np.subtract(A[r0:r0 + rows, k][:, None], BT[k][None, :], out=tr)
            np.multiply(tr, tr, out=tr)
            np.add(Dr, tr, out=Dr)
    return D


def top2_f(D: np.ndarray):
    """(j1, d1, d2) of a float distance matrix; j1 lowest index on ties; d2 = min over j != j1."""
    M = D.shape[0]
    j1 = D.argmin(1)
    d1 = D[np.arange(M), j1]
    D2 = D.copy()
    D2[np.arange(M), j1] = np.inf
    return j1, d1, D2.min(1)


def ratio_accept_exact(d1, d2, num: int, den: int) -> np.ndarray:
    """den^2 * d1 < num^2 * d2 on f64 values, decided as exact rationals."""
    return np.array([Fraction(float(a)) * (den * den) < Fraction(float(b)) * (num * num)
                     for a, b in zip(np.ravel(d1), np.ravel(d2))], dtype=bool)


def bf_match_exact(xa, xb, ratio=(3, 4), mutual: bool = False, return_dist: bool = False):
    """Exact-float-mode matches0 (M,) int64 for f32 descriptors xa (M,d), xb (N,d)."""
    num, den = ratio
    xa = np.asarray(xa, np.float32)
    xb = np.asarray(xb, np.float32)
    M, N = xa.shape[0], xb.shape[0]
    if M == 0 or N < 2:
        out = np.full(M, -1, np.int64)
        nan = np.full(M, np.nan)
        return (out, nan, nan) if return_dist else out
    D = sq_dist_exact(xa, xb)
    j1, d1, d2 = top2_f(D)
    m0 = np.where(ratio_accept_exact(d1, d2, num, den), j1, -1).astype(np.int64)
    if mutual:
        j1b, d1b, d2b = top2_f(D.T)
        m1 = np.where(ratio_accept_exact(d1b, d2b, num, den), j1b, -1)
        keep = (m0 >= 0) & (m1[np.clip(m0, 0, None)] == np.arange(M))
        m0 = np.where(keep, m0, -1)
    return (m0, d1, d2) if return_dist else m0


def bf_match_gemm_f32(xa, xb, ratio=(3, 4)):
    """The host path a numpy user would run at the matching.py:122 call site
    ("numpy oracle GEMM-form", the survey's 192 ms/pair probe):
    f32 d = |a|^2 + |b|^2 - 2 A @ B.T, top two by argpartition, ratio test on
    the f32 values.  bench.py's CPU baseline for the float headline times THIS
    form; it is not the parity oracle (its f32 rounding can reorder near-ties,
    which bf_match_exact decides exactly)."""
    num, den = ratio
    A = np.asarray(xa, np.float32)
    B = np.asarray(xb, np.float32)
    M, N = A.shape[0], B.shape[0]
    if M == 0 or N < 2:
        return np.full(M, -1, np.int64)
    D = (A * A).sum(1)[:, None] + (B * B).sum(1)[None, :] - np.float32(2) * (A @ B.T)
    p = np.argpartition(D, 1, axis=1)[:, :2]
    r = np.arange(M)
    da, db = D[r, p[:, 0]], D[r, p[:, 1]]
    first = (da < db) | ((da == db) & (p[:, 0] < p[:, 1]))
    j1 = np.where(first, p[:, 0], p[:, 1])
    d1, d2 = np.minimum(da, db), np.maximum(da, db)
    ok = np.float32(den * den) * d1 < np.float32(num * num) * d2
    return np.where(ok, j1, -1).astype(np.int64)


def bf_match_exact_mutual_pair(xa, xb, ratio=(3, 4)):
    """(matches0, matches1) of the exact float mode after the mutual filter."""
    return bf_match_exact(xa, xb, ratio, mutual=True), bf_match_exact(xb, xa, ratio, mutual=True)


def vq(obs, code_book):
    """matching.py:27 calls scipy.cluster.vq.vq; the oracle IS that call."""
    return _scipy_vq(np.asarray(obs, np.float64), np.asarray(code_book, np.float64))
