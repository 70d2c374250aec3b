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
"""
from __future__ import annotations

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


def vq(obs, code_book):
    """matching.py:27 calls scipy.cluster.vq.vq; the oracle IS that call."""
    return _scipy_vq(np.asarray(obs, np.float64), np.asarray(code_book, np.float64))
