"""Oracle for §8f row 2 (geometric verification).  TEST INFRASTRUCTURE ONLY.

Reference call sites:
  matching.py:134-139  E, mask = cv2.findEssentialMat(m_kpts0, m_kpts1, K, method=cv2.RANSAC,
                                                        prob=0.999, threshold=1)
                       cv2.recoverPose(E, m_kpts0[mask > 0], m_kpts1[mask > 0], K)
  sfm.py:108,116-120   the same findEssentialMat on (pts0, pts1) f64, then
                       cv2.solvePnPRansac(X, pts1, K, zeros(5,1)) and cv2.recoverPose.

OpenCV is a third-party dependency (requirement.txt:4 ``opencv-python``,
unpinned) that is neither installed here nor vendored under /root/reference,
so this is a restatement of its published 4.x algorithm — **parity unpinned**
at the OpenCV boundary; the tests pin it with known-answer scenes instead:

* ``CvRNG`` — cv::RNG (core): multiply-with-carry, state = (uint64)-1 as in
  RANSACPointSetRegistrator::run (calib3d/src/ptsetreg.cpp); ``uniform(a, b)``
  = a + next() % (b - a).
* ``get_subset`` — RANSACPointSetRegistrator::getSubset: draw ``m`` indices,
  redrawing any index already in the subset.
* ``update_num_iters`` — RANSACUpdateNumIters (ptsetreg.cpp).
* ``ransac`` — RANSACPointSetRegistrator::run: a model replaces the best one iff
  its inlier count > max(best, m - 1); niters shrinks with each new best.
* ``five_point`` — EMEstimatorCallback::runKernel (calib3d/src/five-point.cpp),
  Nister's solver: 4-dim null space of the 5x9 epipolar system, the 10 cubic
  constraints (det E = 0, 2 E E^T E - tr(E E^T) E = 0) in the monomial order
  x^3 y^3 x^2y xy^2 x^2z x^2 y^2z y^2 xyz xy | xz^2 xz x yz^2 yz y z^3 z^2 z 1,
  A[:, :10]^-1 A[:, 10:], the 3x3 polynomial matrix B(z) from rows 4..9,
  det B(z) (degree 10), real roots (|imag| <= 1e-10), null vector of B(z) ->
  (x, y), E = x E0 + y E1 + z E2 + E3 normalised.  Build-defined choices,
  shared with the HIP kernel: real roots are visited in ascending order
  (OpenCV visits them in solvePoly's output order; only ties between two
  models of one sample can differ), LU pivots below 100*DBL_EPSILON make the
  sample degenerate (OpenCV's Mat::inv(DECOMP_LU) returns zeros then).
* ``sampson_error`` — EMEstimatorCallback::computeError, stored as float and
  compared with (float)(thresh^2) (findInliers).
* ``find_essential_mat`` — cv::findEssentialMat (RANSAC, maxIters 1000):
  points normalised (x - cx)/fx, threshold /= (fx + fy)/2.
* ``decompose_essential_mat`` / ``recover_pose`` — cv::decomposeEssentialMat,
  cv::recoverPose (distanceThresh 50, cheirality on the DLT triangulation).
"""
from __future__ import annotations

import math

import numpy as np

from .geometry import triangulate_points

DBL_EPSILON = np.finfo(np.float64).eps
DBL_MIN = np.finfo(np.float64).tiny


# --- cv::RNG + RANSAC driver (ptsetreg.cpp) ----------------------------------
class CvRNG:
    def __init__(self, state: int = (1 << 64) - 1):
        self.state = state & ((1 << 64) - 1)

    def next(self) -> int:
        s = self.state
        self.state = ((s & 0xFFFFFFFF) * 4164903690 + (s >> 32)) & ((1 << 64) - 1)
        return self.state & 0xFFFFFFFF

    def uniform(self, a: int, b: int) -> int:
        return a if a == b else self.next() % (b - a) + a


def get_subset(rng: CvRNG, count: int, m: int) -> list[int]:
    idx: list[int] = []
    while len(idx) < m:
        while True:
            j = rng.uniform(0, count)
            if j not in idx:
                break
        idx.append(j)
    return idx


def cv_round(v: float) -> int:
    return int(np.rint(v))  # lrint: round half to even


def update_num_iters(p: float, ep: float, m: int, max_iters: int) -> int:
    p = min(max(p, 0.0), 1.0)
    ep = min(max(ep, 0.0), 1.0)
    num = max(1.0 - p, DBL_MIN)
    denom = 1.0 - math.pow(1.0 - ep, m)
    if denom < DBL_MIN:
        return 0
    num = math.log(num)
    denom = math.log(denom)
    return max_iters if (denom >= 0 or -num >= max_iters * (-denom)) else cv_round(num / denom)


def ransac(count: int, m: int, kernel, score, threshold: float, confidence: float, max_iters: int):
    """RANSACPointSetRegistrator::run.  kernel(idx) -> list of models;
    score(model) -> bool inlier mask (err <= (float)thresh^2).
    Returns (best_model, best_mask, n_iters_run) or (None, None, it)."""
    niters = max(max_iters, 1)
    if count < m:
        return None, None, 0
    if count == m:
        models = kernel(list(range(count)))
        if not models:
            return None, None, 1
        return models, np.ones(count, bool), 1
    rng = CvRNG()
    best, best_mask, max_good = None, None, 0
    it = 0
    while it < niters:
        idx = get_subset(rng, count, m)
        for model in kernel(idx):
            mask = score(model)
            good = int(mask.sum())
            if good > max(max_good, m - 1):
                best, best_mask, max_good = model, mask, good
                niters = update_num_iters(confidence, (count - good) / count, m, niters)
        it += 1
    if max_good <= 0:
        return None, None, it
    return best, best_mask, it


# --- polynomial algebra in (x, y, z) ------------------------------------------
_LIN = [(1, 0, 0), (0, 1, 0), (0, 0, 1), (0, 0, 0)]
_QUAD = [(2, 0, 0), (1, 1, 0), (1, 0, 1), (1, 0, 0), (0, 2, 0), (0, 1, 1), (0, 1, 0), (0, 0, 2), (0, 0, 1),
         (0, 0, 0)]
CUBIC = [(3, 0, 0), (0, 3, 0), (2, 1, 0), (1, 2, 0), (2, 0, 1), (2, 0, 0), (0, 2, 1), (0, 2, 0), (1, 1, 1),
         (1, 1, 0), (1, 0, 2), (1, 0, 1), (1, 0, 0), (0, 1, 2), (0, 1, 1), (0, 1, 0), (0, 0, 3), (0, 0, 2),
         (0, 0, 1), (0, 0, 0)]


def _add(e, f):
    return (e[0] + f[0], e[1] + f[1], e[2] + f[2])


_LL = np.array([[_QUAD.index(_add(a, b)) for b in _LIN] for a in _LIN])
_QL = np.array([[CUBIC.index(_add(a, b)) for b in _LIN] for a in _QUAD])


def _mul_ll(a, b):
    out = np.zeros(10)
    np.add.at(out, _LL, np.outer(a, b))
    return out


def _mul_ql(q, l):
    out = np.zeros(20)
    np.add.at(out, _QL, np.outer(q, l))
    return out


def coeff_matrix(basis: np.ndarray) -> np.ndarray:
    """basis (4, 9): E = x*b0 + y*b1 + z*b2 + b3 (row-major 3x3).  -> (10, 20)."""
    E = [[basis[:, 3 * i + j] for j in range(3)] for i in range(3)]  # linear polys [x, y, z, 1]
    EEt = [[sum(_mul_ll(E[i][k], E[j][k]) for k in range(3)) for j in range(3)] for i in range(3)]
    tr = EEt[0][0] + EEt[1][1] + EEt[2][2]
    rows = []
    det = (_mul_ql(_mul_ll(E[1][1], E[2][2]) - _mul_ll(E[1][2], E[2][1]), E[0][0])
           - _mul_ql(_mul_ll(E[1][0], E[2][2]) - _mul_ll(E[1][2], E[2][0]), E[0][1])
           + _mul_ql(_mul_ll(E[1][0], E[2][1]) - _mul_ll(E[1][1], E[2][0]), E[0][2]))
    rows.append(det)
    for i in range(3):
        for j in range(3):
            c = sum(2.0 * _mul_ql(EEt[i][k], E[k][j]) for k in range(3)) - _mul_ql(tr, E[i][j])
            rows.append(c)
    return np.array(rows)


def _lu_singular(A: np.ndarray) -> bool:
    """OpenCV hal LU: partial pivoting, singular if |pivot| < 100*DBL_EPSILON."""
    A = A.copy()
    n = A.shape[0]
    for k in range(n):
        p = k + int(np.argmax(np.abs(A[k:, k])))
        if abs(A[p, k]) < 100 * DBL_EPSILON:
            return True
        A[[k, p]] = A[[p, k]]
        A[k + 1:] -= np.outer(A[k + 1:, k] / A[k, k], A[k])
    return False


def five_point(q1: np.ndarray, q2: np.ndarray) -> list[np.ndarray]:
    """EMEstimatorCallback::runKernel on 5 normalised correspondences -> list of E (3,3)."""
    x1, y1 = q1[:, 0], q1[:, 1]
    x2, y2 = q2[:, 0], q2[:, 1]
    Q = np.stack([x1 * x2, y1 * x2, x2, x1 * y2, y1 * y2, y2, x1, y1, np.ones_like(x1)], axis=1)
    _, _, Vt = np.linalg.svd(Q, full_matrices=True)
    basis = Vt[5:9]                       # E = x v5 + y v6 + z v7 + v8
    A = coeff_matrix(basis)
    if _lu_singular(A[:, :10]):
        return []
    Ap = np.linalg.solve(A[:, :10], A[:, 10:])
    # B(z) rows: e = row 4+2r (x^2z, y^2z, xyz), f = row 5+2r (x^2, y^2, xy); B = e - z*f
    # columns of Ap: xz^2 xz x | yz^2 yz y | z^3 z^2 z 1
    px, py, pc = [], [], []
    for r in range(3):
        e, f = Ap[4 + 2 * r], Ap[5 + 2 * r]
        px.append(np.array([-f[0], e[0] - f[1], e[1] - f[2], e[2]]))             # z^3..z^0
        py.append(np.array([-f[3], e[3] - f[4], e[4] - f[5], e[5]]))
        pc.append(np.array([-f[6], e[6] - f[7], e[7] - f[8], e[8] - f[9], e[9]]))  # z^4..z^0
    pm, ps = np.polymul, np.polysub
    det = ps(ps(pm(px[0], ps(pm(py[1], pc[2]), pm(py[2], pc[1]))),
                pm(py[0], ps(pm(px[1], pc[2]), pm(px[2], pc[1])))),
             -pm(pc[0], ps(pm(px[1], py[2]), pm(px[2], py[1]))))
    roots = np.roots(det)
    zs = np.sort(roots[np.abs(roots.imag) <= 1e-10].real)
    out = []
    for z in zs:
        Bz = np.array([[np.polyval(px[r], z), np.polyval(py[r], z), np.polyval(pc[r], z)] for r in range(3)])
        xy1 = np.linalg.svd(Bz)[2][2]
        if abs(xy1[2]) < 1e-10:
            continue
        x, y = xy1[0] / xy1[2], xy1[1] / xy1[2]
        ev = x * basis[0] + y * basis[1] + z * basis[2] + basis[3]
        out.append((ev / np.linalg.norm(ev)).reshape(3, 3))
    return out


def sampson_error(E: np.ndarray, q1: np.ndarray, q2: np.ndarray) -> np.ndarray:
    """EMEstimatorCallback::computeError -> float32 per point."""
    x1 = np.column_stack([q1, np.ones(len(q1))])
    x2 = np.column_stack([q2, np.ones(len(q2))])
    Ex1 = x1 @ E.T
    Etx2 = x2 @ E
    x2tEx1 = np.sum(x2 * Ex1, axis=1)
    a, b = Ex1[:, 0] ** 2, Ex1[:, 1] ** 2
    c, d = Etx2[:, 0] ** 2, Etx2[:, 1] ** 2
    return (x2tEx1 * x2tEx1 / (a + b + c + d)).astype(np.float32)


def normalise(pts: np.ndarray, K: np.ndarray) -> np.ndarray:
    p = np.asarray(pts, np.float64).reshape(-1, 2)
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    return np.column_stack([(p[:, 0] - cx) / fx, (p[:, 1] - cy) / fy])


def find_essential_mat(points1, points2, K, prob: float = 0.999, threshold: float = 1.0,
                       max_iters: int = 1000, return_iters: bool = False):
    """cv::findEssentialMat(method=RANSAC).  -> (E (3,3) or (3k,3) or None, mask (n,1) uint8 or None)."""
    K = np.asarray(K, np.float64)
    q1, q2 = normalise(points1, K), normalise(points2, K)
    thresh = threshold / ((K[0, 0] + K[1, 1]) / 2)
    t = np.float32(thresh * thresh)
    E, mask, it = ransac(len(q1), 5, lambda idx: five_point(q1[idx], q2[idx]),
                         lambda M: sampson_error(M, q1, q2) <= t, thresh, prob, max_iters)
    if E is None:
        res = (None, None)
    else:
        E = np.vstack(E) if isinstance(E, list) else E
        res = (E, mask.astype(np.uint8).reshape(-1, 1))
    return res + (it,) if return_iters else res


def decompose_essential_mat(E: np.ndarray):
    U, _, Vt = np.linalg.svd(np.asarray(E, np.float64).reshape(3, 3))
    if np.linalg.det(U) < 0:
        U = -U
    if np.linalg.det(Vt) < 0:
        Vt = -Vt
    W = np.array([[0.0, 1, 0], [-1, 0, 0], [0, 0, 1]])
    return U @ W @ Vt, U @ W.T @ Vt, U[:, 2:3].copy()


def recover_pose(E, points1, points2, K, distance_thresh: float = 50.0, mask=None):
    """cv::recoverPose -> (n_good, R, t (3,1), mask (n,1) uint8 0/255)."""
    K = np.asarray(K, np.float64)
    q1, q2 = normalise(points1, K), normalise(points2, K)
    R1, R2, t = decompose_essential_mat(E)
    P0 = np.eye(3, 4)
    cands = [(R1, t), (R2, t), (R1, -t), (R2, -t)]
    masks = []
    for R, tt in cands:
        P = np.hstack([R, tt])
        Q = triangulate_points(P0, P, q1.T, q2.T)
        m = Q[2] * Q[3] > 0
        Q = Q / Q[3]
        m &= Q[2] < distance_thresh
        z = (P @ Q)[2]
        m &= (z > 0) & (z < distance_thresh)
        if mask is not None:
            m &= np.asarray(mask).ravel() > 0
        masks.append(m)
    good = [int(m.sum()) for m in masks]
    k = 0
    for c in range(4):
        if all(good[c] >= good[o] for o in range(4)):
            k = c
            break
    R, tt = cands[k]
    return good[k], R, tt, (masks[k].astype(np.uint8) * 255).reshape(-1, 1)
