"""Oracle for S2-S5.  TEST INFRASTRUCTURE ONLY.

OpenCV (cv2) is not installed here and not vendored under /root/reference, so
its arithmetic is restated from the published OpenCV 4.x sources
(calib3d/src/triangulate.cpp cvTriangulatePoints; calib3d/src/calibration.cpp
cvProjectPoints2Internal and cv::Rodrigues).  These are "parity unpinned" at
the OpenCV boundary; the scipy pieces (ba_sparse structure
grouping, approx_derivative) are the reference's own library code.

Reference call sites: sfm.py:27 (triangulatePoints), sfm.py:87-91
(calculate_reprojection_error -> cv2.projectPoints), sfm.py:37-38 / 79-85
(least_squares with jac_sparsity=ba_sparse).
"""
from __future__ import annotations

import math

import numpy as np
from scipy.optimize._numdiff import approx_derivative
from scipy.sparse import lil_matrix


def dlt_system(P0, P1, x0, y0, x1, y1) -> np.ndarray:
    """cvTriangulatePoints matrA (6x4): rows x*P[2]-P[0], y*P[2]-P[1], x*P[1]-y*P[0] per view."""
    A = np.empty((6, 4))
    for v, (P, x, y) in enumerate(((P0, x0, y0), (P1, x1, y1))):
        A[3 * v + 0] = x * P[2] - P[0]
        A[3 * v + 1] = y * P[2] - P[1]
        A[3 * v + 2] = x * P[1] - y * P[0]
    return A


def triangulate_points(P0, P1, pts0, pts1) -> np.ndarray:
    """cv2.triangulatePoints (sfm.py:27): (2,n) x2 -> (4,n), right singular vector
    of the smallest singular value of the 6x4 DLT system (unit norm, w >= 0)."""
    P0 = np.asarray(P0, np.float64)
    P1 = np.asarray(P1, np.float64)
    pts0 = np.asarray(pts0, np.float64).reshape(2, -1)
    pts1 = np.asarray(pts1, np.float64).reshape(2, -1)
    n = pts0.shape[1]
    A = np.empty((n, 6, 4))
    for v, (P, pts) in enumerate(((P0, pts0), (P1, pts1))):
        x = pts[0][:, None]
        y = pts[1][:, None]
        A[:, 3 * v + 0] = x * P[2] - P[0]
        A[:, 3 * v + 1] = y * P[2] - P[1]
        A[:, 3 * v + 2] = x * P[1] - y * P[0]
    _, _, vt = np.linalg.svd(A)
    X = vt[:, 3, :]
    X = X / np.linalg.norm(X, axis=1, keepdims=True)
    X = X * np.where(X[:, 3:4] < 0, -1.0, 1.0)
    return X.T.copy()


def rodrigues(rvec) -> np.ndarray:
    """cv::Rodrigues vector->matrix: R = (c I + c1 r r^T) + s [r]_x, r = rvec/theta."""
    rx, ry, rz = (float(v) for v in np.asarray(rvec, np.float64).ravel()[:3])
    theta = math.sqrt(rx * rx + ry * ry + rz * rz)
    if theta < 2.220446049250313e-16:
        return np.eye(3)
    c, s = math.cos(theta), math.sin(theta)
    c1 = 1.0 - c
    it = 1.0 / theta
    rx, ry, rz = rx * it, ry * it, rz * it
    rrt = [rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz]
    rxm = [0.0, -rz, ry, rz, 0.0, -rx, -ry, rx, 0.0]
    eye = [1.0, 0, 0, 0, 1.0, 0, 0, 0, 1.0]
    return np.array([(c * eye[k] + c1 * rrt[k]) + s * rxm[k] for k in range(9)]).reshape(3, 3)


def rodrigues_inverse(R) -> np.ndarray:
    """cv::Rodrigues matrix->vector (OpenCV 4.x calibration.cpp): project R onto
    SO(3) by SVD, then the axis-angle from the skew part (small- and
    pi-angle branches as in OpenCV).  Returns (3,1)."""
    u, _, vt = np.linalg.svd(np.asarray(R, np.float64))
    R = u @ vt
    rx, ry, rz = R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]
    s = math.sqrt((rx * rx + ry * ry + rz * rz) * 0.25)
    c = (R[0, 0] + R[1, 1] + R[2, 2] - 1) * 0.5
    c = 1.0 if c > 1.0 else (-1.0 if c < -1.0 else c)
    theta = math.acos(c)
    if s < 1e-5:
        if c > 0:
            return np.zeros((3, 1))
        t = (R[0, 0] + 1) * 0.5
        rx = math.sqrt(max(t, 0.0))
        t = (R[1, 1] + 1) * 0.5
        ry = math.sqrt(max(t, 0.0)) * (-1.0 if R[0, 1] < 0 else 1.0)
        t = (R[2, 2] + 1) * 0.5
        rz = math.sqrt(max(t, 0.0)) * (-1.0 if R[0, 2] < 0 else 1.0)
        if abs(rx) < abs(ry) and abs(rx) < abs(rz) and (R[1, 2] > 0) != (ry * rz > 0):
            rz = -rz
        theta /= math.sqrt(rx * rx + ry * ry + rz * rz)
        return np.array([[rx * theta], [ry * theta], [rz * theta]])
    vth = 1.0 / (2 * s) * theta
    return np.array([[rx * vth], [ry * vth], [rz * vth]])


def project_points(X, rvec, tvec, K) -> np.ndarray:
    """cvProjectPoints2Internal with zero distortion: (n,2).

    x = R X + t (left-to-right sums); z = z ? 1/z : 1; x *= z; u = x*fx + cx."""
    R = rodrigues(rvec)
    t = np.asarray(tvec, np.float64).ravel()
    K = np.asarray(K, np.float64).reshape(3, 3)
    X = np.asarray(X, np.float64).reshape(-1, 3)
    x = R[0, 0] * X[:, 0] + R[0, 1] * X[:, 1] + R[0, 2] * X[:, 2] + t[0]
    y = R[1, 0] * X[:, 0] + R[1, 1] * X[:, 1] + R[1, 2] * X[:, 2] + t[1]
    z = R[2, 0] * X[:, 0] + R[2, 1] * X[:, 1] + R[2, 2] * X[:, 2] + t[2]
    with np.errstate(divide="ignore"):
        z = np.where(z != 0, 1.0 / np.where(z != 0, z, 1.0), 1.0)
    x = x * z
    y = y * z
    return np.stack([x * K[0, 0] + K[0, 2], y * K[1, 1] + K[1, 2]], 1)


def reprojection_error(x, K, point_2D) -> np.ndarray:
    """sfm.py:87-91 calculate_reprojection_error with the projectPoints restatement."""
    x = np.asarray(x, np.float64)
    p2 = np.asarray(point_2D, np.float64).reshape(-1, 2)
    proj = project_points(x[6:].reshape(len(p2), 3), x[:3], x[3:6], K)
    return (p2 - proj).ravel()


def ba_sparse(len_point, len_x, y=6):
    """sfm.py:79-85 structure: every row touches the y camera columns; rows 2p and
    2p+1 touch the three columns of point p (y + 3p + 0..2)."""
    n = int(len_point)
    r_cam = np.repeat(np.arange(2 * n), y)
    c_cam = np.tile(np.arange(y), 2 * n)
    r_pt = np.repeat(np.arange(2 * n), 3)
    c_pt = y + 3 * np.repeat(np.arange(n), 6) + np.tile(np.arange(3), 2 * n)
    A = lil_matrix((2 * n, int(len_x)), dtype=int)
    A[np.concatenate([r_cam, r_pt]), np.concatenate([c_cam, c_pt])] = 1
    return A


def fd_jacobian(x, K, point_2D):
    """The Jacobian least_squares(method='trf', jac='2-point', jac_sparsity=
    ba_sparse(...)) builds at sfm.py:38: scipy's own approx_derivative
    (_sparse_difference, groups from group_columns) on the restated residual."""
    x = np.asarray(x, np.float64)
    p2 = np.asarray(point_2D, np.float64).reshape(-1, 2)
    A = ba_sparse(len(p2), len(x), 6)
    f0 = reprojection_error(x, K, p2)
    return approx_derivative(reprojection_error, x, method="2-point", f0=f0, sparsity=A,
                             args=(K, p2))


def fd_jacobian_direct(x, K, point_2D) -> np.ndarray:
    """Per-observation form of the same values: (n, 2, 9) — columns rvec, t, X_i.

    Each value is (f(x + h e_j)[row] - f0[row]) / ((x + h) - x) with
    h = EPS**0.5 * sign0(x) * max(1, |x|) (scipy _compute_absolute_step)."""
    x = np.asarray(x, np.float64)
    p2 = np.asarray(point_2D, np.float64).reshape(-1, 2)
    n = len(p2)
    f0 = reprojection_error(x, K, p2).reshape(n, 2)
    J = np.empty((n, 2, 9))
    rstep = np.finfo(np.float64).eps ** 0.5
    cols = [0, 1, 2, 3, 4, 5]
    for j in cols:
        h = rstep * (1.0 if x[j] >= 0 else -1.0) * max(1.0, abs(x[j]))
        xp = x.copy()
        xp[j] = x[j] + h
        dx = xp[j] - x[j]
        J[:, :, j] = ((reprojection_error(xp, K, p2).reshape(n, 2)) - f0) / dx
    for c in range(3):
        xp = x.copy()
        idx = 6 + 3 * np.arange(n) + c
        xv = x[idx]
        h = rstep * np.where(xv >= 0, 1.0, -1.0) * np.maximum(1.0, np.abs(xv))
        xp[idx] = xv + h
        dx = xp[idx] - xv
        J[:, :, 6 + c] = (reprojection_error(xp, K, p2).reshape(n, 2) - f0) / dx[:, None]
    return J
