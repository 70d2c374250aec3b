"""S1-S5: DLT triangulation, reprojection residual and the scipy grouped
finite-difference Jacobian, with the numpy signatures ``sfm.py`` calls.

Drop-in surfaces:

* :func:`triangulatePoints` — ``cv2.triangulatePoints`` (``sfm.py:27``)
* :func:`projectPoints` — ``cv2.projectPoints`` without distortion (``sfm.py:89``)
* :func:`calculate_reprojection_error` — ``sfm.py:87-91``
* :func:`ba_sparse` — ``sfm.py:79-85``
* :func:`fd_jacobian` — a ``jac=`` callable numerically identical (to the
  tolerance in tests/) to scipy's grouped 2-point FD that
  ``least_squares(..., jac_sparsity=ba_sparse(...))`` builds (``sfm.py:37-38``)
* batched forms (:func:`triangulate_batched`, :func:`residual_jacobian_batched`)
  over many pairs' observations resident on the GPU — the benchmarked path.

``Rodrigues`` and ``convertPointsFromHomogeneous`` are host helpers for the
3x3 / per-pair bookkeeping around the hot path (``sfm.py:29,36,39``); they are
not kernels.
"""
from __future__ import annotations

import math

import numpy as np
import torch
from scipy.sparse import csr_matrix, lil_matrix

from ._abi import call, dev, ptr, require_gpu, stream_ptr


# ---------------------------------------------------------------------------
# host helpers (not on the hot path)
def Rodrigues(src):
    """cv2.Rodrigues: (3,)/(3,1)/(1,3) vector -> ((3,3), None) or (3,3) -> ((3,1), None)."""
    a = np.asarray(src, dtype=np.float64)
    if a.size == 3:
        rx, ry, rz = (float(v) for v in a.ravel())
        theta = math.sqrt(rx * rx + ry * ry + rz * rz)
        if theta < 2.220446049250313e-16:
            return np.eye(3), None
        c, s = math.cos(theta), math.sin(theta)
        c1 = 1.0 - c
        it = 1.0 / theta
        rx, ry, rz = rx * it, ry * it, rz * it
        rrt = np.array([rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz])
        rxm = np.array([0, -rz, ry, rz, 0, -rx, -ry, rx, 0])
        eye = np.eye(3).ravel()
        return ((c * eye + c1 * rrt) + s * rxm).reshape(3, 3), None
    if a.shape != (3, 3):
        raise ValueError("Rodrigues expects a 3-vector or a 3x3 matrix")
    # matrix -> vector (OpenCV's SVD-projected formula)
    u, _, vt = np.linalg.svd(a)
    R = u @ vt
    rx, ry, rz = R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]
    s = math.sqrt((rx * rx + ry * ry + rz * rz) * 0.25)
    c = (R[0, 0] + R[1, 1] + R[2, 2] - 1) * 0.5
    c = min(max(c, -1.0), 1.0)
    theta = math.acos(c)
    if s < 1e-5:
        if c > 0:
            return np.zeros((3, 1)), None
        t = (R[0, 0] + 1) * 0.5
        rx = math.sqrt(max(t, 0.0))
        t = (R[1, 1] + 1) * 0.5
        ry = math.sqrt(max(t, 0.0)) * (-1.0 if R[0, 1] < 0 else 1.0)
        t = (R[2, 2] + 1) * 0.5
        rz = math.sqrt(max(t, 0.0)) * (-1.0 if R[0, 2] < 0 else 1.0)
        if abs(rx) < abs(ry) and abs(rx) < abs(rz) and (R[1, 2] > 0) != (ry * rz > 0):
            rz = -rz
        theta /= math.sqrt(rx * rx + ry * ry + rz * rz)
        return np.array([[rx * theta], [ry * theta], [rz * theta]]), None
    vth = 1.0 / (2 * s) * theta
    return np.array([[rx * vth], [ry * vth], [rz * vth]]), None


def convertPointsFromHomogeneous(src):
    """cv2.convertPointsFromHomogeneous for (n,4) -> (n,1,3)."""
    a = np.asarray(src, dtype=np.float64).reshape(-1, 4)
    w = a[:, 3:4]
    scale = np.where(w != 0, 1.0 / np.where(w != 0, w, 1.0), 1.0)
    return (a[:, :3] * scale)[:, None, :]


def ba_sparse(len_point: int, len_x: int, y: int = 6):
    """sfm.py:79-85 — the (2n, len_x) int sparsity of the BA Jacobian."""
    n = int(len_point)
    A = lil_matrix((2 * n, int(len_x)), dtype=int)
    rows = np.arange(2 * n)
    A[rows, :y] = 1
    for c in range(3):
        cols = y + 3 * np.arange(n) + c
        A[2 * np.arange(n), cols] = 1
        A[2 * np.arange(n) + 1, cols] = 1
    return A


# ---------------------------------------------------------------------------
# GPU-backed drop-ins
def triangulatePoints(projMatr1, projMatr2, projPoints1, projPoints2):
    """cv2.triangulatePoints: P1, P2 (3,4); points (2,n) -> homogeneous (4,n) f64.

    The 4-vector is the unit-norm DLT null vector with w >= 0 (OpenCV's sign is
    arbitrary; ``X / X[3]`` is identical)."""
    P = np.stack([np.asarray(projMatr1, np.float64).reshape(3, 4),
                  np.asarray(projMatr2, np.float64).reshape(3, 4)])[None]
    x0 = np.asarray(projPoints1, np.float64).reshape(2, -1)
    x1 = np.asarray(projPoints2, np.float64).reshape(2, -1)
    n = x0.shape[1]
    if x1.shape[1] != n:
        raise ValueError("projPoints1 and projPoints2 must have the same number of points")
    X4 = triangulate_batched(dev(P, torch.float64), None, dev(x0, torch.float64), dev(x1, torch.float64))
    torch.cuda.synchronize()
    return X4.cpu().numpy()


def triangulate_batched(P: torch.Tensor, pair_of_obs: torch.Tensor | None, x0: torch.Tensor,
                        x1: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Device-resident DLT: P (n_pairs,2,3,4) f64, x0/x1 (2,n) f64 -> (4,n) f64."""
    require_gpu()
    n = x0.shape[1]
    X4 = out if out is not None else torch.empty((4, n), dtype=torch.float64, device=x0.device)
    call("sfmhip_triangulate_dlt", ptr(P), ptr(pair_of_obs), ptr(x0), ptr(x1), n, ptr(X4), stream_ptr())
    return X4


def _K_of(K):
    return np.asarray(K, np.float64).reshape(1, 9)


def projectPoints(objectPoints, rvec, tvec, cameraMatrix, distCoeffs=None):
    """cv2.projectPoints (no distortion): returns ((n,1,2) f64, None).

    The reference discards the analytic jacobian output (``sfm.py:89``)."""
    if distCoeffs is not None and np.any(np.asarray(distCoeffs) != 0):
        raise NotImplementedError("distortion coefficients are not supported (sfm.py passes None)")
    X = np.asarray(objectPoints, np.float64).reshape(-1, 3)
    cam = np.concatenate([np.asarray(rvec, np.float64).ravel(), np.asarray(tvec, np.float64).ravel()])
    r = _residual(cam, _K_of(cameraMatrix), X, None)
    return (-r).reshape(-1, 1, 2), None


def _residual(cam, K, X, pts2d):
    """Host arrays in, host (n,2) out, through sfmhip_reproj_residual_host: one pinned
    staging buffer, one copy each way and a stream synchronisation per call (scipy's
    least_squares calls this ~40 times per pair at sfm.py:38).  pts2d None = zeros."""
    require_gpu()
    n = X.shape[0]
    cam = np.ascontiguousarray(cam, np.float64)
    K = np.ascontiguousarray(K, np.float64)
    X = np.ascontiguousarray(X, np.float64)
    r = np.empty((n, 2), np.float64)
    if pts2d is not None:
        pts2d = np.ascontiguousarray(pts2d, np.float64)
        if pts2d.shape != (n, 2):
            raise ValueError("point_2D must have one (x, y) row per 3D point")
    if cam.size != 6 or K.size != 9 or X.shape != (n, 3):
        raise ValueError("cam (6,), K (3,3) and X (n,3) expected")
    call("sfmhip_reproj_residual_host", cam.ctypes.data, K.ctypes.data, X.ctypes.data,
         None if pts2d is None else pts2d.ctypes.data, n, r.ctypes.data, stream_ptr())
    return r


def calculate_reprojection_error(x, K, point_2D):
    """sfm.py:87-91: x = [rvec(3), t(3), X(3n)] -> (point_2D - proj).ravel() (2n,)."""
    x = np.asarray(x, np.float64)
    p2 = np.asarray(point_2D, np.float64).reshape(-1, 2)
    X = x[6:].reshape(len(p2), 3)
    return _residual(x[:6], _K_of(K), X, p2).ravel()


def _jac_structure(n: int):
    cols = np.empty((n, 2, 9), dtype=np.int32)
    cols[:, :, :6] = np.arange(6, dtype=np.int32)
    cols[:, :, 6:] = (6 + 3 * np.arange(n, dtype=np.int32))[:, None, None] + np.arange(3, dtype=np.int32)
    indptr = np.arange(0, 18 * n + 1, 9, dtype=np.int32)
    return cols.ravel(), indptr


def fd_jacobian(x, K, point_2D, f0=None):
    """``jac=`` callable for ``least_squares``: scipy's 2-point grouped FD of
    :func:`calculate_reprojection_error` as a CSR matrix (2n, 6+3n)."""
    x = np.asarray(x, np.float64)
    p2 = np.asarray(point_2D, np.float64).reshape(-1, 2)
    n = len(p2)
    camt = dev(x[:6].reshape(1, 6), torch.float64)
    Kt = dev(_K_of(K), torch.float64)
    Xt = dev(x[6:].reshape(n, 3), torch.float64)
    pt = dev(p2, torch.float64)
    f0t = dev(np.asarray(f0, np.float64).reshape(n, 2), torch.float64) if f0 is not None else None
    jv = torch.empty((n, 2, 9), dtype=torch.float64, device=Xt.device)
    call("sfmhip_reproj_fd_jacobian", ptr(camt), ptr(Kt), ptr(Xt), ptr(pt), None, 1, n, ptr(f0t), None,
         ptr(jv), stream_ptr())
    torch.cuda.synchronize()
    indices, indptr = _jac_structure(n)
    return csr_matrix((jv.cpu().numpy().ravel(), indices, indptr), shape=(2 * n, 6 + 3 * n))


def residual_jacobian_batched(cam: torch.Tensor, K: torch.Tensor, X: torch.Tensor, pts2d: torch.Tensor,
                              pair_of_obs: torch.Tensor | None, r: torch.Tensor | None = None,
                              jv: torch.Tensor | None = None):
    """Device-resident residual + FD Jacobian over many pairs' observations.

    cam (n_pairs,6), K (n_pairs,3,3), X (n,3), pts2d (n,2) f64; pair_of_obs (n,) int32.
    Returns r (n,2) and jvals (n,2,9) (CSR values, columns rvec, t, X_i)."""
    require_gpu()
    n = X.shape[0]
    dvc = X.device
    r = r if r is not None else torch.empty((n, 2), dtype=torch.float64, device=dvc)
    jv = jv if jv is not None else torch.empty((n, 2, 9), dtype=torch.float64, device=dvc)
    call("sfmhip_reproj_fd_jacobian", ptr(cam), ptr(K), ptr(X), ptr(pts2d), ptr(pair_of_obs),
         int(cam.shape[0]), n, None, ptr(r), ptr(jv), stream_ptr())
    return r, jv


def ba_solve_batched(cam: torch.Tensor, K: torch.Tensor, X: torch.Tensor, pts2d: torch.Tensor,
                     pair_off: torch.Tensor, ftol: float = 1e-8, xtol: float = 1e-8, gtol: float = 1e-8,
                     max_nfev: int | None = None, validate: bool = True) -> dict:
    """The BA solve of sfm.py:37-38 for every pair at once, on the GPU (ba.hip):
    scipy ``least_squares(calculate_reprojection_error, [rvec, t, X], jac_sparsity=
    ba_sparse(...), x_scale='jac', ftol=ftol)`` restated (oracle/ba.py).

    cam (P,6) and X (n,3) f64 device tensors are updated in place; K (P,3,3),
    pts2d (n,2) f64; pair_off (P+1) int64 (pair p owns observations
    [pair_off[p], pair_off[p+1])).  Returns device tensors cost (P,) f64 and
    nfev, njev, status (P,) int32 (scipy's meanings; -1 = malformed offsets).

    ``validate`` checks pair_off on the device (off[0] = 0, non-decreasing,
    off[P] = n) and raises ValueError — one reduction and a host sync; the
    kernel itself never reads or writes outside [0, n) whatever the offsets
    (a pair with bad offsets is skipped with status -1)."""
    require_gpu()
    P = int(cam.shape[0])
    for name, t, dt in (("cam", cam, torch.float64), ("K", K, torch.float64), ("X", X, torch.float64),
                        ("pts2d", pts2d, torch.float64), ("pair_off", pair_off, torch.int64)):
        if t.dtype != dt or not t.is_cuda or not t.is_contiguous():
            raise ValueError(f"{name} must be a contiguous {dt} device tensor")
    n = int(X.shape[0])
    if tuple(cam.shape) != (P, 6) or tuple(K.shape) != (P, 3, 3) or tuple(X.shape) != (n, 3) or \
            tuple(pts2d.shape) != (n, 2) or tuple(pair_off.shape) != (P + 1,):
        raise ValueError("shapes must be cam (P,6), K (P,3,3), X (n,3), pts2d (n,2), pair_off (P+1,)")
    dvc = cam.device
    if validate and P > 0:
        bad = (pair_off[0] != 0) | (pair_off[-1] != n) | (pair_off[1:] < pair_off[:-1]).any()
        if bool(bad.item()):
            raise ValueError("pair_off must start at 0, be non-decreasing and end at X.shape[0]")
    cost = torch.empty(P, dtype=torch.float64, device=dvc)
    nfev = torch.empty(P, dtype=torch.int32, device=dvc)
    njev = torch.empty(P, dtype=torch.int32, device=dvc)
    status = torch.empty(P, dtype=torch.int32, device=dvc)
    call("sfmhip_ba_solve", ptr(cam), ptr(K), ptr(X), ptr(pts2d), ptr(pair_off), P, n, float(ftol), float(xtol),
         float(gtol), int(max_nfev or 0), ptr(cost), ptr(nfev), ptr(njev), ptr(status), stream_ptr())
    return {"cost": cost, "nfev": nfev, "njev": njev, "status": status}


def least_squares_ba(x0, K, point_2D, ftol: float = 1e-8, xtol: float = 1e-8, gtol: float = 1e-8,
                     max_nfev: int | None = None):
    """Drop-in for sfm.py:38 ``least_squares(calculate_reprojection_error, x0,
    jac_sparsity=ba_sparse(...), x_scale='jac', ftol=1e-8, args=(K, point_2D))``
    on one pair: returns an object with scipy's ``x``, ``cost``, ``fun``,
    ``nfev``, ``njev``, ``status`` and ``success``."""
    from types import SimpleNamespace
    dv = require_gpu()
    x0 = np.asarray(x0, np.float64)
    p2 = np.asarray(point_2D, np.float64).reshape(-1, 2)
    n = len(p2)
    if x0.shape != (6 + 3 * n,):
        raise ValueError(f"x0 must have 6 + 3 * {n} entries")
    cam = torch.tensor(x0[:6].reshape(1, 6), device=dv)
    X = torch.tensor(x0[6:].reshape(n, 3), device=dv)
    Kt = torch.tensor(np.asarray(K, np.float64).reshape(1, 3, 3), device=dv)
    pt = torch.tensor(p2, device=dv)
    off = torch.tensor([0, n], dtype=torch.int64, device=dv)
    res = ba_solve_batched(cam, Kt, X, pt, off, ftol, xtol, gtol, max_nfev)
    torch.cuda.synchronize()
    x = np.concatenate([cam.cpu().numpy().ravel(), X.cpu().numpy().ravel()])
    status = int(res["status"].item())
    return SimpleNamespace(x=x, cost=float(res["cost"].item()), fun=calculate_reprojection_error(x, K, p2),
                           nfev=int(res["nfev"].item()), njev=int(res["njev"].item()), status=status,
                           success=status > 0)
