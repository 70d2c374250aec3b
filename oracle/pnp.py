"""Oracle for solvePnPRansac (sfm.py:116, §8f row 2).  TEST INFRASTRUCTURE ONLY.

    ret, rvecs, t, _ = cv2.solvePnPRansac(X, pts1, K, np.zeros((5, 1)), cv2.SOLVEPNP_ITERATIVE)

(the 5th positional argument is ``rvec``, so the call runs with the defaults:
iterationsCount 100, reprojectionError 8, confidence 0.99, flags ITERATIVE).
OpenCV 4.x (calib3d/src/solvepnp.cpp, epnp.cpp, ptsetreg.cpp, calibration.cpp
cvFindExtrinsicCameraParams2 + CvLevMarq) is absent here, so this restates its
published algorithm — **parity unpinned**; tests pin it with known answers:

* points are converted to float32 (solvePnPRansac converts f64 inputs);
* RANSAC (oracle.ransac.ransac: cv::RNG(-1), 5-point samples, a model wins
  iff count > max(best, 4), RANSACUpdateNumIters) whose kernel is EPnP on the
  sample and whose error is the float squared reprojection distance <= 64;
* EPnP (Lepetit et al.; epnp.cpp structure): PCA control points, barycentric
  alphas, M^T M eigenvectors of the 4 smallest eigenvalues, L_6x10 / rho,
  the three beta approximations + 5 Gauss-Newton steps each, Procrustes, the
  best mean reprojection error; build-defined: eigenvector signs are made
  canonical (largest-|.| component positive; cvSVD's signs are
  implementation-defined);
* refinement on the inliers: cvFindExtrinsicCameraParams2 with the RANSAC
  pose as guess = CvLevMarq (lambda 10^-3, x10 on a worse error, /10 on
  accept, 20 iterations, relative step < FLT_EPSILON) on the reprojection
  residual with cvProjectPoints2's analytic Jacobian.
"""
from __future__ import annotations

import math

import numpy as np

from .geometry import project_points, rodrigues, rodrigues_inverse
from .ransac import ransac

F32 = np.float32
FLT_EPSILON = float(np.finfo(np.float32).eps)


def canon(v: np.ndarray) -> np.ndarray:
    i = int(np.argmax(np.abs(v)))
    return v if v[i] >= 0 else -v


def eig_desc(A: np.ndarray):
    """Symmetric eigen-decomposition, eigenvalues descending, rows = canonical eigenvectors."""
    w, V = np.linalg.eigh(A)
    order = np.argsort(-w, kind="stable")
    return w[order], np.array([canon(V[:, k]) for k in order])


class EPnP:
    def __init__(self, K, X, uv):
        K = np.asarray(K, np.float64)
        self.fu, self.fv, self.uc, self.vc = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
        self.pws = np.asarray(X, np.float64).reshape(-1, 3)
        self.us = np.asarray(uv, np.float64).reshape(-1, 2)
        self.n = len(self.pws)

    def control_points(self):
        c0 = self.pws.sum(0) / self.n
        P = self.pws - c0
        dc, uct = eig_desc(P.T @ P)
        cws = [c0] + [c0 + math.sqrt(max(dc[i], 0.0) / self.n) * uct[i] for i in range(3)]
        return np.array(cws)

    def alphas(self, cws):
        CC = np.stack([cws[j] - cws[0] for j in (1, 2, 3)], 1)          # cc[i][j-1] = cws[j][i] - cws[0][i]
        ci = np.linalg.inv(CC)
        a = (self.pws - cws[0]) @ ci.T
        return np.column_stack([1.0 - a[:, 0] - a[:, 1] - a[:, 2], a])

    def M(self, al):
        M = np.zeros((2 * self.n, 12))
        for i in range(4):
            M[0::2, 3 * i] = al[:, i] * self.fu
            M[0::2, 3 * i + 2] = al[:, i] * (self.uc - self.us[:, 0])
            M[1::2, 3 * i + 1] = al[:, i] * self.fv
            M[1::2, 3 * i + 2] = al[:, i] * (self.vc - self.us[:, 1])
        return M

    @staticmethod
    def L_6x10(v):
        pairs = [(a, b) for a in range(4) for b in range(a + 1, 4)]
        dv = np.array([[v[i][3 * a:3 * a + 3] - v[i][3 * b:3 * b + 3] for (a, b) in pairs] for i in range(4)])
        L = np.empty((6, 10))
        for r in range(6):
            d = dv[:, r]
            L[r] = [d[0] @ d[0], 2 * d[0] @ d[1], d[1] @ d[1], 2 * d[0] @ d[2], 2 * d[1] @ d[2], d[2] @ d[2],
                    2 * d[0] @ d[3], 2 * d[1] @ d[3], 2 * d[2] @ d[3], d[3] @ d[3]]
        return L

    @staticmethod
    def rho(cws):
        pairs = [(a, b) for a in range(4) for b in range(a + 1, 4)]
        return np.array([np.sum((cws[a] - cws[b]) ** 2) for (a, b) in pairs])

    @staticmethod
    def betas_1(L, rho):
        b4 = np.linalg.lstsq(L[:, [0, 1, 3, 6]], rho, rcond=None)[0]
        if b4[0] < 0:
            b0 = math.sqrt(-b4[0])
            return np.array([b0, -b4[1] / b0, -b4[2] / b0, -b4[3] / b0])
        b0 = math.sqrt(b4[0])
        return np.array([b0, b4[1] / b0, b4[2] / b0, b4[3] / b0])

    @staticmethod
    def betas_2(L, rho):
        b3 = np.linalg.lstsq(L[:, [0, 1, 2]], rho, rcond=None)[0]
        if b3[0] < 0:
            b = [math.sqrt(-b3[0]), math.sqrt(-b3[2]) if b3[2] < 0 else 0.0]
        else:
            b = [math.sqrt(b3[0]), math.sqrt(b3[2]) if b3[2] > 0 else 0.0]
        if b3[1] < 0:
            b[0] = -b[0]
        return np.array([b[0], b[1], 0.0, 0.0])

    @staticmethod
    def betas_3(L, rho):
        b5 = np.linalg.lstsq(L[:, [0, 1, 2, 3, 4]], rho, rcond=None)[0]
        if b5[0] < 0:
            b = [math.sqrt(-b5[0]), math.sqrt(-b5[2]) if b5[2] < 0 else 0.0]
        else:
            b = [math.sqrt(b5[0]), math.sqrt(b5[2]) if b5[2] > 0 else 0.0]
        if b5[1] < 0:
            b[0] = -b[0]
        return np.array([b[0], b[1], b5[3] / b[0], 0.0])

    @staticmethod
    def gauss_newton(L, rho, betas):
        b = betas.copy()
        for _ in range(5):
            A = np.empty((6, 4))
            r = np.empty(6)
            for i in range(6):
                l = L[i]
                A[i] = [2 * l[0] * b[0] + l[1] * b[1] + l[3] * b[2] + l[6] * b[3],
                        l[1] * b[0] + 2 * l[2] * b[1] + l[4] * b[2] + l[7] * b[3],
                        l[3] * b[0] + l[4] * b[1] + 2 * l[5] * b[2] + l[8] * b[3],
                        l[6] * b[0] + l[7] * b[1] + l[8] * b[2] + 2 * l[9] * b[3]]
                r[i] = rho[i] - (l[0] * b[0] * b[0] + l[1] * b[0] * b[1] + l[2] * b[1] * b[1] + l[3] * b[0] * b[2]
                                 + l[4] * b[1] * b[2] + l[5] * b[2] * b[2] + l[6] * b[0] * b[3]
                                 + l[7] * b[1] * b[3] + l[8] * b[2] * b[3] + l[9] * b[3] * b[3])
            b = b + np.linalg.lstsq(A, r, rcond=None)[0]
        return b

    def R_and_t(self, v, betas, al):
        ccs = sum(betas[i] * v[i] for i in range(4)).reshape(4, 3)
        pcs = al @ ccs
        if pcs[0, 2] < 0:
            ccs, pcs = -ccs, -pcs
        pc0 = pcs.sum(0) / self.n
        pw0 = self.pws.sum(0) / self.n
        ABt = (pcs - pc0).T @ (self.pws - pw0)
        U, _, Vt = np.linalg.svd(ABt)
        R = U @ Vt
        if np.linalg.det(R) < 0:
            R[2] = -R[2]
        t = pc0 - R @ pw0
        Xc = self.pws @ R.T + t
        ue = self.uc + self.fu * Xc[:, 0] / Xc[:, 2]
        ve = self.vc + self.fv * Xc[:, 1] / Xc[:, 2]
        err = np.mean(np.sqrt((self.us[:, 0] - ue) ** 2 + (self.us[:, 1] - ve) ** 2))
        return R, t, err

    def compute_pose(self):
        cws = self.control_points()
        al = self.alphas(cws)
        M = self.M(al)
        _, ut = eig_desc(M.T @ M)
        v = [ut[11 - i] for i in range(4)]
        L, rho = self.L_6x10(v), self.rho(cws)
        sols = [self.R_and_t(v, self.gauss_newton(L, rho, f(L, rho)), al)
                for f in (self.betas_1, self.betas_2, self.betas_3)]
        N = 0
        if sols[1][2] < sols[0][2]:
            N = 1
        if sols[2][2] < sols[N][2]:
            N = 2
        return sols[N][0], sols[N][1]


def rodrigues_jacobian(rvec):
    """cv::Rodrigues vector->matrix Jacobian (3,9): J[i*9+k] = dR_k / dr_i."""
    r = np.asarray(rvec, np.float64).ravel()
    theta = math.sqrt(r @ r)
    if theta < np.finfo(np.float64).eps:
        J = np.zeros((3, 9))
        J[0, 5], J[0, 7] = -1, 1
        J[1, 2], J[1, 6] = 1, -1
        J[2, 1], J[2, 3] = -1, 1
        return J
    c, s = math.cos(theta), math.sin(theta)
    c1, itheta = 1 - c, 1 / theta
    rx, ry, rz = r * itheta
    I = np.eye(3).ravel()
    rrt = np.array([rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz])
    rxm = np.array([0, -rz, ry, rz, 0, -rx, -ry, rx, 0])
    drrt = np.array([[rx + rx, ry, rz, ry, 0, 0, rz, 0, 0],
                     [0, rx, 0, rx, ry + ry, rz, 0, rz, 0],
                     [0, 0, rx, 0, 0, ry, rx, ry, rz + rz]])
    drx = np.array([[0, 0, 0, 0, 0, -1, 0, 1, 0], [0, 0, 1, 0, 0, 0, -1, 0, 0], [0, -1, 0, 1, 0, 0, 0, 0, 0]])
    J = np.empty((3, 9))
    for i, ri in enumerate((rx, ry, rz)):
        a0, a1, a2 = -s * ri, (s - 2 * c1 * itheta) * ri, c1 * itheta
        a3, a4 = (c - s * itheta) * ri, s * itheta
        J[i] = a0 * I + a1 * rrt + a2 * drrt[i] + a3 * rxm + a4 * drx[i]
    return J


def project_with_jacobian(X, param, K):
    """cvProjectPoints2 (zero distortion) -> (proj (n,2), J (2n,6) = [dp/drvec, dp/dt])."""
    R = rodrigues(param[:3])
    dR = rodrigues_jacobian(param[:3])
    t = param[3:]
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    Xc = X @ R.T + t
    z = 1.0 / Xc[:, 2]
    x, y = Xc[:, 0] * z, Xc[:, 1] * z
    proj = np.stack([x * fx + cx, y * fy + cy], 1)
    J = np.zeros((2 * len(X), 6))
    for j in range(3):
        dx0 = X @ dR[j, 0:3]
        dy0 = X @ dR[j, 3:6]
        dz0 = X @ dR[j, 6:9]
        J[0::2, j] = fx * (z * (dx0 - x * dz0))
        J[1::2, j] = fy * (z * (dy0 - y * dz0))
    J[0::2, 3], J[0::2, 5] = fx * z, fx * (-x * z)
    J[1::2, 4], J[1::2, 5] = fy * z, fy * (-y * z)
    return proj, J


def lm_refine(X, m, K, rvec, tvec, max_iter: int = 20, eps: float = FLT_EPSILON):
    """cvFindExtrinsicCameraParams2(useExtrinsicGuess=1): the CvLevMarq state machine."""
    X = np.asarray(X, np.float64).reshape(-1, 3)
    m = np.asarray(m, np.float64).reshape(-1, 2)
    K = np.asarray(K, np.float64)
    param = np.concatenate([np.ravel(rvec), np.ravel(tvec)]).astype(np.float64)
    lam = -3
    iters = 0
    prev_err = np.finfo(np.float64).max

    def step(JtJ, JtErr, prev, lam):
        A = JtJ.copy()
        A[np.diag_indices(6)] *= 1.0 + math.exp(lam * math.log(10.0))
        return prev - np.linalg.lstsq(A, JtErr, rcond=None)[0]

    proj, J = project_with_jacobian(X, param, K)
    err = (proj - m).ravel()
    while True:
        JtJ, JtErr, prev = J.T @ J, J.T @ err, param.copy()
        param = step(JtJ, JtErr, prev, lam)
        if iters == 0:
            prev_err = np.linalg.norm(err)
        while True:
            err = (project_with_jacobian(X, param, K)[0] - m).ravel()
            err_norm = np.linalg.norm(err)
            if err_norm > prev_err:
                lam += 1
                if lam <= 16:
                    param = step(JtJ, JtErr, prev, lam)
                    continue
            break
        lam = max(lam - 1, -16)
        iters += 1
        if iters >= max_iter or np.linalg.norm(param - prev) < eps * np.linalg.norm(prev):
            return param[:3].reshape(3, 1), param[3:].reshape(3, 1)
        prev_err = err_norm
        proj, J = project_with_jacobian(X, param, K)
        err = (proj - m).ravel()


def solve_pnp_ransac(object_points, image_points, K, iterations: int = 100, reprojection_error: float = 8.0,
                     confidence: float = 0.99, return_iters: bool = False):
    """cv2.solvePnPRansac (ITERATIVE, no distortion) -> (ok, rvec (3,1), tvec (3,1), inliers (k,1) int32)."""
    K = np.asarray(K, np.float64)
    op = np.asarray(object_points, np.float64).reshape(-1, 3).astype(F32)
    ip = np.asarray(image_points, np.float64).reshape(-1, 2).astype(F32)
    n = len(op)
    if n < 5:
        raise NotImplementedError("n < 5 (OpenCV would switch to P3P at n == 4)")
    opd, ipd = op.astype(np.float64), ip.astype(np.float64)
    thr = F32(reprojection_error * reprojection_error)

    def kernel(idx):
        R, t = EPnP(K, opd[idx], ipd[idx]).compute_pose()
        return [(rodrigues_inverse(R).ravel(), t)]

    def score(model):
        proj = project_points(opd, model[0], model[1], K).astype(F32)
        d = ip - proj
        return (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) <= thr

    if n == 5:
        rv, t = kernel(list(range(5)))[0]
        res = (True, rv.reshape(3, 1), t.reshape(3, 1), np.arange(5, dtype=np.int32).reshape(-1, 1))
        return res + (1,) if return_iters else res
    model, mask, it = ransac(n, 5, kernel, score, reprojection_error, confidence, iterations)
    if model is None:
        res = (False, None, None, None)
        return res + (it,) if return_iters else res
    rv, t = lm_refine(opd[mask], ipd[mask], K, model[0], model[1])
    res = (True, rv, t, np.nonzero(mask)[0].astype(np.int32).reshape(-1, 1))
    return res + (it,) if return_iters else res
