"""Oracle for the on-device BA solve (sfm.py:37-38).  TEST INFRASTRUCTURE ONLY.

sfm.py:38 calls scipy's ``least_squares(calculate_reprojection_error, x,
jac_sparsity=ba_sparse(...), x_scale='jac', ftol=1e-8, args=(K, pts1))`` per
pair: method 'trf' with tr_solver 'lsmr' (a sparse Jacobian), jac '2-point'
with the ba_sparse column groups, xtol = gtol = 1e-8, max_nfev = 100 len(x).
This module restates that iteration (scipy 1.15 optimize/_lsq/trf.py
``trf_no_bounds`` and _lsq/common.py: compute_jac_scale, build_quadratic_1d,
minimize_quadratic_1d, solve_trust_region_2d, evaluate_quadratic,
update_tr_radius, check_termination) on the per-observation structure of the
BA Jacobian (2x6 camera block + 2x3 point block per observation), with one
deliberate difference: the Gauss-Newton direction ``lsmr(J_h, f, damp=mu)``
(an iterative solve stopped at scipy's default atol = btol = 1e-6) is the
EXACT damped least-squares solution J_h^T (J_h J_h^T + mu I)^-1 f, computed in
O(n) with the Woodbury identity over the block-diagonal point part.  Pinned
against scipy's least_squares itself in tests/test_oracle_ba.py (same nfev,
cost and parameters to the LSMR tolerance).
"""
from __future__ import annotations

import numpy as np

from . import geometry as og


def residual(cam, X, K, pts):
    """(n, 2) = pts - projectPoints(X, rvec, t, K) (sfm.py:87-91)."""
    return (np.asarray(pts, np.float64) - og.project_points(X, cam[:3], cam[3:6], K)).reshape(-1, 2)


def jacobian(cam, X, K, pts):
    """scipy's grouped 2-point FD values per observation: (n, 2, 9) = [camera 6 | point 3]."""
    x = np.concatenate([cam, np.asarray(X, np.float64).ravel()])
    return og.fd_jacobian_direct(x, K, pts)


class _Ops:
    """J_h = J diag(d) on the (camera, points) split."""

    def __init__(self, J, dc, dp):
        self.Jc = J[:, :, :6] * dc[None, None, :]
        self.Jp = J[:, :, 6:] * dp[:, None, :]

    def dot(self, sc, sp):          # J_h s -> (n, 2)
        return self.Jc @ sc + np.einsum("nij,nj->ni", self.Jp, sp)

    def tdot(self, y):              # J_h^T y -> (6,), (n, 3)
        return np.einsum("nij,ni->j", self.Jc, y), np.einsum("nij,ni->nj", self.Jp, y)

    def ridge(self, f, mu):
        """argmin |J_h p - f|^2 + mu |p|^2 = J_h^T (J_h J_h^T + mu I)^-1 f (Woodbury)."""
        B = np.einsum("nij,nkj->nik", self.Jp, self.Jp) + mu * np.eye(2)[None]
        Binv = np.linalg.inv(B)
        u = np.einsum("nij,nj->ni", Binv, f)
        Y = np.einsum("nij,njk->nik", Binv, self.Jc)
        G = np.eye(6) + np.einsum("nij,nik->jk", self.Jc, Y)
        h = np.einsum("nij,ni->j", self.Jc, u)
        z = np.linalg.solve(G, h)
        y = u - Y @ z
        return self.tdot(y)


def solve_trust_region_2d(B, g, Delta):
    """scipy _lsq/common.py solve_trust_region_2d."""
    try:
        L = np.linalg.cholesky(B)
        p = -np.linalg.solve(L.T, np.linalg.solve(L, g))
        if np.dot(p, p) <= Delta ** 2:
            return p
    except np.linalg.LinAlgError:
        pass
    a = B[0, 0] * Delta ** 2
    b = B[0, 1] * Delta ** 2
    c = B[1, 1] * Delta ** 2
    d = g[0] * Delta
    f = g[1] * Delta
    t = np.roots(np.array([-b + d, 2 * (a - c + f), 6 * b, 2 * (-a + c + f), -b - d]))
    t = np.real(t[np.isreal(t)])
    p = Delta * np.vstack((2 * t / (1 + t ** 2), (1 - t ** 2) / (1 + t ** 2)))
    value = 0.5 * np.sum(p * B.dot(p), axis=0) + np.dot(g, p)
    return p[:, np.argmin(value)]


def trf_ba(cam, X, K, pts, ftol=1e-8, xtol=1e-8, gtol=1e-8, max_nfev=None):
    """least_squares(calculate_reprojection_error, [cam, X], jac_sparsity=ba_sparse, x_scale='jac',
    ftol=ftol) restated (module docstring).  Returns dict(cam, X, cost, nfev, njev, status)."""
    cam = np.array(cam, np.float64)
    X = np.array(X, np.float64).reshape(-1, 3)
    n = len(X)
    nx = 6 + 3 * n
    f = residual(cam, X, K, pts)
    nfev, njev = 1, 1
    J = jacobian(cam, X, K, pts)
    cost = 0.5 * np.sum(f * f)

    def grad(J, f):
        return np.einsum("nij,ni->j", J[:, :, :6], f), np.einsum("nij,ni->nj", J[:, :, 6:], f)

    def col_norms(J):
        return np.sqrt(np.sum(J[:, :, :6] ** 2, axis=(0, 1))), np.sqrt(np.sum(J[:, :, 6:] ** 2, axis=1))

    gc, gp = grad(J, f)
    sic, sip = col_norms(J)
    sic[sic == 0] = 1
    sip[sip == 0] = 1
    Delta = np.sqrt(np.sum((cam * sic) ** 2) + np.sum((X * sip) ** 2))
    if Delta == 0:
        Delta = 1.0
    max_nfev = 100 * nx if max_nfev is None else max_nfev
    status = None
    while True:
        g_norm = max(np.abs(gc).max(), np.abs(gp).max())
        if g_norm < gtol:
            status = 1
        if status is not None or nfev == max_nfev:
            break
        dc, dp = 1 / sic, 1 / sip
        ghc, ghp = dc * gc, dp * gp
        ops = _Ops(J, dc, dp)
        # regularize: the 1-D quadratic along -g_h inside the trust region
        v = ops.dot(-ghc, -ghp)
        a = 0.5 * np.sum(v * v)
        gh2 = np.sum(ghc * ghc) + np.sum(ghp * ghp)
        b = -gh2
        to_tr = Delta / np.sqrt(gh2)
        ts = [0.0, to_tr]
        if a != 0:
            ext = -0.5 * b / a
            if 0 < ext < to_tr:
                ts.append(ext)
        ts = np.asarray(ts)
        ag_value = np.min(ts * (a * ts + b))
        mu = -ag_value / Delta ** 2
        gnc, gnp = ops.ridge(f, mu)
        # S = qr([g_h, gn_h]): Gram-Schmidt (the subspace, not the column signs, fixes the step)
        s1n = np.sqrt(gh2)
        s1c, s1p = ghc / s1n, ghp / s1n
        c12 = np.sum(s1c * gnc) + np.sum(s1p * gnp)
        s2c, s2p = gnc - c12 * s1c, gnp - c12 * s1p
        s2n = np.sqrt(np.sum(s2c * s2c) + np.sum(s2p * s2p))
        s2c, s2p = s2c / s2n, s2p / s2n
        JS1, JS2 = ops.dot(s1c, s1p), ops.dot(s2c, s2p)
        B_S = np.array([[np.sum(JS1 * JS1), np.sum(JS1 * JS2)], [np.sum(JS1 * JS2), np.sum(JS2 * JS2)]])
        g_S = np.array([np.sum(s1c * ghc) + np.sum(s1p * ghp), np.sum(s2c * ghc) + np.sum(s2p * ghp)])
        actual_reduction = -1
        while actual_reduction <= 0 and nfev < max_nfev:
            p_S = solve_trust_region_2d(B_S, g_S, Delta)
            shc, shp = p_S[0] * s1c + p_S[1] * s2c, p_S[0] * s1p + p_S[1] * s2p
            Js = ops.dot(shc, shp)
            predicted_reduction = -(0.5 * np.sum(Js * Js) + np.sum(shc * ghc) + np.sum(shp * ghp))
            stc, stp = dc * shc, dp * shp
            cam_new, X_new = cam + stc, X + stp
            f_new = residual(cam_new, X_new, K, pts)
            nfev += 1
            step_h_norm = np.sqrt(np.sum(shc * shc) + np.sum(shp * shp))
            if not np.all(np.isfinite(f_new)):
                Delta = 0.25 * step_h_norm
                continue
            cost_new = 0.5 * np.sum(f_new * f_new)
            actual_reduction = cost - cost_new
            # update_tr_radius
            if predicted_reduction > 0:
                ratio = actual_reduction / predicted_reduction
            elif predicted_reduction == actual_reduction == 0:
                ratio = 1
            else:
                ratio = 0
            Delta_new = Delta
            if ratio < 0.25:
                Delta_new = 0.25 * step_h_norm
            elif ratio > 0.75 and step_h_norm > 0.95 * Delta:
                Delta_new = Delta * 2.0
            step_norm = np.sqrt(np.sum(stc * stc) + np.sum(stp * stp))
            x_norm = np.sqrt(np.sum(cam * cam) + np.sum(X * X))
            ftol_ok = actual_reduction < ftol * cost and ratio > 0.25
            xtol_ok = step_norm < xtol * (xtol + x_norm)
            status = 4 if (ftol_ok and xtol_ok) else 2 if ftol_ok else 3 if xtol_ok else None
            if status is not None:
                break
            Delta = Delta_new
        if actual_reduction > 0:
            cam, X, f, cost = cam_new, X_new, f_new, cost_new
            J = jacobian(cam, X, K, pts)
            njev += 1
            gc, gp = grad(J, f)
            nc, npn = col_norms(J)
            sic, sip = np.maximum(nc, sic), np.maximum(npn, sip)
    return {"cam": cam, "X": X, "cost": cost, "nfev": nfev, "njev": njev, "status": 0 if status is None else status}
