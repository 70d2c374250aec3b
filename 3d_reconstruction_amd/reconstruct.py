"""S1: sfm.py's per-pair ``triangulate`` (sfm.py:26-52) on the sfmhip kernels:
GPU DLT, then the two-view bundle adjustment of camera j + the new points with
scipy ``least_squares`` driving the GPU residual and the GPU grouped-FD
Jacobian (``jac=fd_jacobian`` gives the values ``jac_sparsity=ba_sparse``
would).  Same arguments and the same in-place updates of the stage's state
(``cameras``, ``all_point3ds``) as the reference, which keeps them global.
"""
from __future__ import annotations

import numpy as np
from scipy.optimize import least_squares

from .geometry import (Rodrigues, calculate_reprojection_error, convertPointsFromHomogeneous, fd_jacobian,
                       triangulatePoints)


def triangulate(i, j, pts0, pts1, idx0, idx1, idx3d, K, cameras, all_point3ds, all_colors):
    """sfm.py:26-52.  Returns the focal length (K[0][0]) like the reference."""
    X4 = triangulatePoints(np.matmul(K, cameras[i]), np.matmul(K, cameras[j]), pts0.T, pts1.T)
    X4 = X4 / X4[3]
    new_pts = convertPointsFromHomogeneous(X4.T)[:, 0, :]
    for w, track in enumerate(idx3d):       # later duplicates overwrite earlier ones, as in the reference
        all_point3ds[0][track] = new_pts[w]
        all_point3ds[1][track] = all_colors[i][idx0[w]]
    rvec = Rodrigues(cameras[j][:3, :3])[0].ravel()
    x0 = np.hstack((rvec, cameras[j][:3, 3].ravel(), np.stack([all_point3ds[0][t] for t in idx3d]).ravel()))
    res = least_squares(calculate_reprojection_error, x0, jac=fd_jacobian, x_scale="jac", ftol=1e-8,
                        args=(K, pts1))
    R = Rodrigues(res.x[:3])[0]
    t = res.x[3:6]
    refined = res.x[6:].reshape(len(idx3d), 3)
    for w, track in enumerate(idx3d):
        all_point3ds[0][track] = refined[w]
    cameras[j] = np.hstack((R, t.reshape((3, 1))))
    return K[0][0]
