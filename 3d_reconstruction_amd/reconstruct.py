"""S1: sfm.py's per-pair ``triangulate`` (sfm.py:26-52) and its incremental
loop (sfm.py:101-131, ``incremental_sfm``) on the sfmhip kernels.

``triangulate`` (sfm.py:26-52):
GPU DLT, then the two-view bundle adjustment of camera j + the new points with
scipy ``least_squares`` driving the GPU residual and the GPU grouped-FD
Jacobian (``jac=fd_jacobian`` gives the values ``jac_sparsity=ba_sparse``
would).  Same arguments and the same in-place updates of the stage's state
(``cameras``, ``all_point3ds``) as the reference, which keeps them global.
"""
from __future__ import annotations

import numpy as np
from scipy.optimize import least_squares

from .geometry import (Rodrigues, calculate_reprojection_error, convertPointsFromHomogeneous, fd_jacobian, least_squares_ba,
                       triangulatePoints)
from . import verify as _verify

FOCAL = 2378.98305085   # sfm.py:24


def triangulate(i, j, pts0, pts1, idx0, idx1, idx3d, K, cameras, all_point3ds, all_colors, solver: str = "host"):
    """sfm.py:26-52.  Returns the focal length (K[0][0]) like the reference.

    ``solver`` for the BA of sfm.py:38: "host" = scipy's least_squares driving
    the GPU residual and FD Jacobian (the reference's iteration, one device
    round trip per evaluation); "device" = the whole TRF solve on the GPU
    (geometry.least_squares_ba: one launch, the same algorithm restated)."""
    X4 = triangulatePoints(np.matmul(K, cameras[i]), np.matmul(K, cameras[j]), pts0.T, pts1.T)
    X4 = X4 / X4[3]
    new_pts = convertPointsFromHomogeneous(X4.T)[:, 0, :]
    for w, track in enumerate(idx3d):       # later duplicates overwrite earlier ones, as in the reference
        all_point3ds[0][track] = new_pts[w]
        all_point3ds[1][track] = all_colors[i][idx0[w]]
    rvec = Rodrigues(cameras[j][:3, :3])[0].ravel()
    x0 = np.hstack((rvec, cameras[j][:3, 3].ravel(), np.stack([all_point3ds[0][t] for t in idx3d]).ravel()))
    if solver == "device":
        res = least_squares_ba(x0, K, pts1, ftol=1e-8)
    elif solver == "host":
        res = least_squares(calculate_reprojection_error, x0, jac=fd_jacobian, x_scale="jac", ftol=1e-8,
                            args=(K, pts1))
    else:
        raise ValueError(f"solver must be 'host' or 'device', got {solver!r}")
    R = Rodrigues(res.x[:3])[0]
    t = res.x[3:6]
    refined = res.x[6:].reshape(len(idx3d), 3)
    for w, track in enumerate(idx3d):
        all_point3ds[0][track] = refined[w]
    cameras[j] = np.hstack((R, t.reshape((3, 1))))
    return K[0][0]


class GpuOps:
    """The cv2 / scipy calls of sfm.py:101-131, on the sfmhip kernels."""
    findEssentialMat = staticmethod(_verify.findEssentialMat)
    recoverPose = staticmethod(_verify.recoverPose)
    solvePnPRansac = staticmethod(_verify.solvePnPRansac)
    Rodrigues = staticmethod(Rodrigues)
    triangulate = staticmethod(triangulate)


def incremental_sfm(img_pairs, all_matches, all_points, all_colors, n_images: int, focal: float = FOCAL,
                    ops=GpuOps):
    """sfm.py:101-131 -> (cameras list (None for unregistered), all_point3ds [points, colors]).

    Per pair (i, j) in BFS order: findEssentialMat RANSAC on the matched
    keypoints, keep its inliers; register camera j from recoverPose (first
    pair) or solvePnPRansac on the already-triangulated tracks; triangulate +
    bundle-adjust the new tracks that pass recoverPose's cheirality."""
    n_tracks = int(np.max(np.hstack([m[2] for m in all_matches]))) + 1
    all_point3ds = [[None] * n_tracks, [None] * n_tracks]
    cameras = [None] * n_images
    for index, (i, j) in enumerate(img_pairs):
        idx0, idx1, idx3d = (np.asarray(a) for a in all_matches[index])
        pts0 = np.asarray(all_points[i])[idx0].astype("float64")
        pts1 = np.asarray(all_points[j])[idx1].astype("float64")
        point3ds = np.array(all_point3ds[0], dtype=object)[idx3d]
        K = np.array([[focal, 0, 0], [0, focal, 0], [0, 0, 1]])
        E, mask = ops.findEssentialMat(pts0, pts1, K, _verify.RANSAC, 0.999, 1)
        keep = mask.ravel() == 1
        idx0, idx1, idx3d = idx0[keep], idx1[keep], idx3d[keep]
        pts0, pts1, point3ds = pts0[keep], pts1[keep], point3ds[keep]
        mask_ = np.array([pt is None for pt in point3ds])
        if index != 0:
            _, rvecs, t, _ = ops.solvePnPRansac(np.stack(point3ds[mask_ == 0]), pts1[mask_ == 0], K,
                                                np.zeros((5, 1), dtype=np.float32), 0)
            R, _ = ops.Rodrigues(rvecs)
            _, _, _, mask_inliers = ops.recoverPose(E, pts0, pts1, K)
        else:
            _, R, t, mask_inliers = ops.recoverPose(E, pts0, pts1, K)
        mask_ = mask_ * (mask_inliers.ravel() > 0)
        cameras[j] = np.hstack((R, np.asarray(t).reshape(3, 1)))
        if cameras[i] is None:
            cameras[i] = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0]])
        if np.sum(mask_) > 0:
            sel = mask_ == 1
            focal = ops.triangulate(i, j, pts0[sel], pts1[sel], idx0[sel], idx1[sel], idx3d[sel], K, cameras,
                                    all_point3ds, all_colors)
    return cameras, all_point3ds


def save_sfm_outputs(out_dir: str, img_list, cameras, all_point3ds) -> None:
    """sfm.py:133-146 formats: reconstructed_img.txt, cameras_extrinsic.npy, points_3d.npy."""
    import os
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "reconstructed_img.txt"), "wt") as fh:
        for name, cam in zip(img_list, cameras):
            if cam is not None:
                fh.write(name + "\n")
    np.save(os.path.join(out_dir, "cameras_extrinsic.npy"), np.array([c for c in cameras if c is not None]))
    pts = np.array(all_point3ds[0], dtype=object)
    have = np.array([p is not None for p in pts])
    np.save(os.path.join(out_dir, "points_3d.npy"), np.stack(pts[have]).astype(float))
