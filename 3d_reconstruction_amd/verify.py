"""§8f row 2: geometric verification on the GPU, behind cv2's signatures.

* :func:`findEssentialMat` — ``cv2.findEssentialMat(p0, p1, K, method=cv2.RANSAC,
  prob=0.999, threshold=1)`` (matching.py:134, sfm.py:108).
* :func:`recoverPose` — ``cv2.recoverPose(E, p0, p1, K)`` (matching.py:139,
  sfm.py:117,119), distanceThresh 50.
* :func:`find_essential_batched` / :func:`recover_pose_batched` — the same over
  many image pairs in one launch (one workgroup per pair), device-resident.
* :func:`essential_inliers` — the matching.py:130-144 acceptance count
  (RANSAC inliers that also pass recoverPose's cheirality), usable as the
  ``verify`` callback of :func:`tracks.bfs_tracks`; :class:`EssentialVerifier`
  batches it over every candidate pair of the BoW connection graph.

Semantics follow OpenCV 4.x (restated in oracle/ransac.py; parity unpinned:
cv2 is not installed here).  Every call runs ``sfmhip_find_essential`` /
``sfmhip_recover_pose``; there is no CPU path.
"""
from __future__ import annotations

import numpy as np
import torch

from ._abi import call, dev, ptr, require_gpu, stream_ptr

RANSAC = 8          # cv2.RANSAC
MAX_MODELS = 10


def _cam(K) -> np.ndarray:
    K = np.asarray(K, np.float64).reshape(3, 3)
    return np.array([K[0, 0], K[1, 1], K[0, 2], K[1, 2]])

def _cam_rows(cam, P: int) -> torch.Tensor:
    """[fx, fy, cx, cy] per problem as a contiguous (P, 4) f64 device tensor.  A device tensor stays
    on the device (one row is broadcast there): no host round trip, so a batched call never waits
    for the work queued before it."""
    if isinstance(cam, torch.Tensor):
        t = dev(cam, torch.float64).reshape(-1, 4)
        if t.shape[0] not in (1, P):
            raise ValueError(f"camera rows must be 1 or {P}, got {t.shape[0]}")
        return (t.expand(P, 4) if t.shape[0] == 1 else t).contiguous()
    return dev(np.broadcast_to(np.asarray(cam, np.float64).reshape(-1, 4), (P, 4)).copy(), torch.float64)



def pack_pairs(pts0_list, pts1_list):
    """Lists of (n_p, 2) arrays -> (pts0 (N,2) f64 device, pts1, offsets (P+1,) int64 device)."""
    require_gpu()
    n = [len(np.asarray(a).reshape(-1, 2)) for a in pts0_list]
    offs = np.zeros(len(n) + 1, np.int64)
    offs[1:] = np.cumsum(n)
    cat = lambda L: np.concatenate([np.asarray(a, np.float64).reshape(-1, 2) for a in L]) if L else \
        np.zeros((0, 2))
    return dev(cat(pts0_list), torch.float64), dev(cat(pts1_list), torch.float64), dev(offs, torch.int64)


def find_essential_batched(pts0: torch.Tensor, pts1: torch.Tensor, offsets: torch.Tensor, cam,
                           prob: float = 0.999, threshold: float = 1.0, max_iters: int = 1000) -> dict:
    """Device tensors pts0/pts1 (N,2) f64, offsets (P+1,) int64, cam (P,4) or (4,)
    [fx, fy, cx, cy].  Returns device tensors E (P,10,9), n_models (P,),
    mask (N,) u8 0/1, n_inliers (P,), iters (P,)."""
    p0 = dev(pts0, torch.float64)
    p1 = dev(pts1, torch.float64)
    of = dev(offsets, torch.int64)
    P = of.numel() - 1
    N = p0.shape[0]
    c = _cam_rows(cam, P)
    d = p0.device
    out = dict(E=torch.zeros((P, MAX_MODELS, 9), dtype=torch.float64, device=d),
               n_models=torch.empty(P, dtype=torch.int32, device=d),
               mask=torch.empty(N, dtype=torch.uint8, device=d),
               n_inliers=torch.empty(P, dtype=torch.int32, device=d),
               iters=torch.empty(P, dtype=torch.int32, device=d))
    work = torch.empty((max(N, 1), 4), dtype=torch.float64, device=d)
    call("sfmhip_find_essential", ptr(p0), ptr(p1), ptr(of), P, ptr(c), float(prob), float(threshold),
         int(max_iters), ptr(work), ptr(out["E"]), ptr(out["n_models"]), ptr(out["mask"]), ptr(out["n_inliers"]),
         ptr(out["iters"]), stream_ptr())
    return out


def recover_pose_batched(E: torch.Tensor, pts0: torch.Tensor, pts1: torch.Tensor, offsets: torch.Tensor, cam,
                         mask: torch.Tensor | None = None, distance_thresh: float = 50.0) -> dict:
    """E (P,9) / (P,3,3) / (P,10,9) device f64 (model 0 used).  Returns R (P,3,3),
    t (P,3), mask (N,) u8 0/255, n_good (P,)."""
    p0 = dev(pts0, torch.float64)
    p1 = dev(pts1, torch.float64)
    of = dev(offsets, torch.int64)
    P = of.numel() - 1
    N = p0.shape[0]
    Et = dev(E, torch.float64).reshape(P, -1)
    c = _cam_rows(cam, P)
    mk = None if mask is None else dev(mask, torch.uint8)
    d = p0.device
    out = dict(R=torch.empty((P, 3, 3), dtype=torch.float64, device=d),
               t=torch.empty((P, 3), dtype=torch.float64, device=d),
               mask=torch.empty(N, dtype=torch.uint8, device=d),
               n_good=torch.empty(P, dtype=torch.int32, device=d))
    call("sfmhip_recover_pose", ptr(Et), Et.shape[1], ptr(p0), ptr(p1), ptr(of), P, ptr(c), ptr(mk),
         float(distance_thresh), ptr(out["R"]), ptr(out["t"]), ptr(out["mask"]), ptr(out["n_good"]),
         stream_ptr())
    return out


def findEssentialMat(points1, points2, cameraMatrix, method: int = RANSAC, prob: float = 0.999,
                     threshold: float = 1.0, maxIters: int = 1000, mask=None):
    """cv2.findEssentialMat (RANSAC) -> (E (3,3) f64, mask (n,1) u8) or (None, None)."""
    if method != RANSAC:
        raise NotImplementedError("only method=cv2.RANSAC (the reference's call) is implemented")
    p0 = np.asarray(points1, np.float64).reshape(-1, 2)
    p1 = np.asarray(points2, np.float64).reshape(-1, 2)
    if len(p0) != len(p1):
        raise ValueError("points1 and points2 must have the same number of points")
    a, b, of = pack_pairs([p0], [p1])
    r = find_essential_batched(a, b, of, _cam(cameraMatrix), prob, threshold, maxIters)
    nm = int(r["n_models"][0])
    if nm == 0:
        return None, None
    E = r["E"][0, :nm].cpu().numpy().reshape(3 * nm, 3)
    return E, r["mask"].cpu().numpy().reshape(-1, 1)


def recoverPose(E, points1, points2, cameraMatrix, R=None, t=None, mask=None, distanceThresh: float = 50.0):
    """cv2.recoverPose(E, p1, p2, K[, R, t, mask]) -> (retval, R (3,3), t (3,1), mask (n,1) u8 0/255)."""
    p0 = np.asarray(points1, np.float64).reshape(-1, 2)
    p1 = np.asarray(points2, np.float64).reshape(-1, 2)
    a, b, of = pack_pairs([p0], [p1])
    Ed = np.asarray(E, np.float64).reshape(-1, 3)[:3].reshape(1, 9)
    mk = None if mask is None else (np.asarray(mask).ravel() > 0).astype(np.uint8)
    r = recover_pose_batched(Ed, a, b, of, _cam(cameraMatrix), mk, distanceThresh)
    return (int(r["n_good"][0]), r["R"][0].cpu().numpy(), r["t"][0].cpu().numpy().reshape(3, 1),
            r["mask"].cpu().numpy().reshape(-1, 1))


def essential_inliers_batched(pts0_list, pts1_list, K, prob: float = 0.999, threshold: float = 1.0):
    """matching.py:134-144 for many pairs at once: per pair the number of
    points kept by findEssentialMat's mask AND recoverPose's cheirality mask
    on those inliers, or -1 where findEssentialMat returns no model."""
    a, b, of = pack_pairs(pts0_list, pts1_list)
    cam = _cam(K)
    r = find_essential_batched(a, b, of, cam, prob, threshold)
    rp = recover_pose_batched(r["E"], a, b, of, cam, mask=r["mask"])
    good = rp["n_good"].cpu().numpy().astype(np.int64)
    good[r["n_models"].cpu().numpy() == 0] = -1
    return good


def essential_inliers(pts0, pts1, K, prob: float = 0.999, threshold: float = 1.0):
    return int(essential_inliers_batched([pts0], [pts1], K, prob, threshold)[0])


class EssentialVerifier:
    """The ``verify`` callback of :func:`tracks.bfs_tracks` (matching.py:130-144):
    findEssentialMat RANSAC + recoverPose on the matched keypoints, returning
    the surviving count or None (no model).  Speculative batching: every
    ordered pair the BFS can examine — (u, v) with v in connection[u] or u in
    connection[v] — is verified up front in ONE batched launch (one workgroup
    per pair), so the sequential BFS only reads a table."""

    def __init__(self, connection, match_fn, all_points, K, prob: float = 0.999, threshold: float = 1.0):
        self.match_fn, self.points, self.K = match_fn, all_points, np.asarray(K, np.float64)
        self.prob, self.threshold = prob, threshold
        cand = sorted({(u, int(v)) for u in range(len(connection)) for v in connection[u]} |
                      {(int(v), u) for u in range(len(connection)) for v in connection[u]})
        cand = [(u, v) for u, v in cand if u != v]
        p0, p1 = [], []
        for r, i in cand:
            a, b = self._pts(r, i)
            p0.append(a)
            p1.append(b)
        counts = essential_inliers_batched(p0, p1, self.K, prob, threshold) if cand else []
        self.table = {c: int(n) for c, n in zip(cand, counts)}

    def _pts(self, r, i):
        idx0, idx1 = self.match_fn(r, i)
        return (np.asarray(self.points[r])[idx0].astype(np.float32),
                np.asarray(self.points[i])[idx1].astype(np.float32))

    def __call__(self, ref, nid, idx0, idx1):
        n = self.table.get((int(ref), int(nid)))
        if n is None:
            a = np.asarray(self.points[ref])[idx0].astype(np.float32)
            b = np.asarray(self.points[nid])[idx1].astype(np.float32)
            n = essential_inliers(a, b, self.K, self.prob, self.threshold)
        return None if n < 0 else n


SOLVEPNP_ITERATIVE = 0   # cv2.SOLVEPNP_ITERATIVE


def pnp_ransac_batched(obj: torch.Tensor, img: torch.Tensor, offsets: torch.Tensor, cam, iterations: int = 100,
                       reprojection_error: float = 8.0, confidence: float = 0.99) -> dict:
    """Device (N,3) / (N,2) f64 correspondences, offsets (P+1,) int64, cam (P,4) or (4,).
    Returns device rvec (P,3), tvec (P,3), mask (N,) u8, n_inliers, iters, ok (P,)."""
    X = dev(obj, torch.float64)
    u = dev(img, torch.float64)
    of = dev(offsets, torch.int64)
    P = of.numel() - 1
    N = X.shape[0]
    c = _cam_rows(cam, P)
    d = X.device
    out = dict(rvec=torch.empty((P, 3), dtype=torch.float64, device=d),
               tvec=torch.empty((P, 3), dtype=torch.float64, device=d),
               mask=torch.empty(N, dtype=torch.uint8, device=d),
               n_inliers=torch.empty(P, dtype=torch.int32, device=d),
               iters=torch.empty(P, dtype=torch.int32, device=d),
               ok=torch.empty(P, dtype=torch.int32, device=d))
    work = torch.empty((max(N, 1), 5), dtype=torch.float32, device=d)
    call("sfmhip_pnp_ransac", ptr(X), ptr(u), ptr(of), P, ptr(c), int(iterations), float(reprojection_error),
         float(confidence), ptr(work), ptr(out["rvec"]), ptr(out["tvec"]), ptr(out["mask"]), ptr(out["n_inliers"]),
         ptr(out["iters"]), ptr(out["ok"]), stream_ptr())
    return out


def solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs=None, rvec=None, tvec=None,
                   useExtrinsicGuess: bool = False, iterationsCount: int = 100, reprojectionError: float = 8.0,
                   confidence: float = 0.99, inliers=None, flags: int = SOLVEPNP_ITERATIVE):
    """cv2.solvePnPRansac (sfm.py:116) -> (retval, rvec (3,1), tvec (3,1), inliers (k,1) int32).
    ``rvec``/``tvec`` are outputs only (the reference passes SOLVEPNP_ITERATIVE
    positionally as rvec); distortion must be absent or zero."""
    if distCoeffs is not None and np.any(np.asarray(distCoeffs) != 0):
        raise NotImplementedError("non-zero distortion is not part of the reference's call")
    if useExtrinsicGuess:
        raise NotImplementedError("useExtrinsicGuess=True is not part of the reference's call")
    if flags != SOLVEPNP_ITERATIVE:
        raise NotImplementedError("only SOLVEPNP_ITERATIVE (the reference's call) is implemented")
    X = np.asarray(objectPoints, np.float64).reshape(-1, 3)
    m = np.asarray(imagePoints, np.float64).reshape(-1, 2)
    if len(X) != len(m):
        raise ValueError("objectPoints and imagePoints must have the same number of points")
    if len(X) < 5:
        raise NotImplementedError("fewer than 5 points (OpenCV switches to P3P at 4)")
    require_gpu()
    offs = torch.tensor([0, len(X)], dtype=torch.int64)
    r = pnp_ransac_batched(X, m, offs, _cam(cameraMatrix), iterationsCount, reprojectionError, confidence)
    if not int(r["ok"][0]):
        return False, None, None, None
    inl = np.nonzero(r["mask"].cpu().numpy())[0].astype(np.int32).reshape(-1, 1)
    return True, r["rvec"][0].cpu().numpy().reshape(3, 1), r["tvec"][0].cpu().numpy().reshape(3, 1), inl
