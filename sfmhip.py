"""``sfmhip`` -- importable alias of the ``3d_reconstruction_amd`` package.

The package directory name is not a Python identifier, so the reference's
stage scripts cannot ``import`` it directly.  With the repository root on
``sys.path`` this module IS the package (``sys.modules['sfmhip']`` is replaced
by it), so the reference binds by changing one import line:

* sfm.py:2       ``import cv2``  ->  ``import sfmhip as cv2``
  (triangulatePoints, convertPointsFromHomogeneous, Rodrigues, projectPoints,
  findEssentialMat, RANSAC, solvePnPRansac, SOLVEPNP_ITERATIVE, recoverPose)
* matching.py:11 ``import cv2``  ->  ``import sfmhip as cv2``
  (findEssentialMat, RANSAC, recoverPose); matching.py:20
  ``LightGlue(features='disk')`` -> ``sfmhip.Matcher(features='disk')``
* matching.py:27 / bow.py:23 ``from scipy.cluster.vq import vq, kmeans``
  -> ``from sfmhip import vq, kmeans``

See INTEGRATION.md for the full call-site map.
"""
import importlib
import sys

_pkg = importlib.import_module("3d_reconstruction_amd")
sys.modules[__name__] = _pkg
