"""sfmhip — MI355X-native (gfx950) backend for the dense-compute path of
daovietanh190499/3D_Reconstruction: BF-L2 descriptor matching + ratio test,
DLT triangulation, reprojection residual / FD Jacobian, voxel-grid work.

The directory name is not a Python identifier; import it as ``sfmhip`` (the
alias module ``sfmhip.py`` at the repository root) or with
``importlib.import_module("3d_reconstruction_amd")``.
The cv2 names sfm.py / matching.py use (RANSAC, SOLVEPNP_ITERATIVE and the
functions) are top-level, so ``import sfmhip as cv2`` binds them.
Every compute entry point runs a HIP kernel from ``libsfmhip.so``; there is no
CPU fallback.
"""
from ._abi import LIB_PATH, SfmHipError, knobs_reload, lib, require_gpu  # noqa: F401  (fails loudly if the .so is missing)
from .match import (MODE_FLOAT, MODE_SIFT, DescriptorBank, Matcher, all_pairs,  # noqa: F401
                    bf_match, vq)
from .geometry import (Rodrigues, ba_sparse, calculate_reprojection_error,  # noqa: F401
                       convertPointsFromHomogeneous, fd_jacobian, projectPoints,
                       residual_jacobian_batched, triangulatePoints, triangulate_batched, ba_solve_batched,
                       least_squares_ba)
from .voxel import (MASK_PLENOXEL, MASK_SDF, VoxelGrid, tsdf_block_table, tsdf_cull_stats, tsdf_integrate,  # noqa: F401,E501
                    tsdf_layer_cost, tsdf_layer_stats, voxel_traversal)
from . import bow, pipeline, reconstruct, tracks, verify  # noqa: F401,E402
from .bow import kmeans  # noqa: F401
from .reconstruct import triangulate  # noqa: F401
from .tracks import MatchGraph, bfs_tracks  # noqa: F401
from .verify import RANSAC, SOLVEPNP_ITERATIVE, findEssentialMat, recoverPose, solvePnPRansac  # noqa: F401
from .dist import RcclComm, match_all_pairs_sharded  # noqa: F401

__version__ = "0.1.0"
