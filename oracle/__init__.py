"""oracle — CPU restatement of the reference's hot-path algorithms.

TEST INFRASTRUCTURE ONLY.  Imported exclusively by ``tests/``,
``__graft_entry__.smoke()`` (as the checker) and ``bench.py``'s
``cpu_baseline`` leg.  The product package (``3d_reconstruction_amd``) never
imports, calls or links anything here; it fails loudly without its HIP library.

Each function cites the reference file:line it restates.  Pinning status
(DESIGN.md §Parity):

* match.bf_match        build-defined semantics (the reference has no BF
                         matcher); top-1 pinned against scipy.cluster.vq.vq
                         (what matching.py:27 calls) and the mutual rule against
                         the reference's lightglue filter_matches — golden
                         fixtures in tests/golden/.
* match.vq              IS scipy.cluster.vq.vq (the reference's own call).
* geometry.*            OpenCV restatements (cv2 is absent here and not
                         vendored): DLT / projectPoints / Rodrigues are
                         "parity unpinned" at the OpenCV boundary; the FD
                         Jacobian runs scipy's own approx_derivative.
* voxel.voxel_traversal pinned: golden fixtures from the reference file.
* voxel.grid_sample /
  sh_colour / composite pinned: golden fixtures from sdf.py / plenoxel.py.
* voxel.tsdf_integrate  build-defined, parity unpinned (no reference TSDF);
                         checked by analytic known answers.
"""
