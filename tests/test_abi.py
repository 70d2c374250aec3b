"""CPU: the C-ABI library loads and exports exactly what include/sfmhip.h declares.
No compute calls (no GPU here)."""
import ctypes
import os
import re

from conftest import ROOT


def header_decls():
    src = open(os.path.join(ROOT, "include", "sfmhip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    decls = {}
    for m in re.finditer(r"\b(?:int|const char\*)\s+(sfmhip_\w+)\s*\(([^;]*?)\)\s*;", src, flags=re.S):
        args = m.group(2).strip()
        n = 0 if args in ("", "void") else len([a for a in args.split(",") if a.strip()])
        decls[m.group(1)] = n
    return decls


def test_header_parses():
    d = header_decls()
    assert len(d) >= 17
    assert d["sfmhip_match_pairs"] == 15


def test_library_exports_every_declared_symbol(sfm):
    lib = ctypes.CDLL(sfm.LIB_PATH)
    for name in header_decls():
        assert hasattr(lib, name), name


def test_ctypes_signatures_match_header(sfm):
    from importlib import import_module
    abi = import_module("3d_reconstruction_amd._abi")
    decls = header_decls()
    assert set(abi.SIGNATURES) == set(decls)
    for name, n in decls.items():
        assert len(abi.SIGNATURES[name]) == n, name


def test_version_and_error_channel(sfm):
    assert sfm.lib.sfmhip_version() == 0x000300   # 0.3.0: the int16-graph match entry points
    # an argument error is reported without touching the GPU
    rc = sfm.lib.sfmhip_match_pairs(None, None, None, None, 1, 128, 128, None, 1, 3, 4, None, None, None, None)
    assert rc == -1
    assert b"null pointer" in sfm.lib.sfmhip_last_error()
    rc = sfm.lib.sfmhip_tsdf_integrate(1, 1, 4, 4, 4, 3, 2, 1, 1, 1, 1, 1, 1, 1, 1, ctypes.c_float(0.1), None)
    assert rc == -1 and b"z range" in sfm.lib.sfmhip_last_error()


def test_sfmhip_alias_and_cv2_names(sfm):
    """`import sfmhip as cv2` binds what sfm.py / matching.py call (one import line)."""
    import sfmhip
    assert sfmhip is sfm
    assert sfmhip.RANSAC == 8 and sfmhip.SOLVEPNP_ITERATIVE == 0
    for name in ("triangulatePoints", "convertPointsFromHomogeneous", "Rodrigues", "projectPoints",
                 "findEssentialMat", "recoverPose", "solvePnPRansac", "Matcher", "vq", "kmeans",
                 "match_all_pairs_sharded", "RcclComm"):
        assert callable(getattr(sfmhip, name)), name


def test_comm_argument_errors_without_gpu(sfm):
    """The comm entry points report argument errors without touching RCCL or a GPU."""
    assert sfm.lib.sfmhip_comm_init_rank(0, None, 0, None) == -1
    assert b"null pointer" in sfm.lib.sfmhip_last_error()
    assert sfm.lib.sfmhip_allgather(None, None, None, 0, 0, None) == -1
    assert sfm.lib.sfmhip_comm_destroy(None) == 0


def test_product_has_no_oracle_dependency():
    """The product package must never import the oracle (no CPU fallback)."""
    pkg = os.path.join(ROOT, "3d_reconstruction_amd")
    for fn in os.listdir(pkg):
        if fn.endswith(".py"):
            src = open(os.path.join(pkg, fn)).read()
            assert "oracle" not in re.sub(r"#.*", "", src).replace('"""', "").split("import")[0] or \
                not re.search(r"^\s*(from|import)\s+oracle", src, flags=re.M), fn
            assert not re.search(r"^\s*(from|import)\s+oracle", src, flags=re.M), fn
