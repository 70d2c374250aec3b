"""ctypes binding of ``libsfmhip.so`` (the C-ABI declared in ``include/sfmhip.h``).

This is the only place the package touches native code.  The library is built
in-tree by ``__graft_entry__.build()`` (``make -C 3d_reconstruction_amd/csrc``)
and is REQUIRED: importing the package on a machine without it raises, and the
compute entry points raise when no HIP device is present.  There is no CPU
fallback anywhere in the product path.

Device memory is handed over as raw pointers (``tensor.data_ptr()``) of
torch-ROCm tensors; torch is used only as the allocator / stream provider.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsfmhip.so")

SFMHIP_OK = 0
SFMHIP_E_ARG = -1
SFMHIP_E_HIP = -2
SFMHIP_E_UNSUPPORTED = -3
SFMHIP_E_OVERFLOW = -4
SFMHIP_E_COMM = -5

# sfmhip_allgather element types (include/sfmhip.h SFMHIP_DT_*)
DT_INT8, DT_UINT8, DT_INT16, DT_INT32, DT_INT64, DT_FLOAT32, DT_FLOAT64 = range(7)
DT_OF = {torch.int8: DT_INT8, torch.uint8: DT_UINT8, torch.int16: DT_INT16, torch.int32: DT_INT32,
         torch.int64: DT_INT64, torch.float32: DT_FLOAT32, torch.float64: DT_FLOAT64}


class SfmHipError(RuntimeError):
    """Raised when a libsfmhip call returns a non-zero status."""

    def __init__(self, func: str, code: int, msg: str):
        super().__init__(f"{func} failed ({code}): {msg}")
        self.code = code


_p = ctypes.c_void_p
_i32 = ctypes.c_int
_i64 = ctypes.c_int64
_f32 = ctypes.c_float
_f64 = ctypes.c_double
_u64 = ctypes.c_uint64
_sz = ctypes.c_size_t

# name -> argtypes, in the order of include/sfmhip.h
SIGNATURES = {
    "sfmhip_version": [],
    "sfmhip_last_error": [],
    "sfmhip_device_arch": [ctypes.c_char_p, _i32],
    "sfmhip_scratch_trim": [_u64],
    "sfmhip_scratch_release_stream": [_p],
    "sfmhip_knobs_reload": [],
    "sfmhip_desc_quantize": [_p, _i32, _i32, _i32, _p, _i32, _p, _p],
    "sfmhip_desc_prepare": [_p, _i32, _i32, _i32, _p, _p, _p, _p],
    "sfmhip_desc_prepare_shifted": [_p, _i32, _i32, _i32, _p, _i32, _p, _p, _p, _p],
    "sfmhip_match_pairs": [_p, _p, _p, _p, _i32, _i32, _i32, _p, _i32, _i32, _i32, _p, _p, _p, _p],
    "sfmhip_match_pairs_i16": [_p, _p, _p, _p, _i32, _i32, _i32, _p, _i32, _i32, _i32, _p, _p],
    "sfmhip_mutual_filter": [_p, _p, _i32, _i32, _p],
    "sfmhip_desc_residual": [_p, _p, _i32, _i32, _i32, _p, _i32, _p, _p, _p],
    "sfmhip_match_pairs_exact": [_p, _p, _p, _p, _p, _p, _p, _i32, _p, _i32, _i32, _i32, _p, _i32, _i32, _i32,
                                 _p, _p, _p, _p, _p],
    "sfmhip_match_pairs_exact_i16": [_p, _p, _p, _p, _p, _p, _p, _i32, _p, _i32, _i32, _i32, _p, _i32, _i32,
                                     _i32, _p, _p, _p],
    "sfmhip_vq": [_p, _i64, _p, _i32, _i32, _p, _p, _p],
    "sfmhip_word_histogram": [_p, _p, _i32, _i32, _p, _p],
    "sfmhip_kmeans_update": [_p, _i64, _i32, _p, _i32, _p, _p, _p],
    "sfmhip_track_interlace": [_p, _i64, _p, _i64, _p, _p, _i64, _p],
    "sfmhip_track_merge": [_p, _i64, _p, _i64, _p, _p, _i64, _p, _p],
    "sfmhip_triangulate_dlt": [_p, _p, _p, _p, _i64, _p, _p],
    "sfmhip_reproj_residual": [_p, _p, _p, _p, _p, _i64, _p, _p],
    "sfmhip_reproj_residual_host": [_p, _p, _p, _p, _i64, _p, _p],
    "sfmhip_reproj_fd_jacobian": [_p, _p, _p, _p, _p, _i32, _i64, _p, _p, _p, _p],
    "sfmhip_ba_solve": [_p, _p, _p, _p, _p, _i32, _i64, _f64, _f64, _f64, _i32, _p, _p, _p, _p, _p],
    "sfmhip_voxel_traversal_count": [_p, _i64, _f32, _i32, _p, _p],
    "sfmhip_voxel_traversal": [_p, _i64, _f32, _i32, _p, _p],
    "sfmhip_voxel_traversal_capped": [_p, _i64, _f32, _i32, _p, _p, _p],
    "sfmhip_voxel_traversal_rows": [_p, _i32, _p, _i64, _i32, _p, _p],
    "sfmhip_grid_sample": [_p, _i32, _i32, _i32, _i32, _p, _p, _i32, _p, _i64, _p, _p],
    "sfmhip_nerf_forward": [_p, _i32, _i32, _i32, _p, _p, _i32, _p, _p, _i64, _p, _p, _p],
    "sfmhip_grid_to_voxel_major": [_p, _i32, _i32, _i32, _i32, _p, _p],
    "sfmhip_render_rays": [_p, _i32, _i32, _i32, _p, _p, _i32, _p, _p, _p, _i64, _i32, _p, _p],
    "sfmhip_render_rays_sdf": [_p, _p, _i32, _i32, _i32, _p, _p, _i32, _p, _p, _p, _i64, _i32, _p, _p],
    "sfmhip_tsdf_integrate": [_p, _p, _i32, _i32, _i32, _i32, _i32, _p, _i32, _i32, _i32, _p, _p, _p, _p,
                              _f32, _p],
    "sfmhip_tsdf_block_table": [_p, _i32, _i32, _i32, _i32, _i32, _p, _p],
    "sfmhip_tsdf_integrate_tab": [_p, _p, _i32, _i32, _i32, _i32, _i32, _p, _i32, _i32, _i32, _p, _p, _p, _p,
                                  _f32, _p, _p],
    "sfmhip_tsdf_cull_stats": [_i32, _i32, _i32, _i32, _i32, _p, _i32, _i32, _i32, _p, _p, _p, _p, _f32, _p, _p],
    "sfmhip_tsdf_layer_stats": [_i32, _i32, _i32, _p, _i32, _i32, _i32, _p, _p, _p, _p, _f32, _p, _p],
    "sfmhip_find_essential": [_p, _p, _p, _i32, _p, _f64, _f64, _i32, _p, _p, _p, _p, _p, _p, _p],
    "sfmhip_recover_pose": [_p, _i64, _p, _p, _p, _i32, _p, _p, _f64, _p, _p, _p, _p, _p],
    "sfmhip_pnp_ransac": [_p, _p, _p, _i32, _p, _i32, _f64, _f64, _p, _p, _p, _p, _p, _p, _p, _p],
    "sfmhip_render_train": [_p, _i32, _i32, _i32, _p, _p, _i32, _p, _p, _p, _p, _i64, _i32, _p, _p, _p, _p, _p],
    "sfmhip_adam_step": [_p, _p, _p, _p, _i64, _f64, _f64, _f64, _f64, _i64, _i32, _p],
    "sfmhip_adam_step_flagged": [_p, _p, _p, _p, _i64, _f64, _f64, _f64, _f64, _i64, _i32, _p, _i32, _p],
    "sfmhip_grid_from_voxel_major": [_p, _i32, _i32, _i32, _i32, _p, _p],
    "sfmhip_ray_aabb": [_p, _p, _i64, _p, _p, _p, _p, _p, _p],
    "sfmhip_stratified_samples": [_p, _p, _p, _i64, _i32, _i32, _p, _p],
    "sfmhip_comm_unique_id": [_p],
    "sfmhip_comm_init_rank": [_i32, _p, _i32, _p],
    "sfmhip_comm_init_all": [_i32, _p, _p],
    "sfmhip_comm_info": [_p, _p, _p, _p],
    "sfmhip_allgather": [_p, _p, _p, _sz, _i32, _p],
    "sfmhip_comm_group_start": [],
    "sfmhip_comm_group_end": [],
    "sfmhip_comm_destroy": [_p],
}


def _load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libsfmhip.so not found at {LIB_PATH}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (make -C 3d_reconstruction_amd/csrc)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = _i32
    lib.sfmhip_last_error.restype = ctypes.c_char_p
    return lib


lib = _load()


def call(name: str, *args) -> None:
    """Invoke ``name`` and raise :class:`SfmHipError` on a non-zero status."""
    rc = getattr(lib, name)(*args)
    if rc != SFMHIP_OK:
        msg = lib.sfmhip_last_error().decode(errors="replace")
        raise SfmHipError(name, rc, msg)


def knobs_reload() -> None:
    """Re-read the library's runtime knobs (SFMHIP_*) from the
    environment; the library reads them once, at its first call."""
    call("sfmhip_knobs_reload")


def require_gpu() -> torch.device:
    """The compute path runs only on a HIP device; fail loudly otherwise."""
    if not torch.cuda.is_available():
        raise RuntimeError("sfmhip: no HIP device visible — the MI355X kernels cannot run "
                           "(there is deliberately no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()


def dev(x, dtype: torch.dtype) -> torch.Tensor:
    """numpy / tensor -> contiguous device tensor of ``dtype`` (copy only if needed)."""
    d = require_gpu()
    if isinstance(x, torch.Tensor):
        t = x
    else:
        t = torch.as_tensor(x)
    if t.device != d or t.dtype != dtype:
        t = t.to(device=d, dtype=dtype)
    return t.contiguous()
