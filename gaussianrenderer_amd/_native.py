"""ctypes binding of libgsr.so (the C ABI declared in include/gsr.h).

The shared library is built in-tree by ``make`` (``__graft_entry__.build()``)
into ``gaussianrenderer_amd/lib/libgsr.so``.  There is no Python or CPU
fallback for anything that renders: if the library is missing, importing this
module raises.

Import torch BEFORE this module in processes that use both: torch ships its
own ``libamdhip64.so`` (SONAME ``libamdhip64.so.7``) and the dynamic loader
then binds libgsr to that same HIP runtime instead of loading a second one.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int64, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
# GSR_LIBRARY: another build of the same library (tools/ab_libs.sh A/B runs of two builds
# on one box); the product default is the in-tree build.
LIB_PATH = os.environ.get("GSR_LIBRARY") or os.path.join(_HERE, "lib", "libgsr.so")

GSR_OK = 0
GSR_E_ARG = -1
GSR_E_HIP = -2
GSR_E_IO = -3
GSR_E_FORMAT = -4
GSR_E_OVERFLOW = -5
GSR_PATH_NO_JOIN = 1   # gsr_render_path_ex flags (include/gsr.h)
GSR_PATH_NO_FORK = 2
GSR_E_DISPLAY = -6
GSR_FRAME_PAIR_OVERFLOW = 1   # gsr_render_path_status validity bits (include/gsr.h)
GSR_FRAME_DEPTH_PASSES = 2
GSR_FRAME_SPEC_MISS = 4

LAYOUT_SCENE_BLOCK = 0
LAYOUT_AOS = 1
LAYOUT_SCENE_BLOCK_4D = 2
LAYOUT_SCENE_BLOCK_SH3 = 3
PLY_TYPED = 1
PLY_SH3 = 2

STAGES = ("preprocess", "depth_sort", "emit", "tile_sort", "ranges", "blend", "resume")
NUM_STAGES = len(STAGES)
TILE_PX = 16
SPLAT_RECORD_BYTES = 64
SCENE_NARRAYS = 38
SCENE4D_NARRAYS = 49
SCENE_SH3_NARRAYS = 59


class Camera(ctypes.Structure):
    """Layout-identical to the reference ``Camera`` (scene/camera.hpp:2-41), 484 B."""

    _fields_ = [
        ("position", c_float * 3),
        ("lookAt", c_float * 3),
        ("w_up", c_float * 3),
        ("fovY", c_float),
        ("aspectRatio", c_float),
        ("nearClip", c_float),
        ("farClip", c_float),
        ("forward_vec", c_float * 3),
        ("right_vec", c_float * 3),
        ("up_vec", c_float * 3),
        ("P_matrix", c_float * 16),
        ("V_matrix", c_float * 16),
        ("M_matrix", c_float * 16),
        ("f_axis", c_float * 3),
        ("r_axis", c_float * 3),
        ("u_axis", c_float * 3),
        ("r_cam", c_float * 9),
        ("r_cam_T", c_float * 9),
        ("plane_normals", c_float * 24),
    ]


assert ctypes.sizeof(Camera) == 484


class Lwg(ctypes.Structure):
    """``lightWeightGaussian`` (utils/gaussians.hpp:32-35), 16 B."""

    _fields_ = [("radix_id", c_uint64), ("gaussian_id", c_uint32)]


assert ctypes.sizeof(Lwg) == 16

# (name, restype, argtypes) for every symbol of include/gsr.h and include/gsr_gl.h.
SIGNATURES = [
    ("preprocessCUDAGaussians", None,
     [c_void_p, POINTER(c_float), c_int, Camera, c_int, c_int, c_int, c_int, c_int, c_int, c_float]),
    ("gsr_load_ply_device", c_void_p, [c_char_p, POINTER(c_int)]),
    ("gsr_load_ply_device_ex", c_void_p, [c_char_p, POINTER(c_int), c_int, POINTER(c_int)]),
    ("oneSweep3DGaussianSort", None, [POINTER(Lwg), c_int, c_int, POINTER(c_float)]),
    ("oneSweepSort", None, [POINTER(c_int), POINTER(c_int), c_int, c_int, POINTER(c_float)]),
    # include/gsr_gl.h: display interop (SSBO written in place, no host round trip)
    ("preprocessCUDAGaussiansGL", None,
     [c_void_p, ctypes.c_uint, c_int, Camera, c_int, c_int, c_int, c_int, c_int, c_int, c_float]),
    ("gsr_display_register_gl", c_int, [ctypes.c_uint, POINTER(c_void_p)]),
    ("gsr_display_wrap_device", c_int, [c_void_p, ctypes.c_size_t, POINTER(c_void_p)]),
    ("gsr_display_free", c_int, [c_void_p]),
    ("gsr_display_gl_current", c_int, []),
    ("gsr_render_display", c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int64, POINTER(Camera), c_int, c_int,
                                   c_int, c_int, c_int, c_int, c_float, c_void_p]),
    ("gsr_create", c_void_p, []),
    ("gsr_destroy", None, [c_void_p]),
    ("gsr_reserve", c_int, [c_void_p, c_int64, c_int64]),
    ("gsr_render", c_int, [c_void_p, c_void_p, c_int, c_int64, POINTER(Camera), c_int, c_int, c_int, c_int,
                           c_int, c_int, c_float, c_void_p, c_void_p]),
    ("gsr_render_path", c_int, [c_void_p, c_void_p, c_int, c_int64, POINTER(Camera), c_void_p, c_int, c_int,
                                c_int, c_int, c_int, c_int, c_int, c_float, c_void_p, c_void_p]),
    ("gsr_render_path_ex", c_int, [c_void_p, c_void_p, c_int, c_int64, POINTER(Camera), c_void_p, c_int, c_int,
                                   c_int, c_int, c_int, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_int]),
    ("gsr_render_path_status", c_int, [c_void_p, c_void_p, c_int, c_int64, POINTER(Camera), c_void_p, c_int,
                                       c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_int, c_void_p]),
    ("gsr_set_frames_in_flight", c_int, [c_void_p, c_int]),
    ("gsr_frames_in_flight", c_int, [c_void_p]),
    ("gsr_preprocess", c_int, [c_void_p, c_void_p, c_int, c_int64, POINTER(Camera), c_int, c_int, c_int, c_int,
                               c_int, c_int, c_float, c_void_p]),
    ("gsr_sort", c_int, [c_void_p, c_void_p]),
    ("gsr_blend", c_int, [c_void_p, c_void_p, c_void_p]),
    ("gsr_sync", c_int, [c_void_p]),
    ("gsr_pair_count", c_int64, [c_void_p]),
    ("gsr_row_item_count", c_int64, [c_void_p]),
    ("gsr_read_splats", c_int, [c_void_p, c_void_p, c_int64]),
    ("gsr_read_depth_order", c_int, [c_void_p, c_void_p, c_int64]),
    ("gsr_read_pairs", c_int64, [c_void_p, c_void_p, c_int64]),
    ("gsr_tile_grid", c_int, [c_void_p, POINTER(c_int), POINTER(c_int)]),
    ("gsr_read_tile_ranges", c_int, [c_void_p, c_void_p, c_int64]),
    ("gsr_set_timing", c_int, [c_void_p, c_int]),
    ("gsr_stage_times", c_int, [c_void_p, POINTER(c_double), POINTER(c_int64)]),
    ("gsr_set_diagnostics", c_int, [c_void_p, c_int]),
    ("gsr_blend_records_loaded", c_int64, [c_void_p]),
    ("gsr_blend_counters", c_int, [c_void_p, c_void_p]),
    ("gsr_set_blend_variant", c_int, [c_void_p, c_int]),
    ("gsr_blend_stamps", c_int, [c_void_p, c_void_p, c_int64]),
    ("gsr_blend_counters_ex", c_int, [c_void_p, c_void_p, c_int]),
    ("gsr_blend_take_map", c_int, [c_void_p, c_void_p, c_int64]),
    ("gsr_set_tuning", c_int, [c_void_p, c_int, c_int]),
    ("gsr_get_tuning", c_int, [c_void_p, c_int, c_void_p]),
    ("gsr_set_timing_stride", c_int, [c_void_p, c_int, c_int]),
    ("gsr_depth_passes", c_int, [c_void_p]),
    ("gsr_bucket_sizes", c_int, [c_void_p, c_void_p, c_int]),
    ("gsr_scene_upload", c_void_p, [c_void_p, c_int64]),
    ("gsr_scene_upload_ex", c_void_p, [c_void_p, c_int, c_int64]),
    ("gsr_set_time", c_int, [c_void_p, c_float]),
    ("gsr_scene_free", None, [c_void_p]),
    ("gsr_scene_download", c_int, [c_void_p, c_void_p, c_int64]),
    ("gsr_scene_bytes", c_int64, [c_int, c_int64]),
    ("gsr_scene_copy", c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p]),
    ("gsr_ply_read_host", c_int, [c_char_p, c_void_p, c_int64, POINTER(c_int64)]),
    ("gsr_ply_read_host_ex", c_int, [c_char_p, c_void_p, c_int, c_int64, POINTER(c_int64), c_int, POINTER(c_int)]),
    ("gsr_synth_write_ply", c_int, [c_char_p, c_int64, c_uint64]),
    ("gsr_synth_write_ply4d", c_int, [c_char_p, c_int64, c_uint64]),
    ("gsr_camera_default", None, [POINTER(Camera)]),
    ("gsr_camera_update", None, [POINTER(Camera)]),
    ("gsr_camera_update_frustum", None, [POINTER(Camera)]),
    ("gsr_camera_zoom", None, [POINTER(Camera), c_float]),
    ("gsr_camera_orbit", None, [POINTER(Camera), c_float, c_float]),
    ("gsr_camera_intrinsics", None, [POINTER(Camera), POINTER(c_float), POINTER(c_float)]),
    ("gsr_last_error", c_char_p, []),
    ("gsr_version", c_char_p, []),
    ("gsr_device_available", c_int, []),
    ("gsr_math_probe", c_int, [c_void_p, c_int, c_void_p]),
    ("gsr_exp_probe", c_int, [c_float, c_float, c_float, c_void_p, c_void_p, c_void_p]),
    ("gsr_exp_probe2", c_int, [c_float, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("gsr_alpha_cut_probe", c_int, [c_void_p, c_int, c_void_p]),
    ("gsr_rank_order_check", c_int, [POINTER(c_int64), POINTER(c_int64)]),
]

# C++-linkage drop-in loader (misc.cuh:4): mangled name of
# Gaussian* loadGaussianCudaFromPly(const std::string&, int*).
CXX_SYMBOLS = ["_Z23loadGaussianCudaFromPlyRKNSt7__cxx1112basic_stringIcSt11char_traitsIcESaIcEEEPi"]

_lib = None


def lib() -> ctypes.CDLL:
    """Load libgsr.so once; raises if it was not built (no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `make` (or __graft_entry__.build()) first")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, res, args in SIGNATURES:
        try:
            fn = getattr(L, name)
        except AttributeError:
            if os.environ.get("GSR_LIBRARY"):   # an older build in an A/B run: its API subset
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


class GsrError(RuntimeError):
    def __init__(self, code: int, where: str):
        msg = lib().gsr_last_error().decode(errors="replace")
        super().__init__(f"{where} failed ({code}): {msg}")
        self.code = code


def check(code: int, where: str) -> int:
    if code != GSR_OK:
        raise GsrError(code, where)
    return code
