"""ctypes binding of the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_float, c_int, c_int64, c_void_p

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# GSR_ORACLE_LIBRARY: another build of the oracle (tests/test_sanitizers.py runs the loader
# and golden tests against the ASan/UBSan build, build/asan/liboracle.so)
ORACLE_SO = os.environ.get("GSR_ORACLE_LIBRARY") or os.path.join(ROOT, "oracle", "liboracle.so")
REF_DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_driver")

SPLAT_DTYPE = np.dtype([
    ("status", "<i4"), ("color", "<f4", 3), ("ndc", "<f4", 3), ("view", "<f4", 3),
    ("inv_covar", "<f4", 4), ("aabb", "<i4", 4), ("px_x", "<i4"), ("px_y", "<i4"),
    ("depth_key", "<u4"), ("opacity", "<f4"),
])

_L = None


def lib():
    global _L
    if _L is None:
        if not os.path.exists(ORACLE_SO):
            raise ImportError(f"{ORACLE_SO} missing: run `make -C oracle`")
        from gaussianrenderer_amd._native import Camera
        L = ctypes.CDLL(ORACLE_SO)
        cam = POINTER(Camera)
        L.orc_ply_read.argtypes = [ctypes.c_char_p, c_void_p, c_int64, POINTER(c_int64)]
        L.orc_ply_read.restype = c_int
        L.orc_ply_read_ex.argtypes = [ctypes.c_char_p, c_void_p, c_int, c_int64, POINTER(c_int64)]
        L.orc_ply_read_ex.restype = c_int
        L.orc_temporal.argtypes = [c_void_p, c_int64, c_float, c_void_p]
        L.orc_temporal.restype = None
        L.orc_set_sh3.argtypes = [c_int]
        L.orc_set_sh3.restype = None
        L.orc_set_blend_variant.argtypes = [c_int, c_int, c_int]
        L.orc_set_blend_variant.restype = None
        L.orc_intrinsics.argtypes = [cam, POINTER(c_float), POINTER(c_float)]
        L.orc_preprocess.argtypes = [c_void_p, c_int64, cam, c_int, c_int, c_float, c_void_p]
        L.orc_preprocess.restype = c_int
        L.orc_render.argtypes = [c_void_p, c_int64, cam, c_int, c_int, c_int, c_int, c_int, c_int, c_float,
                                 c_void_p, c_int]
        L.orc_render.restype = c_int
        L.orc_render_takes.argtypes = [c_void_p, c_int64, cam, c_int, c_int, c_int, c_int, c_int, c_int, c_float,
                                       c_void_p, c_void_p, c_int]
        L.orc_render_takes.restype = c_int
        L.orc_alpha_take_min_x.argtypes = [c_float]
        L.orc_alpha_take_min_x.restype = c_float
        L.orc_alpha_taken.argtypes = [c_float, c_float]
        L.orc_alpha_taken.restype = c_int
        L.orc_render_tiled.argtypes = [c_void_p, c_int64, cam, c_int, c_int, c_int, c_int, c_int, c_int,
                                       c_float, c_void_p]
        L.orc_render_tiled.restype = c_int
        L.orc_project.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
        L.orc_covariance_chain.argtypes = [c_void_p, c_void_p, c_void_p, c_float, c_float, c_void_p, c_void_p,
                                           c_void_p]
        for f in ("orc_expf", "orc_blend_expf", "orc_sinf", "orc_cosf"):
            getattr(L, f).argtypes = [c_float]
            getattr(L, f).restype = c_float
        L.orc_blend_exp_sweep.argtypes = [c_float, c_float, c_void_p, c_void_p]
        L.orc_blend_exp_sweep.restype = None
        L.orc_atan2f.argtypes = [c_float, c_float]
        L.orc_atan2f.restype = c_float
        assert SPLAT_DTYPE.itemsize == 88
        _L = L
    return _L


def ply_read(path: str) -> np.ndarray:
    n = c_int64(-1)
    rc = lib().orc_ply_read(path.encode(), None, 0, ctypes.byref(n))
    if rc:
        raise IOError(f"orc_ply_read({path}) = {rc}")
    soa = np.zeros((38, n.value), dtype=np.float32)
    rc = lib().orc_ply_read(path.encode(), soa.ctypes.data, n.value, ctypes.byref(n))
    if rc:
        raise IOError(f"orc_ply_read({path}) = {rc}")
    return soa


def ply_read_sh3(path: str) -> np.ndarray:
    """(59, n) SH-3 ("Inria-correct") arrays through the oracle's reader."""
    n = c_int64(-1)
    rc = lib().orc_ply_read_ex(path.encode(), None, 59, 0, ctypes.byref(n))
    if rc:
        raise IOError(f"orc_ply_read_ex({path}) = {rc}")
    soa = np.zeros((59, n.value), dtype=np.float32)
    rc = lib().orc_ply_read_ex(path.encode(), soa.ctypes.data, 59, n.value, ctypes.byref(n))
    if rc:
        raise IOError(f"orc_ply_read_ex({path}) = {rc}")
    return soa


class sh3_mode:
    """Context manager: the oracle evaluates degree-3 SH on 59-array scenes."""

    def __enter__(self):
        lib().orc_set_sh3(1)

    def __exit__(self, *exc):
        lib().orc_set_sh3(0)


class blend_variant:
    """Context manager: the oracle's blend with another FMA contraction of render.cu:331
    and 337 (md2 0..4, rgb 0..1) or the host libm expf (exp 1); (1, 1, 0) is the shipped
    choice the kernels share (gsr_oracle.c blend_step_var)."""

    def __init__(self, md2: int = 1, rgb: int = 1, exp: int = 0):
        self.v = (md2, rgb, exp)

    def __enter__(self):
        lib().orc_set_blend_variant(*self.v)

    def __exit__(self, *exc):
        lib().orc_set_blend_variant(1, 1, 0)


def ply_read4d(path: str) -> np.ndarray:
    """(49, n) arrays of a 4D (config 5) .ply through the oracle's reader."""
    n = c_int64(-1)
    rc = lib().orc_ply_read_ex(path.encode(), None, 49, 0, ctypes.byref(n))
    if rc:
        raise IOError(f"orc_ply_read_ex({path}) = {rc}")
    soa = np.zeros((49, n.value), dtype=np.float32)
    rc = lib().orc_ply_read_ex(path.encode(), soa.ctypes.data, 49, n.value, ctypes.byref(n))
    if rc:
        raise IOError(f"orc_ply_read_ex({path}) = {rc}")
    return soa


def temporal(soa49: np.ndarray, t: float) -> np.ndarray:
    """Config 5: the (38, n) 3D scene at time t (no temporal cull)."""
    soa49 = np.ascontiguousarray(soa49, dtype=np.float32)
    n = soa49.shape[1]
    out = np.zeros((38, n), dtype=np.float32)
    lib().orc_temporal(soa49.ctypes.data, n, float(t), out.ctypes.data)
    return out


def preprocess(soa: np.ndarray, cam, W: int, H: int, k: float) -> np.ndarray:
    soa = np.ascontiguousarray(soa, dtype=np.float32)
    n = soa.shape[1]
    out = np.zeros(n, dtype=SPLAT_DTYPE)
    lib().orc_preprocess(soa.ctypes.data, n, ctypes.byref(cam), W, H, k, out.ctypes.data)
    return out


def render(soa: np.ndarray, cam, W: int, H: int, k: float, tiling=None, threads: int = 0) -> np.ndarray:
    soa = np.ascontiguousarray(soa, dtype=np.float32)
    nx, ny, ws, hs = tiling if tiling else (1, 1, W, H)
    out = np.zeros((3, H, W), dtype=np.float32)
    rc = lib().orc_render(soa.ctypes.data, soa.shape[1], ctypes.byref(cam), W, H, nx, ny, ws, hs, k,
                          out.ctypes.data, threads)
    assert rc == 0
    return out


def render_takes(soa: np.ndarray, cam, W: int, H: int, k: float, tiling=None, threads: int = 0):
    """render() plus the take map (gsr_blend_take_map): per pixel, the splats composited
    as count | (sum of (index + 1) * 2654435761 mod 2^32) << 32."""
    soa = np.ascontiguousarray(soa, dtype=np.float32)
    nx, ny, ws, hs = tiling if tiling else (1, 1, W, H)
    out = np.zeros((3, H, W), dtype=np.float32)
    takes = np.zeros((H, W), dtype=np.uint64)
    rc = lib().orc_render_takes(soa.ctypes.data, soa.shape[1], ctypes.byref(cam), W, H, nx, ny, ws, hs, k,
                                out.ctypes.data, takes.ctypes.data, threads)
    assert rc == 0
    return out, takes


def render_tiled(soa: np.ndarray, cam, W: int, H: int, k: float, tiling) -> np.ndarray:
    soa = np.ascontiguousarray(soa, dtype=np.float32)
    nx, ny, ws, hs = tiling
    out = np.zeros((3, H, W), dtype=np.float32)
    rc = lib().orc_render_tiled(soa.ctypes.data, soa.shape[1], ctypes.byref(cam), W, H, nx, ny, ws, hs, k,
                                out.ctypes.data)
    assert rc == 0
    return out


def expected_depth_order(spl: np.ndarray) -> np.ndarray:
    """(depth_key << 32 | index) of every Gaussian, stable-sorted by key (index tie-break);
    culled / dropped Gaussians carry key 0xFFFFFFFF."""
    n = spl.shape[0]
    keys = np.where(spl["status"] == 2, spl["depth_key"], np.uint32(0xFFFFFFFF)).astype(np.uint64)
    items = (keys << np.uint64(32)) | np.arange(n, dtype=np.uint64)
    return np.sort(items, kind="stable")
