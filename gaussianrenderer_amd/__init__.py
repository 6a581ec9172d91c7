"""gaussianrenderer_amd — MI355X-native 3D Gaussian splatting rasterizer.

Host-side mirror of the reference's interface (wwangg22/GaussianRenderer):

* :func:`loadGaussianCudaFromPly`  — misc.cu:13-134 (device scene block)
* :func:`preprocessCUDAGaussians`  — render.cu:871-1157 (whole frame, host image)
* :func:`preprocessCUDAGaussiansGL` — Canvas::render (canvas.cpp:337-351) into the
  viewer's colour SSBO, no host round trip (include/gsr_gl.h; :class:`DisplayTarget`)
* :class:`TilingInformation`       — utils/gaussians.hpp:38-60
* :func:`make_camera` / :func:`orbit` — scene/camera.cpp

and the native stream-ordered API (:class:`Renderer`) used by the bench.
Everything that renders runs in libgsr.so (hand-written gfx950 HIP kernels);
there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_float, c_int, c_int64, c_void_p

import numpy as np

from . import _native
from ._native import (Camera, GsrError, LAYOUT_AOS, LAYOUT_SCENE_BLOCK, LAYOUT_SCENE_BLOCK_4D,
                      LAYOUT_SCENE_BLOCK_SH3, NUM_STAGES, PLY_SH3, PLY_TYPED, SCENE4D_NARRAYS, SCENE_NARRAYS,
                      SCENE_SH3_NARRAYS,
                      SPLAT_RECORD_BYTES, STAGES, TILE_PX, check, lib)

__all__ = [
    "Camera", "GsrError", "Renderer", "Scene", "TilingInformation", "make_camera", "orbit",
    "loadGaussianCudaFromPly", "preprocessCUDAGaussians", "read_ply", "write_synthetic_ply",
    "SPLAT_DTYPE", "STAGES", "TILE_PX", "lib", "DisplayTarget", "display_gl_current", "preprocessCUDAGaussiansGL",
]

# gsr_read_splats record (include/gsr.h).
SPLAT_DTYPE = np.dtype([
    ("inv_covar", "<f4", 4), ("opacity", "<f4"), ("color", "<f4", 3),
    ("px_x", "<i4"), ("px_y", "<i4"), ("x_range", "<u4"), ("y_range", "<u4"),
    ("tile_x_range", "<u4"), ("tile_y_range", "<u4"), ("tile_count", "<u4"), ("depth_key", "<u4"),
])
assert SPLAT_DTYPE.itemsize == SPLAT_RECORD_BYTES


class TilingInformation:
    """utils/gaussians.hpp:38-60 — ctor argument order (ny, nx, h, w)."""

    def __init__(self, ny: int, nx: int, h: int, w: int):
        self.num_tile_y, self.num_tile_x, self.H, self.W = ny, nx, h, w
        self._strides()

    def _strides(self):
        self.width_stride = max(1, (self.W + self.num_tile_x - 1) // self.num_tile_x)
        self.height_stride = max(1, (self.H + self.num_tile_y - 1) // self.num_tile_y)

    def resize(self, h: int, w: int, num_tile_x: int, num_tile_y: int):
        self.H, self.W, self.num_tile_x, self.num_tile_y = h, w, num_tile_x, num_tile_y
        self._strides()


def make_camera(position=(0.0, 0.0, 4.0), look_at=(0.0, 0.0, 0.0), up=(0.0, 1.0, 0.0), fov_y=50.0,
                aspect=16.0 / 9.0, near=0.1, far=100.0) -> Camera:
    """Camera() + setters + updateCameraMatrices() + updateFrustumPlanes() (camera.cpp)."""
    cam = Camera()
    L = lib()
    L.gsr_camera_default(byref(cam))
    cam.position[:] = [float(v) for v in position]
    cam.lookAt[:] = [float(v) for v in look_at]
    cam.w_up[:] = [float(v) for v in up]
    cam.fovY, cam.aspectRatio, cam.nearClip, cam.farClip = fov_y, aspect, near, far
    L.gsr_camera_update(byref(cam))
    L.gsr_camera_update_frustum(byref(cam))
    return cam


def orbit(cam: Camera, azimuth_deg: float, elevation_deg: float = 0.0) -> Camera:
    """Camera::orbit (camera.cpp:130-158), in place; returns cam."""
    lib().gsr_camera_orbit(byref(cam), azimuth_deg, elevation_deg)
    return cam


def camera_intrinsics(cam: Camera):
    fx, fy = c_float(), c_float()
    lib().gsr_camera_intrinsics(byref(cam), byref(fx), byref(fy))
    return fx.value, fy.value


def read_ply(path: str, typed: bool = False, four_d: bool | None = False, sh3: bool = False) -> np.ndarray:
    """Host PLY parse -> (38, n) float32 SoA (reference loader semantics), or the
    hardened typed reader (typed=True: declared types, ascii, big-endian).
    four_d=True returns the (49, n) 4D arrays; four_d=None picks by the file;
    sh3=True the (59, n) "Inria-correct" degree-3 SH arrays."""
    L = lib()
    n = c_int64(-1)
    is4d = c_int(0)
    flags = (PLY_TYPED if typed else 0) | (PLY_SH3 if sh3 else 0)
    check(L.gsr_ply_read_host_ex(path.encode(), None, SCENE_SH3_NARRAYS if sh3 else SCENE_NARRAYS, 0, byref(n),
                                 flags, byref(is4d)), "gsr_ply_read_host")
    na = SCENE4D_NARRAYS if (four_d or (four_d is None and is4d.value)) else SCENE_NARRAYS
    if sh3:
        na = SCENE_SH3_NARRAYS
    soa = np.zeros((na, n.value), dtype=np.float32)
    check(L.gsr_ply_read_host_ex(path.encode(), soa.ctypes.data, na, n.value, byref(n), flags, None),
          "gsr_ply_read_host")
    return soa


def write_synthetic_ply(path: str, n: int, seed: int) -> None:
    """Seeded synthetic 62-property 3DGS PLY."""
    check(lib().gsr_synth_write_ply(path.encode(), int(n), int(seed)), "gsr_synth_write_ply")


def write_synthetic_ply4d(path: str, n: int, seed: int) -> None:
    """Seeded synthetic 4D (Spacetime-Gaussian style, 73-property) PLY for config 5."""
    check(lib().gsr_synth_write_ply4d(path.encode(), int(n), int(seed)), "gsr_synth_write_ply4d")


class Scene:
    """A device scene block (one hipMalloc: header + SoA arrays)."""

    def __init__(self, ptr: int, n: int, owned: bool = True, narrays: int = SCENE_NARRAYS):
        self.ptr, self.n, self.owned, self.narrays = ptr, n, owned, narrays

    @property
    def is_4d(self) -> bool:
        return self.narrays == SCENE4D_NARRAYS

    @property
    def is_sh3(self) -> bool:
        return self.narrays == SCENE_SH3_NARRAYS

    @property
    def layout(self) -> int:
        return (LAYOUT_SCENE_BLOCK_4D if self.is_4d else LAYOUT_SCENE_BLOCK_SH3 if self.is_sh3
                else LAYOUT_SCENE_BLOCK)

    @classmethod
    def from_soa(cls, soa: np.ndarray) -> "Scene":
        soa = np.ascontiguousarray(soa, dtype=np.float32)
        assert soa.shape[0] in (SCENE_NARRAYS, SCENE4D_NARRAYS, SCENE_SH3_NARRAYS)
        ptr = lib().gsr_scene_upload_ex(soa.ctypes.data, soa.shape[0], soa.shape[1])
        if not ptr:
            raise GsrError(-2, "gsr_scene_upload")
        return cls(ptr, soa.shape[1], narrays=soa.shape[0])

    @classmethod
    def from_ply(cls, path: str, typed: bool = False, allow_4d: bool = True, sh3: bool = False) -> "Scene":
        """Device scene from a .ply (the reference loader unless typed=True); a file
        with the 4D properties loads as a 4D scene when allow_4d; sh3=True gives
        the "Inria-correct" degree-3 SH scene."""
        n = c_int(0)
        na = c_int(SCENE_NARRAYS)
        flags = (PLY_TYPED if typed else 0) | (PLY_SH3 if sh3 else 0)
        ptr = lib().gsr_load_ply_device_ex(path.encode(), byref(n), flags,
                                           byref(na) if (allow_4d or sh3) else None)
        if not ptr:
            raise GsrError(-3, f"loadGaussianCudaFromPly({path}): {lib().gsr_last_error().decode()}")
        return cls(ptr, n.value, narrays=na.value if (allow_4d or sh3) else SCENE_NARRAYS)

    def download(self) -> np.ndarray:
        soa = np.zeros((self.narrays, self.n), dtype=np.float32)
        check(lib().gsr_scene_download(self.ptr, soa.ctypes.data, self.n), "gsr_scene_download")
        return soa

    def free(self):
        if self.ptr and self.owned:
            lib().gsr_scene_free(self.ptr)
        self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def loadGaussianCudaFromPly(path: str):
    """misc.cu:13-134 -> (device pointer or 0, numGaussians)."""
    n = c_int(0)
    ptr = lib().gsr_load_ply_device(path.encode(), byref(n))
    return (ptr or 0), n.value


def preprocessCUDAGaussians(d_gaussians: int, num_gaussians: int, cam: Camera, num_tile_y: int, num_tile_x: int,
                            width_stride: int, height_stride: int, tile_W: int, tile_H: int,
                            k: float, out: np.ndarray = None) -> np.ndarray:
    """render.cu:871-1157 through the drop-in C symbol; returns the host image (3, H, W).

    `out`: optional persistent C-contiguous float32 (3, H, W) host image to render
    into (the reference viewer's loop reuses one host buffer the same way)."""
    if out is None:
        out = np.zeros((3, tile_H, tile_W), dtype=np.float32)
    elif out.dtype != np.float32 or out.shape != (3, tile_H, tile_W) or not out.flags.c_contiguous:
        raise ValueError(f"out must be C-contiguous float32 (3, {tile_H}, {tile_W})")
    lib().preprocessCUDAGaussians(d_gaussians, out.ctypes.data_as(ctypes.POINTER(c_float)), num_gaussians, cam,
                                  num_tile_y, num_tile_x, width_stride, height_stride, tile_W, tile_H, k)
    return out


def display_gl_current() -> bool:
    """True if a GL context (GLX or EGL) is current on this thread."""
    return bool(lib().gsr_display_gl_current())


class DisplayTarget:
    """Where a frame is displayed (include/gsr_gl.h): the viewer's colour SSBO
    registered with HIP (`from_gl`), or device memory such as an imported
    Vulkan buffer (`from_device`).  The render writes it in place."""

    def __init__(self, ptr: int):
        self.ptr = ptr

    @classmethod
    def from_gl(cls, gl_buffer: int) -> "DisplayTarget":
        p = c_void_p()
        check(lib().gsr_display_register_gl(int(gl_buffer), byref(p)), "gsr_display_register_gl")
        return cls(p.value)

    @classmethod
    def from_device(cls, d_ptr: int, nbytes: int) -> "DisplayTarget":
        p = c_void_p()
        check(lib().gsr_display_wrap_device(d_ptr, int(nbytes), byref(p)), "gsr_display_wrap_device")
        return cls(p.value)

    def free(self):
        if self.ptr:
            p, self.ptr = self.ptr, 0
            check(lib().gsr_display_free(p), "gsr_display_free")

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def preprocessCUDAGaussiansGL(d_gaussians: int, gl_buffer: int, num_gaussians: int, cam: Camera, num_tile_y: int,
                              num_tile_x: int, width_stride: int, height_stride: int, tile_W: int, tile_H: int,
                              k: float) -> None:
    """Canvas::render (canvas.cpp:337-342) into the colour SSBO, no host round trip
    (include/gsr_gl.h).  Needs the viewer's GL context current on this thread."""
    lib().preprocessCUDAGaussiansGL(d_gaussians, int(gl_buffer), num_gaussians, cam, num_tile_y, num_tile_x,
                                    width_stride, height_stride, tile_W, tile_H, k)


def _event_handle(ev, wait: bool = False):
    """hipEvent_t of a torch.cuda.Event, or of a raw integer handle; None -> NULL.
    An event the library records into (wait=False) is created on first use (torch
    creates the HIP event lazily, at its first record).  A wait event that was never
    recorded has nothing to wait for: NULL (recording it here would make the lane wait
    on all work queued on torch's current stream, an implicit fork)."""
    if ev is None:
        return None
    if isinstance(ev, int):
        return ev
    if not ev.cuda_event:
        if wait:
            return None
        ev.record()
    return ev.cuda_event


class Renderer:
    """Persistent render context (stream-ordered, device-resident)."""

    def __init__(self):
        self.ctx = lib().gsr_create()

    def close(self):
        if self.ctx:
            lib().gsr_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reserve(self, n: int, pairs: int):
        check(lib().gsr_reserve(self.ctx, n, pairs), "gsr_reserve")

    def render(self, scene, cam: Camera, W: int, H: int, out_ptr: int, k: float = 3.0, tiling=None,
               stream: int = 0, layout: int = LAYOUT_SCENE_BLOCK, n: int | None = None,
               time: float | None = None) -> int:
        """Enqueue one frame into the device buffer out_ptr (3*W*H float32).
        4D scenes render at `time` (or the last gsr_set_time value).

        Returns GSR_OK, or GSR_E_OVERFLOW when an earlier frame overflowed the
        pair buffer (it has been grown; that frame must be re-rendered)."""
        ptr = scene.ptr if isinstance(scene, Scene) else int(scene)
        n = scene.n if n is None else n
        if isinstance(scene, Scene) and layout == LAYOUT_SCENE_BLOCK:
            layout = scene.layout
        if time is not None:
            self.set_time(time)
        t = tiling or TilingInformation(1, 1, H, W)
        rc = lib().gsr_render(self.ctx, ptr, layout, n, byref(cam), W, H, t.num_tile_x, t.num_tile_y,
                              t.width_stride, t.height_stride, k, out_ptr, stream or None)
        if rc not in (_native.GSR_OK, _native.GSR_E_OVERFLOW):
            raise GsrError(rc, "gsr_render")
        return rc

    def set_frames_in_flight(self, frames: int):
        """Frames render_path runs concurrently (1..8; lanes 1.. own private workspaces)."""
        check(lib().gsr_set_frames_in_flight(self.ctx, int(frames)), "gsr_set_frames_in_flight")

    def frames_in_flight(self) -> int:
        return int(lib().gsr_frames_in_flight(self.ctx))

    def render_path(self, scene, cams, W: int, H: int, out_ptrs, k: float = 3.0, tiling=None, stream: int = 0,
                    layout: int = LAYOUT_SCENE_BLOCK, n: int | None = None, times=None, events=None,
                    join: bool = True, fork: bool = True, wait_events=None, status=None) -> int:
        """Enqueue len(cams) frames (camera cams[i], 4D time times[i]) into the device
        buffers out_ptrs[i] with up to frames_in_flight() of them concurrent
        (gsr_render_path, include/gsr.h).  Stream-ordered on `stream` at entry and exit.
        events (gsr_render_path_ex): per-frame torch.cuda.Event (or None), recorded on
        frame i's lane after its blend; join=False skips the exit join (the caller then
        orders reads and buffer reuse through the events); wait_events[i] (or None): frame
        i's lane waits for it first; fork=False: lanes 1.. do not wait for `stream`.
        status (gsr_render_path_status): per-frame device address (or None) of a uint32
        validity word, 0 when frame i came out complete, else GSR_FRAME_* bits.
        Same returns as render()."""
        ptr = scene.ptr if isinstance(scene, Scene) else int(scene)
        n = scene.n if n is None else n
        if isinstance(scene, Scene) and layout == LAYOUT_SCENE_BLOCK:
            layout = scene.layout
        nf = len(cams)
        if len(out_ptrs) != nf or (times is not None and len(times) != nf):
            raise ValueError("render_path: cams, out_ptrs and times must have the same length")
        cam_arr = (Camera * max(1, nf))(*cams)
        out_arr = (c_void_p * max(1, nf))(*[int(p) for p in out_ptrs])
        t_arr = (c_float * nf)(*[float(t) for t in times]) if times is not None else None
        t = tiling or TilingInformation(1, 1, H, W)
        if events is None and wait_events is None and join and fork and status is None:
            rc = lib().gsr_render_path(self.ctx, ptr, layout, n, cam_arr, t_arr, nf, W, H, t.num_tile_x,
                                       t.num_tile_y, t.width_stride, t.height_stride, k, out_arr, stream or None)
        else:
            if any(x is not None and len(x) != nf for x in (events, wait_events, status)):
                raise ValueError("render_path: events, wait_events and status must have one entry per frame")
            ev_arr = (c_void_p * max(1, nf))(*[_event_handle(e) for e in (events or [None] * nf)])
            wt_arr = (c_void_p * max(1, nf))(*[_event_handle(e, wait=True) for e in (wait_events or [None] * nf)])
            st_arr = (c_void_p * max(1, nf))(*[int(p) if p else None for p in status]) if status else None
            rc = lib().gsr_render_path_status(self.ctx, ptr, layout, n, cam_arr, t_arr, nf, W, H, t.num_tile_x,
                                              t.num_tile_y, t.width_stride, t.height_stride, k, out_arr,
                                              stream or None, ev_arr, wt_arr,
                                              (0 if join else _native.GSR_PATH_NO_JOIN) |
                                              (0 if fork else _native.GSR_PATH_NO_FORK), st_arr)
        if rc not in (_native.GSR_OK, _native.GSR_E_OVERFLOW):
            raise GsrError(rc, "gsr_render_path")
        return rc

    def render_display(self, target: "DisplayTarget", scene, cam: Camera, W: int, H: int, k: float = 3.0,
                       tiling=None, stream: int = 0, layout: int = LAYOUT_SCENE_BLOCK, n: int | None = None,
                       time: float | None = None) -> int:
        """Enqueue one frame straight into a display target (include/gsr_gl.h):
        map, check it holds 3*W*H floats, render, unmap.  Same returns as render()."""
        ptr = scene.ptr if isinstance(scene, Scene) else int(scene)
        n = scene.n if n is None else n
        if isinstance(scene, Scene) and layout == LAYOUT_SCENE_BLOCK:
            layout = scene.layout
        if time is not None:
            self.set_time(time)
        t = tiling or TilingInformation(1, 1, H, W)
        rc = lib().gsr_render_display(self.ctx, target.ptr, ptr, layout, n, byref(cam), W, H, t.num_tile_x,
                                      t.num_tile_y, t.width_stride, t.height_stride, k, stream or None)
        if rc not in (_native.GSR_OK, _native.GSR_E_OVERFLOW):
            raise GsrError(rc, "gsr_render_display")
        return rc

    def set_time(self, t: float):
        check(lib().gsr_set_time(self.ctx, float(t)), "gsr_set_time")

    def preprocess(self, scene, cam: Camera, W: int, H: int, k: float = 3.0, tiling=None, stream: int = 0,
                   layout: int = LAYOUT_SCENE_BLOCK, n: int | None = None, time: float | None = None):
        ptr = scene.ptr if isinstance(scene, Scene) else int(scene)
        n = scene.n if n is None else n
        if isinstance(scene, Scene) and layout == LAYOUT_SCENE_BLOCK:
            layout = scene.layout
        if time is not None:
            self.set_time(time)
        t = tiling or TilingInformation(1, 1, H, W)
        rc = lib().gsr_preprocess(self.ctx, ptr, layout, n, byref(cam), W, H, t.num_tile_x, t.num_tile_y,
                                  t.width_stride, t.height_stride, k, stream or None)
        if rc not in (_native.GSR_OK, _native.GSR_E_OVERFLOW):
            raise GsrError(rc, "gsr_preprocess")

    def sort(self, stream: int = 0):
        check(lib().gsr_sort(self.ctx, stream or None), "gsr_sort")

    def blend(self, out_ptr: int, stream: int = 0):
        check(lib().gsr_blend(self.ctx, out_ptr, stream or None), "gsr_blend")

    def sync(self) -> int:
        rc = lib().gsr_sync(self.ctx)
        if rc not in (_native.GSR_OK, _native.GSR_E_OVERFLOW):
            raise GsrError(rc, "gsr_sync")
        return rc

    def pair_count(self) -> int:
        return int(lib().gsr_pair_count(self.ctx))

    def row_item_count(self) -> int:
        """(tile row, Gaussian) items of the last frame's row pass; -1 on the pair-sort path."""
        return int(lib().gsr_row_item_count(self.ctx))

    def read_splats(self, n: int) -> np.ndarray:
        out = np.zeros(n, dtype=SPLAT_DTYPE)
        check(lib().gsr_read_splats(self.ctx, out.ctypes.data, n), "gsr_read_splats")
        return out

    def read_depth_order(self, n: int) -> np.ndarray:
        out = np.zeros(n, dtype=np.uint64)
        check(lib().gsr_read_depth_order(self.ctx, out.ctypes.data, n), "gsr_read_depth_order")
        return out

    def read_pairs(self) -> np.ndarray:
        cap = max(self.pair_count(), 0)
        out = np.zeros(max(cap, 1), dtype=np.uint64)
        m = lib().gsr_read_pairs(self.ctx, out.ctypes.data, cap)
        if m < 0:
            raise GsrError(int(m), "gsr_read_pairs")
        return out[:m]

    def tile_grid(self):
        tx, ty = c_int(), c_int()
        check(lib().gsr_tile_grid(self.ctx, byref(tx), byref(ty)), "gsr_tile_grid")
        return tx.value, ty.value

    def read_tile_ranges(self) -> np.ndarray:
        tx, ty = self.tile_grid()
        out = np.zeros((tx * ty, 2), dtype=np.uint32)
        check(lib().gsr_read_tile_ranges(self.ctx, out.ctypes.data, tx * ty), "gsr_read_tile_ranges")
        return out

    def set_timing(self, mode: int, stride: int = 1):
        """0 off, 1 blend events, 2 every stage; events on every `stride`-th frame."""
        check(lib().gsr_set_timing_stride(self.ctx, mode, stride), "gsr_set_timing")

    def set_diagnostics(self, on: bool):
        check(lib().gsr_set_diagnostics(self.ctx, int(on)), "gsr_set_diagnostics")

    def blend_records_loaded(self) -> int:
        return int(lib().gsr_blend_records_loaded(self.ctx))

    def blend_counters(self) -> dict:
        v = np.zeros(8, dtype=np.int64)
        check(lib().gsr_blend_counters(self.ctx, v.ctypes.data), "gsr_blend_counters")
        keys = ("records_loaded", "wave_splat_iters", "active_lanes", "taken_lanes", "slow_path_iters",
                "zero_taken_iters", "lane_slots", "no_candidate_pair_iters")
        return dict(zip(keys, (int(x) for x in v)))

    def blend_counters_ex(self) -> dict:
        """blend_counters() plus the fast-exp blend's re-blended blocks and their
        suspect pixels (gsr_blend_counters_ex)."""
        v = np.zeros(16, dtype=np.int64)
        check(lib().gsr_blend_counters_ex(self.ctx, v.ctypes.data, 16), "gsr_blend_counters_ex")
        d = self.blend_counters()
        d["reblended_blocks"], d["suspect_pixels"] = int(v[8]), int(v[9])
        return d

    def take_map(self, W: int, H: int) -> np.ndarray:
        """Per-pixel take map of the last diagnostics frame (gsr_blend_take_map):
        splats composited | (index-mix sum << 32), shape (H, W)."""
        out = np.zeros((H, W), dtype=np.uint64)
        check(lib().gsr_blend_take_map(self.ctx, out.ctypes.data, out.size), "gsr_blend_take_map")
        return out

    def set_blend_variant(self, variant: int):
        check(lib().gsr_set_blend_variant(self.ctx, int(variant)), "gsr_set_blend_variant")

    def set_tuning(self, knob: int, value: int):
        """gsr_set_tuning: 0 blend schedule, 1 tile-sort items/thread, 2 depth-sort items/thread."""
        check(lib().gsr_set_tuning(self.ctx, int(knob), int(value)), "gsr_set_tuning")

    def get_tuning(self, knob: int) -> int:
        """gsr_get_tuning: the knob's current value (the default unless set)."""
        v = ctypes.c_int(0)
        check(lib().gsr_get_tuning(self.ctx, int(knob), ctypes.byref(v)), "gsr_get_tuning")
        return int(v.value)

    def depth_passes(self) -> int:
        """Depth-sort digit passes the last frame ran (trailing identities are skipped)."""
        rc = lib().gsr_depth_passes(self.ctx)
        if rc < 0:
            raise GsrError(rc, "gsr_depth_passes")
        return rc

    def bucket_sizes(self):
        """gsr_bucket_sizes: per-bucket item counts of the last frame when it was
        bucket-sorted (the last bucket: key 0xFFFFFFFF, the culled items), else None."""
        out = np.zeros(MAX_BUCKETS, dtype=np.uint32)
        rc = lib().gsr_bucket_sizes(self.ctx, out.ctypes.data, out.size)
        if rc < 0:
            raise GsrError(rc, "gsr_bucket_sizes")
        return out[:rc] if rc else None

    def blend_stamps(self, n_groups: int) -> np.ndarray:
        """{start, end} s_memrealtime stamps (100 MHz) per blend workgroup of the
        last diagnostics frame rendered with schedule 2 (one per tile) or 3 (one
        per 8x8 block)."""
        out = np.zeros(2 * n_groups, dtype=np.uint64)
        check(lib().gsr_blend_stamps(self.ctx, out.ctypes.data, out.size), "gsr_blend_stamps")
        return out.reshape(n_groups, 2)

    def stage_times(self):
        ms = (ctypes.c_double * NUM_STAGES)()
        frames = c_int64()
        check(lib().gsr_stage_times(self.ctx, ms, byref(frames)), "gsr_stage_times")
        return dict(zip(STAGES, list(ms))), frames.value


def device_available() -> bool:
    return bool(lib().gsr_device_available())


# gsr_set_tuning knobs used by the tests and tools (include/gsr.h lists them all)
TUNE_DEPTH_SORT_ITEMS = 2
TUNE_DEPTH_SORT_GROUPS = 4
TUNE_TILE_BINNING = 7
TUNE_TILE_SPANS = 19
TUNE_RANK_ATOMIC = 20
TUNE_RANK_ATOMIC_ACTIVE = 21
TUNE_BLEND_EXP = 22
TUNE_DEPTH_SPLIT = 23
TUNE_DEPTH_SPLIT_PERMILLE = 24
TUNE_DEPTH_SPLIT_UNSAT = 25
TUNE_DEPTH_SPLIT_STATE = 26
TUNE_DEPTH_BUCKETS = 28
TUNE_DEPTH_BUCKETS_OVER = 29
TUNE_BUCKET_ROWS = 30
TUNE_COL_CHUNK = 31
TUNE_FAIL_FRAME = 32
TUNE_DEPTH_BUCKETS_WORK = 33
MAX_BUCKETS = 4096             # gsr_internal.h kMaxBuckets: the bucket sort's largest bucket count


def rank_order_check() -> tuple[int, int]:
    """gsr_rank_order_check: (lane-operations checked, lanes out of lane order) of the
    device self-check behind the atomic rank path (include/gsr.h)."""
    ops, bad = c_int64(0), c_int64(0)
    check(lib().gsr_rank_order_check(byref(ops), byref(bad)), "gsr_rank_order_check")
    return int(ops.value), int(bad.value)


def math_probe(xy: np.ndarray) -> np.ndarray:
    """Evaluate the gsr_detmath functions on the GPU (see include/gsr.h)."""
    xy = np.ascontiguousarray(xy, dtype=np.float32).reshape(-1, 2)
    out = np.zeros((xy.shape[0], 9), dtype=np.float32)
    check(lib().gsr_math_probe(xy.ctypes.data, xy.shape[0], out.ctypes.data), "gsr_math_probe")
    return out


def exp_probe(x_lo: float, x_hi: float, x_big: float) -> tuple[int, int, float, float]:
    """gsr_exp_probe: (monotonicity violations of gsr_blend_expf, packed-loop exp
    mismatches, max relative fast-exp error, the same over x >= x_big) over every float
    in [x_lo, x_hi), on the GPU."""
    v, pk, ea, eb = c_int64(0), c_int64(0), ctypes.c_float(0), ctypes.c_float(0)
    check(lib().gsr_exp_probe2(x_lo, x_hi, x_big, byref(v), byref(pk), byref(ea), byref(eb)), "gsr_exp_probe2")
    return int(v.value), int(pk.value), float(ea.value), float(eb.value)


def alpha_cut_probe(op: np.ndarray) -> np.ndarray:
    """gsr_alpha_take_min_x evaluated on the GPU for each opacity."""
    op = np.ascontiguousarray(op, dtype=np.float32).ravel()
    out = np.zeros_like(op)
    check(lib().gsr_alpha_cut_probe(op.ctypes.data, op.size, out.ctypes.data), "gsr_alpha_cut_probe")
    return out
