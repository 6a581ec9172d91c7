#!/usr/bin/env python3
"""Where the drop-in frame's time goes (preprocessCUDAGaussians: render + 24.9 MB
device-to-host copy into the caller's pageable image), config 2 on one GPU:

* the whole drop-in call (bench.py's dropin_host_fps);
* the device render alone (gsr_render + sync) and the layout-probe reads;
* hipMemcpy D2H of the image into pageable host memory: whole, and in bands of rows
  (the shape a blend/copy overlap would use), and into pinned memory.

    python tools/dropin_probe.py [--frames 30]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=30)
    a = ap.parse_args()
    import torch
    import bench
    import gaussianrenderer_amd as gsr
    from gaussianrenderer_amd import multi
    n, W, H, seed = bench.CONFIGS[2]
    d = os.path.join(tempfile.gettempdir(), "gsr_bench")
    os.makedirs(d, exist_ok=True)
    ply = os.path.join(d, f"config2_n{n}_s{seed}.ply")
    if not os.path.exists(ply):
        gsr.write_synthetic_ply(ply + ".tmp", n, seed)
        os.replace(ply + ".tmp", ply)
    scene = gsr.Scene.from_ply(ply)
    cam = multi.orbit_camera(0, W, H)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipDeviceSynchronize.argtypes = []
    D2H = 2
    F = a.frames

    def rate(fn, frames=F):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(frames):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / frames * 1e6

    t = gsr.TilingInformation(50, 50, H, W)
    img = gsr.preprocessCUDAGaussians(scene.ptr, scene.n, cam, t.num_tile_y, t.num_tile_x, t.width_stride,
                                      t.height_stride, W, H, 3.0)
    us_dropin = rate(lambda: gsr.preprocessCUDAGaussians(scene.ptr, scene.n, cam, t.num_tile_y, t.num_tile_x,
                                                         t.width_stride, t.height_stride, W, H, 3.0, out=img))
    r = gsr.Renderer()
    out = torch.empty(3 * W * H, device="cuda")

    def render_sync():
        r.render(scene, cam, W, H, out.data_ptr())
        r.sync()
    us_render = rate(render_sync)
    magic = np.zeros(64, np.uint8)
    us_probe = rate(lambda: (hip.hipMemcpy(magic.ctypes.data, scene.ptr, 16, D2H),
                             hip.hipMemcpy(magic.ctypes.data, scene.ptr, 64, D2H)))
    host = np.empty(3 * W * H, np.float32)
    nbytes = host.nbytes
    us_copy = rate(lambda: hip.hipMemcpy(host.ctypes.data, out.data_ptr(), nbytes, D2H))
    res = {}
    for bands in (2, 4, 8):
        rows = (H + bands - 1) // bands

        def banded():
            for b in range(bands):
                y0, y1 = b * rows, min(H, (b + 1) * rows)
                for ch in range(3):
                    off = (ch * H * W + y0 * W) * 4
                    hip.hipMemcpy(host.ctypes.data + off, out.data_ptr() + off, (y1 - y0) * W * 4, D2H)
        res[bands] = rate(banded)
    pinned = torch.empty(3 * W * H, dtype=torch.float32).pin_memory()
    us_pinned = rate(lambda: hip.hipMemcpy(pinned.data_ptr(), out.data_ptr(), nbytes, D2H))
    print(f"drop-in call {us_dropin:.0f} us ({1e6 / us_dropin:.0f} frames/s); render + sync {us_render:.0f} us; "
          f"layout probe reads {us_probe:.0f} us")
    print(f"D2H {nbytes / 1e6:.1f} MB pageable: whole {us_copy:.0f} us ({nbytes / us_copy / 1e3:.1f} GB/s); " +
          "; ".join(f"{b} bands x 3 planes {u:.0f} us" for b, u in res.items()) +
          f"; pinned whole {us_pinned:.0f} us ({nbytes / us_pinned / 1e3:.1f} GB/s)")


if __name__ == "__main__":
    main()
