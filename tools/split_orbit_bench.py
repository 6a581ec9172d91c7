"""Depth split on a moving camera (analysis tool): the config-3 scene rendered along an
orbit (STEP degrees per frame) through gsr_render_path with 4 frames in flight, split on
(default) and off, interleaved.  Frames that come back GSR_E_OVERFLOW (a speculative
frame that needed phase B, or a pair buffer that grew) are rendered again, as the
re-render contract asks, and counted.  Prints frames/s including those re-renders.
Usage: python tools/split_orbit_bench.py [STEP ...]"""
import os
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gaussianrenderer_amd as gsr  # noqa: E402

N, W, H, SEED = 5_000_000, 1600, 1063, 3
FRAMES = int(os.environ.get("FRAMES", 400))
CHUNK = 8


def run(r, scene, cams, outs):
    """All frames in chunks of CHUNK; a chunk whose check reports an overflow is rendered
    again (every frame since the last clean check).  Returns (seconds, re-rendered chunks)."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    redo = 0
    for c0 in range(0, len(cams), CHUNK):
        chunk = cams[c0:c0 + CHUNK]
        for _ in range(4):
            rc = r.render_path(scene, chunk, W, H, [o.data_ptr() for o in outs[:len(chunk)]])
            if rc == 0 and r.sync() == 0:
                break
            redo += 1
    torch.cuda.synchronize()
    return time.perf_counter() - t0, redo


def main():
    steps = [float(a) for a in sys.argv[1:]] or [0.25, 1.0]
    ply = os.path.join(tempfile.gettempdir(), f"split_orbit_{N}_{SEED}.ply")
    if not os.path.exists(ply):
        gsr.write_synthetic_ply(ply, N, SEED)
    scene = gsr.Scene.from_ply(ply)
    outs = [torch.empty(3 * W * H, dtype=torch.float32, device="cuda") for _ in range(CHUNK)]
    for step in steps:
        cams = []
        for i in range(FRAMES):
            cam = gsr.make_camera(position=(0, 0, 4), fov_y=50, aspect=W / H)
            gsr.orbit(cam, step * i, 0.0)
            cams.append(cam)
        res = {}
        for rnd in range(2):
            for split in (2, 0):
                r = gsr.Renderer()
                r.set_tuning(gsr.TUNE_DEPTH_SPLIT, split)
                r.set_frames_in_flight(4)
                run(r, scene, cams[:64], outs)             # warm: buffers grow, the split settles
                el, redo = run(r, scene, cams, outs)
                res.setdefault(split, []).append((round(FRAMES / el, 1), redo, r.get_tuning(gsr.TUNE_DEPTH_SPLIT_STATE),
                                                  r.get_tuning(gsr.TUNE_DEPTH_SPLIT_PERMILLE)))
                r.close()
        for split, v in res.items():
            print(f"orbit {step} deg/frame: split {'on ' if split else 'off'} frames/s, re-rendered chunks, "
                  f"state, split point: {v}", flush=True)


if __name__ == "__main__":
    main()
