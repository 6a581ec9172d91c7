"""Depth split on a scene with background (analysis tool): the config-3 scene with the
camera turned off centre (look_at (X, 0, 0)), so part of the image sees past the
scene and never saturates.  Frames one at a time (gsr_render) and with 4 frames in
flight (gsr_render_path), split on (default) and off, interleaved; prints frames/s,
the split state and point.  Usage: python tools/split_bg_bench.py [X ...]"""
import os
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gaussianrenderer_amd as gsr  # noqa: E402

N, W, H, SEED = 5_000_000, 1600, 1063, 3
FRAMES, WARM = 200, 300


def rate(r, scene, cam, outs, inflight):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if inflight:
        for i in range(0, FRAMES, 8):
            r.render_path(scene, [cam] * 8, W, H, [o.data_ptr() for o in outs])
    else:
        for i in range(FRAMES):
            r.render(scene, cam, W, H, outs[i % len(outs)].data_ptr())
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    rc = r.sync()
    if rc:
        rc = (rc, gsr.lib().gsr_last_error().decode(errors="replace"))
    return FRAMES / el, rc


def main():
    looks = [float(a) for a in sys.argv[1:]] or [0.0, 1.2, 2.0]
    global FRAMES, WARM
    FRAMES = int(os.environ.get("FRAMES", FRAMES))
    WARM = int(os.environ.get("WARM", WARM))
    ply = os.path.join(tempfile.gettempdir(), f"split_bg_{N}_{SEED}.ply")
    if not os.path.exists(ply):
        gsr.write_synthetic_ply(ply, N, SEED)
    scene = gsr.Scene.from_ply(ply)
    outs = [torch.empty(3 * W * H, dtype=torch.float32, device="cuda") for _ in range(8)]
    for x in looks:
        cam = gsr.make_camera(position=(0, 0, 4), look_at=(x, 0, 0), fov_y=50, aspect=W / H)
        res = {}
        for rnd in range(2):
            for split in [int(v) for v in os.environ.get("PMS", "2 0").split()]:
                r = gsr.Renderer()
                # PMS entries: 2 = the default controller, 0 = split off, > 2 = forced split
                # starting at that split point (the controller still moves it)
                r.set_tuning(gsr.TUNE_DEPTH_SPLIT, split if split <= 2 else 1)
                if split > 2:
                    r.set_tuning(gsr.TUNE_DEPTH_SPLIT_PERMILLE, split)
                r.set_frames_in_flight(4)
                for i in range(WARM):   # the controller settles; every lane's buffers grow
                    r.render_path(scene, [cam] * 8, W, H, [o.data_ptr() for o in outs]) if i % 2 else \
                        r.render(scene, cam, W, H, outs[0].data_ptr())
                    if i % 16 == 15:
                        r.sync()
                r.sync()
                seq, rc1 = rate(r, scene, cam, outs, False)
                inf, rc2 = rate(r, scene, cam, outs, True)
                st = (r.get_tuning(gsr.TUNE_DEPTH_SPLIT_STATE), r.get_tuning(gsr.TUNE_DEPTH_SPLIT_PERMILLE),
                      r.get_tuning(gsr.TUNE_DEPTH_SPLIT_UNSAT))
                res.setdefault(split, []).append((round(inf, 1), round(seq, 1), st, rc1, rc2))
                r.close()
        for split, v in res.items():
            print(f"look_at x={x}: split {'on ' if split else 'off'} in flight / one at a time / "
                  f"(state, split point, unsaturated blocks) / overflow rc: {v}", flush=True)


if __name__ == "__main__":
    main()
