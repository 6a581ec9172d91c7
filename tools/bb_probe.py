#!/usr/bin/env python3
"""Big-bucket probe (analysis only): config 3 on an orbit with knob 28 = BUCKETS (default 1: big buckets), per frame the
largest live bucket, its index, the edge buckets and the items the global path took."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import gaussianrenderer_amd as gsr
    n, W, H = 5_000_000, 1600, 1063
    d = "/tmp/gsr_bench"
    os.makedirs(d, exist_ok=True)
    ply = os.path.join(d, f"config3_n{n}_s3.ply")
    if not os.path.exists(ply):
        gsr.write_synthetic_ply(ply, n, 3)
    scene = gsr.Scene.from_ply(ply)
    r = gsr.Renderer()
    r.set_tuning(gsr.TUNE_DEPTH_SPLIT, 0)
    r.set_tuning(gsr.TUNE_DEPTH_BUCKETS, int(os.environ.get("BUCKETS", "1")))
    for kv in filter(None, os.environ.get("TUNE", "").split(",")):   # more knobs: "31=4096,..."
        k, v = kv.split("=")
        r.set_tuning(int(k), int(v))
    out = torch.empty(3 * W * H, device="cuda")
    for i in range(int(os.environ.get("FRAMES", "24"))):
        c = gsr.make_camera(position=(0, 0, 4), fov_y=50, aspect=W / H)
        gsr.orbit(c, 0.25 * i, 0.0)
        o0 = r.get_tuning(gsr.TUNE_DEPTH_BUCKETS_OVER)
        r.render(scene, c, W, H, out.data_ptr())
        r.sync()
        s = r.bucket_sizes()
        over = r.get_tuning(gsr.TUNE_DEPTH_BUCKETS_OVER) - o0
        if s is None:
            print(i, "LSD frame", flush=True)
            continue
        live = s[:-1]
        top = np.argsort(live)[-4:][::-1]
        print(i, "max", int(live.max()), "at", [int(t) for t in top], [int(live[t]) for t in top],
              "edges", int(live[0]), int(live[-1]), "mean", round(float(live.mean()), 1), "over", over, flush=True)


if __name__ == "__main__":
    main()
