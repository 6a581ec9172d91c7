#!/usr/bin/env python3
"""Interleaved A/B of one gsr_set_tuning knob in ONE process: per round, K
frames per value with every stage timed (gsr_set_timing(2)); prints per-stage
medians per value and checks the images are bit-identical across values.

    python tools/ab_tune.py --knob 1 --values 16,8 [--config 2] [--rounds 5] [--k-frames 30]

knobs: 0 blend schedule, 1 tile-sort items/thread, 2 depth-sort items/thread.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--knob", type=int, required=True)
    ap.add_argument("--values", required=True)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--k-frames", type=int, default=30)
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import gaussianrenderer_amd as gsr

    n, W, H, seed = bench.CONFIGS[args.config]
    d = os.path.join(tempfile.gettempdir(), "gsr_bench")
    os.makedirs(d, exist_ok=True)
    ply = os.path.join(d, f"config{args.config}_n{n}_s{seed}.ply")
    if not os.path.exists(ply):
        gsr.write_synthetic_ply(ply, n, seed)
    scene = gsr.Scene.from_ply(ply)
    cam = gsr.make_camera(position=(0.0, 0.0, 4.0), fov_y=50.0, aspect=W / H)
    values = [int(v) for v in args.values.split(",")]
    r = gsr.Renderer()
    out = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    for _ in range(3):
        r.render(scene, cam, W, H, out.data_ptr())
    while r.sync() != 0:
        r.render(scene, cam, W, H, out.data_ptr())
    ref, same = None, {}
    for v in values:
        r.set_tuning(args.knob, v)
        r.render(scene, cam, W, H, out.data_ptr())
        r.sync()
        img = out.cpu().numpy().view(np.uint32).copy()
        ref = img if ref is None else ref
        same[v] = bool(np.array_equal(img, ref))
    res = {v: {} for v in values}
    for rnd in range(args.rounds):
        for v in values:
            r.set_tuning(args.knob, v)
            for _ in range(3):
                r.render(scene, cam, W, H, out.data_ptr())
            r.sync()
            r.set_timing(2)
            for _ in range(args.k_frames):
                r.render(scene, cam, W, H, out.data_ptr())
            ms, frames = r.stage_times()
            r.set_timing(0)
            for k, x in ms.items():
                res[v].setdefault(k, []).append(x / max(1, frames))
        print(f"round {rnd}: " + "; ".join(f"{v}: " + ", ".join(f"{k} {res[v][k][-1]:.4f}" for k in res[v])
                                           for v in values), flush=True)
    summary = {v: {k: round(sorted(x)[len(x) // 2], 4) for k, x in res[v].items()} for v in values}
    for v in values:
        summary[v]["total"] = round(sum(summary[v].values()), 4)
        summary[v]["identical_to_first"] = same[v]
    print(json.dumps({"config": args.config, "knob": args.knob, "median_ms": summary}, indent=1))


if __name__ == "__main__":
    main()
