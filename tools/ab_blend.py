#!/usr/bin/env python3
"""Interleaved A/B timing of blend builds / schedules (gsr_set_blend_variant: 0, or 3
with timeline stamps) in ONE
process on one scene: every round renders K frames per variant (HIP events
around each blend launch), so clock/thermal drift hits all variants alike.
Also checks that every variant's image is bit-identical to variant 0's and
prints each variant's diagnostics counters.

    python tools/ab_blend.py [--config 2] [--variants 0,...] [--rounds 5] [--k-frames 40]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--variants", default="0")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--k-frames", type=int, default=40)
    ap.add_argument("--orbit", type=float, default=0.0, help="orbit azimuth (deg) of the camera")
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
    if args.orbit:
        gsr.orbit(cam, args.orbit, 0.0)
    variants = [int(v) for v in args.variants.split(",")]
    r = gsr.Renderer()
    out = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        r.render(scene, cam, W, H, out.data_ptr(), stream=stream)
    while r.sync() != 0:
        r.render(scene, cam, W, H, out.data_ptr(), stream=stream)

    ref = None
    report = {}
    for v in variants:
        r.set_blend_variant(v)
        r.set_diagnostics(True)
        r.render(scene, cam, W, H, out.data_ptr(), stream=stream)
        r.sync()
        c = r.blend_counters()
        r.set_diagnostics(False)
        img = out.cpu().numpy().copy()
        if ref is None:
            ref = img
        same = bool(np.array_equal(img.view(np.uint32), ref.view(np.uint32)))
        report[v] = {"identical_to_first": same, "counters": c,
                     "lane_eff": round(c["active_lanes"] / max(1, c["lane_slots"]), 4), "ms": []}
    for rnd in range(args.rounds):
        for v in variants:
            r.set_blend_variant(v)
            for _ in range(3):
                r.render(scene, cam, W, H, out.data_ptr(), stream=stream)
            r.sync()
            r.set_timing(1)
            for _ in range(args.k_frames):
                r.render(scene, cam, W, H, out.data_ptr(), stream=stream)
            ms, frames = r.stage_times()
            r.set_timing(0)
            report[v]["ms"].append(ms["blend"] / max(1, frames))
        print(f"round {rnd}: " + ", ".join(f"v{v} {report[v]['ms'][-1]:.4f}" for v in variants), flush=True)
    for v in variants:
        ms = sorted(report[v]["ms"])
        report[v]["median_ms"] = round(ms[len(ms) // 2], 4)
        report[v]["ms"] = [round(x, 4) for x in report[v]["ms"]]
    print(json.dumps({"config": args.config, "orbit": args.orbit, "variants": report}, indent=1))


if __name__ == "__main__":
    main()
