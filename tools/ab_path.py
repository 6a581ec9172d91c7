#!/usr/bin/env python3
"""Interleaved A/B of the frames-in-flight path (gsr_render_path) in ONE process:
per round, K frames through render_path for every (inflight, cu-reserve)
pair; prints fps per setting and checks every frame equals the sequential image.

    python tools/ab_path.py [--config 2] [--rounds 5] [--frames 200] [--inflight 2 3 4]
                            [--settings 0=0 0=1 14=2,13=4 ...]

A setting is a comma-separated list of gsr_set_tuning knob=value pairs (knobs:
include/gsr.h GSR_TUNE_*; "-" = library defaults; the first setting is the
baseline).  Before each setting every knob that any setting names goes back to
its default (gsr_get_tuning at start), so nothing carries over.  One Renderer
for all settings: separate renderers would put their lane streams on different
hardware-queue assignments and bias the comparison.
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--inflight", type=int, nargs="+", default=[3])
    ap.add_argument("--settings", nargs="+", default=["0=0", "0=1"])
    ap.add_argument("--tol", type=float, default=0.0,
                    help="largest |image - reference| accepted (0: bit-exact; the fast-exp blend, "
                         "GSR_TUNE_BLEND_EXP 1, differs from the exact one by < 1e-6)")
    a = ap.parse_args()
    import torch
    import bench
    import gaussianrenderer_amd as gsr
    from gaussianrenderer_amd import multi
    n, W, H, seed = bench.CONFIGS[a.config]
    d = os.path.join(tempfile.gettempdir(), "gsr_bench")
    os.makedirs(d, exist_ok=True)
    ply = os.path.join(d, f"config{a.config}_n{n}_s{seed}.ply")
    if not os.path.exists(ply):
        gsr.write_synthetic_ply(ply + ".tmp", n, seed)
        os.replace(ply + ".tmp", ply)
    scene = gsr.Scene.from_ply(ply)
    cam = multi.orbit_camera(0, W, H)
    stream = torch.cuda.current_stream().cuda_stream
    r = gsr.Renderer()
    parsed = {m: [tuple(int(x) for x in kv.split("=")) for kv in m.split(",") if kv and kv != "-"]
              for m in a.settings}
    defaults = {kn: r.get_tuning(kn) for kvs in parsed.values() for kn, _ in kvs}
    F = max(a.inflight)
    outs = [torch.empty(3 * W * H, dtype=torch.float32, device="cuda") for _ in range(F)]
    r.render(scene, cam, W, H, outs[0].data_ptr(), stream=stream)
    while r.sync() != 0:
        r.render(scene, cam, W, H, outs[0].data_ptr(), stream=stream)
    torch.cuda.synchronize()
    ref = outs[0].clone()
    res = {}
    for rnd in range(a.rounds + 1):          # round 0 warms every setting up (lane buffers grow)
        for f in a.inflight:
            for m in a.settings:
                for kn, v in defaults.items():
                    r.set_tuning(kn, v)
                for kn, v in parsed[m]:
                    r.set_tuning(kn, v)
                r.set_frames_in_flight(f)
                for o in outs:
                    o.zero_()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                r.render_path(scene, [cam] * a.frames, W, H, [outs[i % f].data_ptr() for i in range(a.frames)],
                              stream=stream)
                torch.cuda.synchronize()
                el = time.perf_counter() - t0
                ov = r.sync()
                for i in range(f):
                    if a.tol > 0:
                        d = (outs[i] - ref).abs().max().item()
                        assert d <= a.tol, f"inflight {f} setting {m}: lane {i} image differs by {d}"
                    else:
                        assert torch.equal(outs[i], ref), f"inflight {f} setting {m}: lane {i} image differs"
                if rnd and not ov:
                    res.setdefault((f, m), []).append(a.frames / el)
    for (f, m), v in sorted(res.items()):
        v = sorted(v)
        print(f"inflight {f} [{m}]: fps median {v[len(v) // 2]:.1f}  all " +
              " ".join(f"{x:.1f}" for x in v), flush=True)


if __name__ == "__main__":
    main()
