#!/usr/bin/env python3
"""Trace the depth split's controller on a bench scene: the split point and state
(GSR_TUNE_DEPTH_SPLIT_PERMILLE / _STATE) after every frame, for frames one at a time
and for batches through gsr_render_path, printing only the changes and every
GSR_E_OVERFLOW (a speculative frame that left blocks unsaturated, or a grown buffer).

    python tools/split_trace.py [--config 3] [--frames 3000] [--inflight 4] [--diag-every 0]
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KNOB_PM, KNOB_UNSAT, KNOB_STATE = 24, 25, 26


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--frames", type=int, default=3000)
    ap.add_argument("--inflight", type=int, default=4)
    ap.add_argument("--diag-every", type=int, default=0,
                    help="a diagnostics frame (gsr_set_diagnostics) every N frames one at a time, as bench.py runs one")
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
    F = a.inflight
    outs = [torch.empty(3 * W * H, dtype=torch.float32, device="cuda") for _ in range(F)]
    last = None

    def note(tag, i, rc):
        nonlocal last
        cur = (r.get_tuning(KNOB_STATE), r.get_tuning(KNOB_PM))
        if cur != last or rc != 0:
            print(f"{tag} frame {i}: rc {rc} state {cur[0]} permille {cur[1]} unsat {r.get_tuning(KNOB_UNSAT)}",
                  flush=True)
            last = cur

    for i in range(a.frames):
        diag = a.diag_every and i % a.diag_every == a.diag_every - 1
        if diag:
            r.set_diagnostics(True)
        r.render(scene, cam, W, H, outs[0].data_ptr(), stream=stream)
        rc = r.sync()
        if diag:
            r.set_diagnostics(False)
            print(f"diag frame {i}: pairs {r.pair_count()} state {r.get_tuning(KNOB_STATE)}", flush=True)
        note("one", i, rc)
    for b in range(a.frames // (4 * F)):
        rc = r.render_path(scene, [cam] * (4 * F), W, H, [outs[j % F].data_ptr() for j in range(4 * F)],
                           stream=stream)
        rc2 = r.sync()
        note("path", b * 4 * F, rc or rc2)
    torch.cuda.synchronize()
    print("end", r.get_tuning(KNOB_STATE), r.get_tuning(KNOB_PM), flush=True)


if __name__ == "__main__":
    main()
