#!/usr/bin/env python3
"""The fast-exp blend's guard on a bench scene: one diagnostics frame, printing the
blocks re-blended exactly, their suspect pixels and the exact one-splat path's
iterations (gsr_blend_counters_ex), for the library GSR_LIBRARY names.

    python tools/fx_suspects.py [--config 2] [--ranks 0 1 ...]  (multi.orbit_camera of each rank)
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--ranks", type=int, nargs="+", default=[0, 3])
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
    stream = torch.cuda.current_stream().cuda_stream
    r = gsr.Renderer()
    r.set_tuning(23, 0)          # GSR_TUNE_DEPTH_SPLIT off: split frames blend exactly
    out = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    lib = os.environ.get("GSR_LIBRARY", "default")
    for rk in a.ranks:
        cam = multi.orbit_camera(rk, W, H)
        # one plain frame first: a renderer's first diagnostics frame reports no counters
        r.render(scene, cam, W, H, out.data_ptr(), stream=stream)
        r.sync()
        r.set_diagnostics(True)
        r.render(scene, cam, W, H, out.data_ptr(), stream=stream)
        r.sync()
        torch.cuda.synchronize()
        c = r.blend_counters_ex()
        r.set_diagnostics(False)
        print(os.path.basename(lib), f"config {a.config} camera of rank {rk}:",
              {k: c[k] for k in ("reblended_blocks", "suspect_pixels", "slow_path_iters", "zero_taken_iters", "no_candidate_pair_iters",
                                 "wave_splat_iters", "taken_lanes")}, flush=True)


if __name__ == "__main__":
    main()
