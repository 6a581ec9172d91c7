#!/usr/bin/env python3
"""Distribution of per-tile list lengths (16x16 tiles) for the bench configs:
sizes a per-tile LDS sort would see.  python tools/tile_lengths.py [--configs 2 3 5]"""
import argparse
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {2: (1_000_000, 1920, 1080, 2, False), 3: (5_000_000, 1600, 1063, 3, False),
           5: (2_000_000, 1920, 1080, 5, True)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", type=int, nargs="+", default=[2, 3, 5])
    a = ap.parse_args()
    import numpy as np
    import torch
    import gaussianrenderer_amd as gsr
    from gaussianrenderer_amd import multi
    for c in a.configs:
        n, W, H, seed, four_d = CONFIGS[c]
        d = os.path.join(tempfile.gettempdir(), "gsr_bench")
        os.makedirs(d, exist_ok=True)
        ply = os.path.join(d, f"config{c}_n{n}_s{seed}{'_4d' if four_d else ''}.ply")
        if not os.path.exists(ply):
            (gsr.write_synthetic_ply4d if four_d else gsr.write_synthetic_ply)(ply + ".tmp", n, seed)
            os.replace(ply + ".tmp", ply)
        scene = gsr.Scene.from_ply(ply)
        r = gsr.Renderer()
        out = torch.empty(3 * W * H, device="cuda")
        for cam_i in (0, 3):
            cam = multi.orbit_camera(cam_i, W, H)
            while True:
                r.render(scene, cam, W, H, out.data_ptr(), time=0.5 if four_d else None)
                if r.sync() == 0:
                    break
            rg = r.read_tile_ranges().reshape(-1, 2).astype(np.int64)
            ln = rg[:, 1] - rg[:, 0]                 # [start, end) per tile
            q = np.percentile(ln, [50, 90, 99, 99.9, 100])
            print(f"config {c} cam {cam_i}: tiles {ln.size} pairs {ln.sum()} mean {ln.mean():.0f} "
                  f"p50/p90/p99/p99.9/max {q.astype(int).tolist()} "
                  f">2048: {(ln > 2048).sum()} >4096: {(ln > 4096).sum()} >8192: {(ln > 8192).sum()} "
                  f"pairs in >4096 tiles: {ln[ln > 4096].sum()}", flush=True)


if __name__ == "__main__":
    main()
