#!/usr/bin/env python3
"""Blend workgroup timeline (per-wave s_memrealtime stamps of the one-wave-per-
8x8-block kernel, blend schedule 3).

Reports the kernel span, the workgroup-duration distribution, how many
workgroups were in flight over time, and the share of the span spent in the
drain (fewer workgroups in flight than the device holds).

    python tools/blend_timeline.py [--config 2] [--orbit DEG]
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
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--orbit", type=float, default=0.0)
    ap.add_argument("--resident", type=int, default=2048, help="workgroups the device holds at once")
    ap.add_argument("--schedule", type=int, default=3, choices=(3,))
    ap.add_argument("--band-tiles", type=int, default=None, help="schedule 3: GSR_TUNE_BLEND_BAND_TILES value")
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
    r = gsr.Renderer()
    out = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    for _ in range(3):
        r.render(scene, cam, W, H, out.data_ptr())
    r.sync()
    r.set_blend_variant(args.schedule)
    if args.band_tiles is not None:
        r.set_tuning(13, args.band_tiles)
    r.set_diagnostics(True)
    res = []
    for rep in range(3):
        r.render(scene, cam, W, H, out.data_ptr())
        r.sync()
        tx, ty = r.tile_grid()
        # schedule 3: the grid may be padded (band layout): read it whole, skip blocks
        # that exited without stamps
        st = r.blend_stamps(6 * tx * ty + 32 if args.schedule == 3 else tx * ty).astype(np.int64)
        keep = st[:, 0] != 0
        xcd = np.nonzero(keep)[0] % 8
        st = st[keep]
        place = None
        if args.schedule == 3:   # second word: duration (40 bits) | placement << 40
            place = (st[:, 1] >> 40).astype(np.int64)
            st[:, 1] = st[:, 0] + (st[:, 1] & ((1 << 40) - 1))
        t0 = st[:, 0].min()
        s, e = (st[:, 0] - t0) * 10.0, (st[:, 1] - t0) * 10.0       # 100 MHz -> ns
        span = e.max()
        dur = e - s
        # in-flight count over time
        ev = np.concatenate([np.stack([s, np.ones_like(s)], 1), np.stack([e, -np.ones_like(e)], 1)])
        ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
        t, c = ev[:, 0], np.cumsum(ev[:, 1])
        full = c >= 0.95 * args.resident
        last_full = t[np.where(full)[0][-1]] if full.any() else 0.0
        area = dur.sum() / (args.resident * span)
        res.append({"span_us": round(span / 1e3, 2), "wg": int(len(s)),
                    "dur_us": {"mean": round(dur.mean() / 1e3, 2), "p50": round(float(np.median(dur)) / 1e3, 2),
                               "p95": round(float(np.percentile(dur, 95)) / 1e3, 2),
                               "max": round(dur.max() / 1e3, 2)},
                    "max_in_flight": int(c.max()),
                    "drain_us": round((span - last_full) / 1e3, 2),
                    "occupancy_area": round(float(area), 3),
                    "last_start_us": round(s.max() / 1e3, 2),
                    "in_flight_by_tenth": [int(c[np.searchsorted(t, span * (q + 0.5) / 10.0) - 1]) for q in range(10)],
                    "starts_by_tenth": np.histogram(s, bins=10, range=(0, span))[0].tolist(),
                    "dur_by_start_tenth_us": [round(float(dur[(s >= span * q / 10) & (s < span * (q + 1) / 10)].mean()) / 1e3, 1)
                                              if ((s >= span * q / 10) & (s < span * (q + 1) / 10)).any() else 0.0
                                              for q in range(10)],
                    # hardware dispatch sends workgroup b to XCD b % 8
                    "xcd_end_us": [round(float(e[xcd == x].max()) / 1e3, 1) for x in range(8)],
                    "xcd_busy_us": [round(float(dur[xcd == x].sum()) / 1e3 / 1024, 1) for x in range(8)]})
        if place is not None:
            # HW_ID (gfx9 layout): wave 3:0, SIMD 5:4, CU 11:8, SH 12, SE 15:13; XCC above
            cu = place >> 8   # XCC / SE / SH / CU
            cus, inv = np.unique(cu, return_inverse=True)
            mid = span * 0.5
            live = (s <= mid) & (e >= mid)
            per_cu_mid = np.bincount(inv[live], minlength=len(cus))
            res[-1]["cus_seen"] = int(len(cus))
            res[-1]["waves_per_cu_at_mid"] = {"min": int(per_cu_mid.min()), "mean": round(float(per_cu_mid.mean()), 2),
                                              "max": int(per_cu_mid.max()),
                                              "hist": np.bincount(per_cu_mid).tolist()}
            slot = place & 0xF
            res[-1]["wave_slot_ids_seen"] = sorted(set(slot.tolist()))
    print(json.dumps({"config": args.config, "runs": res}, indent=1))


if __name__ == "__main__":
    main()
