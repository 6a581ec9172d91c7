#!/usr/bin/env python3
"""Frames in flight: throughput of F independent contexts on F HIP streams,
frames dealt round-robin (frame i -> context i % F), vs F = 1.

    python tools/inflight_probe.py [--frames 200] [--inflight 1 2 3]

Every context owns its workspace, so frames on different streams share only the
(read-only) scene; the GPU overlaps one frame's latency-bound sort/binning
kernels with another frame's VALU-bound blend.  Images are checked equal to
the F = 1 image (same camera).
"""
import argparse
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--inflight", type=int, nargs="+", default=[1, 2, 3, 4])
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    import gaussianrenderer_amd as gsr
    n, W, H, seed = 1_000_000, 1920, 1080, 2
    d = os.path.join(tempfile.gettempdir(), "gsr_bench")
    os.makedirs(d, exist_ok=True)
    ply = os.path.join(d, f"config2_n{n}_s{seed}.ply")
    if not os.path.exists(ply):
        gsr.write_synthetic_ply(ply + ".tmp", n, seed)
        os.replace(ply + ".tmp", ply)
    scene = gsr.Scene.from_ply(ply)
    cam = gsr.make_camera(aspect=W / H) if "aspect" in gsr.make_camera.__code__.co_varnames else None
    from gaussianrenderer_amd import multi
    cam = multi.orbit_camera(0, W, H)
    F = max(a.inflight)
    rs = [gsr.Renderer() for _ in range(F)]
    streams = [torch.cuda.Stream() for _ in range(F)]
    outs = [torch.empty(3 * W * H, dtype=torch.float32, device="cuda") for _ in range(F)]
    for f in range(F):
        for _ in range(5):
            rs[f].render(scene, cam, W, H, outs[f].data_ptr(), stream=streams[f].cuda_stream)
        while rs[f].sync() != 0:
            rs[f].render(scene, cam, W, H, outs[f].data_ptr(), stream=streams[f].cuda_stream)
    torch.cuda.synchronize()
    ref = outs[0].clone()
    res = {k: [] for k in a.inflight}
    for _ in range(a.rounds):
        for k in a.inflight:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.frames):
                f = i % k
                rs[f].render(scene, cam, W, H, outs[f].data_ptr(), stream=streams[f].cuda_stream)
            torch.cuda.synchronize()
            res[k].append(a.frames / (time.perf_counter() - t0))
            for f in range(k):
                assert torch.equal(outs[f], ref), f"inflight {k}: context {f} image differs"
    for k in a.inflight:
        print(f"inflight {k}: fps " + " ".join(f"{v:.1f}" for v in res[k]) + f"  best {max(res[k]):.1f}", flush=True)

    # stage split over two streams per context: preprocess + sort on one, blend on the
    # other, with the given priorities (HIP: lower number = higher priority)
    lo_p, hi_p = torch.cuda.Stream.priority_range()
    print(f"stream priority range: low {lo_p} high {hi_p}", flush=True)
    for name, ps, pb in (("split equal", 0, 0), ("split sort-high", hi_p, lo_p), ("split blend-high", lo_p, hi_p)):
        for k in a.inflight:
            if k == 1:
                continue
            ss = [torch.cuda.Stream(priority=ps) for _ in range(k)]
            sb = [torch.cuda.Stream(priority=pb) for _ in range(k)]
            ev_sorted = [torch.cuda.Event() for _ in range(k)]
            ev_done = [torch.cuda.Event() for _ in range(k)]
            best = []
            for _ in range(a.rounds):
                torch.cuda.synchronize()
                for f in range(k):
                    ev_done[f].record(sb[f])
                t0 = time.perf_counter()
                for i in range(a.frames):
                    f = i % k
                    ss[f].wait_event(ev_done[f])
                    rs[f].preprocess(scene, cam, W, H, stream=ss[f].cuda_stream)
                    rs[f].sort(stream=ss[f].cuda_stream)
                    ev_sorted[f].record(ss[f])
                    sb[f].wait_event(ev_sorted[f])
                    rs[f].blend(outs[f].data_ptr(), stream=sb[f].cuda_stream)
                    ev_done[f].record(sb[f])
                torch.cuda.synchronize()
                best.append(a.frames / (time.perf_counter() - t0))
                for f in range(k):
                    assert torch.equal(outs[f], ref), f"{name} {k}: context {f} image differs"
            print(f"{name} inflight {k}: fps " + " ".join(f"{v:.1f}" for v in best) + f"  best {max(best):.1f}",
                  flush=True)


if __name__ == "__main__":
    main()
