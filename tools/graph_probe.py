#!/usr/bin/env python3
"""Launch-overhead probe: the same config-2 frame rendered K times with direct
launches vs captured once into a HIP graph (torch.cuda.graph on the render
stream) and replayed K times.  Prints ms/frame for both and checks the images
are bit-identical.  Experiment only (the captured frame bakes its camera)."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    import gaussianrenderer_amd as gsr
    n, W, H, seed = bench.CONFIGS[2]
    d = os.path.join(tempfile.gettempdir(), "gsr_bench")
    os.makedirs(d, exist_ok=True)
    ply = os.path.join(d, f"config2_n{n}_s{seed}.ply")
    if not os.path.exists(ply):
        gsr.write_synthetic_ply(ply, n, seed)
    scene = gsr.Scene.from_ply(ply)
    cam = gsr.make_camera(position=(0.0, 0.0, 4.0), fov_y=50.0, aspect=W / H)
    r = gsr.Renderer()
    out = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(5):
            r.render(scene, cam, W, H, out.data_ptr(), stream=s.cuda_stream)
        while r.sync() != 0:
            r.render(scene, cam, W, H, out.data_ptr(), stream=s.cuda_stream)
    ref = out.cpu().numpy().view(np.uint32).copy()
    r.set_tuning(11, 0)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        r.render(scene, cam, W, H, out.data_ptr(), stream=s.cuda_stream)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    same = bool(np.array_equal(out.cpu().numpy().view(np.uint32), ref))
    K = 200
    res = {"direct": [], "graph": []}
    for rnd in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            for _ in range(K):
                r.render(scene, cam, W, H, out.data_ptr(), stream=s.cuda_stream)
        torch.cuda.synchronize()
        res["direct"].append((time.perf_counter() - t0) / K * 1e3)
        t0 = time.perf_counter()
        for _ in range(K):
            g.replay()
        torch.cuda.synchronize()
        res["graph"].append((time.perf_counter() - t0) / K * 1e3)
    print(json.dumps({"identical": same, "ms_per_frame": {k: sorted(v)[2] for k, v in res.items()}}))


if __name__ == "__main__":
    main()
