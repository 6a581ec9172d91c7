#!/usr/bin/env python3
"""RCCL rehearsal of the multi-GPU frame loop on whatever GPUs one box has.

bench.py --gpus N uses the nccl (= RCCL) backend only when N > 1, and RCCL cannot
put two ranks on one GPU, so on a one-GPU box the RCCL code path of
multi.FrameShard (one async gather per chunk on RCCL's stream, gather-done waits
before a buffer set is reused, the max-reduce of the elapsed time on a device tensor) would
first run in the driver's 8-GPU scaling run.  This script runs that path with
however many ranks the launcher starts (one per GPU; world 1 is enough to exercise
every call) and checks the gathered frames bit for bit against a plain render of
each rank's camera:

    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 \\
        --master-port 29512 tools/nccl_rehearsal.py [--steps 20]
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--gaussians", dest="n", type=int, default=200_000)
    ap.add_argument("--W", type=int, default=1280)
    ap.add_argument("--H", type=int, default=720)
    ap.add_argument("--chunk", type=int, default=8)
    ap.add_argument("--inflight", type=int, default=4)
    ap.add_argument("--gather", choices=("step", "none"), default="step",
                    help="none: the same frames with no gathers (one render_path call, the N=1 bench loop)")
    ap.add_argument("--warm-ms", type=float, default=0.0, help="untimed sustained frames before the timed ones")
    ap.add_argument("--no-gather-calls", action="store_true",
                    help="diagnostic: the chunked per-step loop without issuing the gathers (no buffer check)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="render_path joins at every chunk (the drain the per-frame events remove)")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    from gaussianrenderer_amd import multi
    info = multi.rank_info()
    torch.cuda.set_device(info.local_rank)
    dist.init_process_group("nccl", device_id=torch.device("cuda", info.local_rank))
    import gaussianrenderer_amd as gsr
    ply = os.path.join(tempfile.gettempdir(), f"nccl_rehearsal_{a.n}.ply")
    if info.local_rank == 0 and not os.path.exists(ply):
        gsr.write_synthetic_ply(ply + ".tmp", a.n, 4)
        os.replace(ply + ".tmp", ply)
    dist.barrier()
    scene = gsr.Scene.from_ply(ply)
    W, H = a.W, a.H
    cam = multi.orbit_camera(info.rank, W, H)
    r = gsr.Renderer()
    r.set_frames_in_flight(a.inflight)
    stream = torch.cuda.current_stream().cuda_stream
    shard = multi.FrameShard(dist, r, scene, cam, W, H, steps=a.steps, gather=a.gather, inflight=a.inflight, chunk=a.chunk,
                             stream=stream, overlap=not a.no_overlap)
    if a.no_gather_calls:
        shard.gather = lambda s, m, cid=0, i0=0: None
    # reference image of this rank's camera (grows the pair buffers too)
    ref = torch.empty(3 * W * H, device="cuda")
    for _ in range(3):
        r.render(scene, cam, W, H, ref.data_ptr(), stream=stream)
        if r.sync() == 0:
            break
    for _ in range(3):            # warm the lanes (their pair buffers grow on overflow)
        rc = shard.path(0, 8, [j % len(shard.outs) for j in range(8)])
        if r.sync() == 0 and rc == 0:
            break
    torch.cuda.synchronize()
    w0 = time.perf_counter()
    while (time.perf_counter() - w0) * 1e3 < a.warm_ms:
        shard.run(a.steps)
        shard.drain()
        torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    shard.run(a.steps)
    t_enq = time.perf_counter() - t0          # host time to enqueue the frames and gathers
    shard.drain()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    assert not shard.finish("cuda"), "overflow in the timed frames"
    mx = multi.max_over_ranks(dist, elapsed, "cuda")
    # every rank's reference to rank 0, compared with what the per-step gathers delivered
    refs = multi.gather_frames(dist, ref)
    ok = True
    if info.rank == 0 and (shard.recv is None or a.no_gather_calls):
        print(f"nccl rehearsal: world {info.world}, {a.steps} frames per rank, no gathers; "
              f"{info.world * a.steps / mx:.1f} frames/s aggregate ({a.inflight} lanes, warm {a.warm_ms:.0f} ms, "
              f"{'chunked step loop without gather calls, ' if a.no_gather_calls else ''}"
              f"host enqueue {t_enq * 1e3:.2f} ms)",
              flush=True)
    elif info.rank == 0:
        used = sorted({(c0 // shard.chunk % shard.nsets) * shard.per_set + j
                       for c0 in range(0, a.steps, shard.chunk) for j in range(min(shard.chunk, a.steps - c0))})
        for b in used:
            for src in range(info.world):
                same = torch.equal(shard.gathered(b)[src], refs[src])
                ok = ok and same
                if not same:
                    print(f"MISMATCH buffer {b} rank {src}", flush=True)
        print(f"nccl rehearsal: world {info.world}, {a.steps} frames per rank, {len(used)} buffers checked, "
              f"{'bit-exact' if ok else 'FAILED'}; {info.world * a.steps / mx:.1f} frames/s aggregate "
              f"(max elapsed {mx * 1e3:.2f} ms, host enqueue {t_enq * 1e3:.2f} ms, {'join per chunk' if a.no_overlap else 'frame events, no join'}, "
              f"chunk {a.chunk}, {a.inflight} lanes, "
              f"HW queues {os.environ.get('GPU_MAX_HW_QUEUES', 'default')}, warm {a.warm_ms:.0f} ms, {W}x{H}, n {a.n})", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
