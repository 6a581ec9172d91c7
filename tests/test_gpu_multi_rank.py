"""World-size-2 run of the multi-GPU frame loop (multi.FrameShard, the code behind
bench.py --gpus N) with the HIP renderer: two gloo ranks share cuda:0, each renders
its orbit camera (azimuth 45 deg * rank, camera.cpp:130-158) through
Renderer.render_path with frames in flight, hands every frame to rank 0 per step
(double-buffered chunks, pending-gather reuse), and max-reduces the elapsed time.
Rank 0's gathered frames must equal the oracle's renders of cameras 0 and 1 bit for
bit.  Also: the RCCL branch at world 1, and bench.py --gpus 2 launches two real ranks
and prints n_gpus 2."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import assert_frames
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ply, W, H, steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import gaussianrenderer_amd as gsr
    from gaussianrenderer_amd import multi
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank 0 loads the scene; rank 1 gets the device block by broadcast
    scene = multi.broadcast_scene(dist, gsr.Scene.from_ply(ply) if rank == 0 else None, gloo=True)
    r = gsr.Renderer()
    r.set_frames_in_flight(2)
    cam = multi.orbit_camera(rank, W, H)
    shard = multi.FrameShard(dist, r, scene, cam, W, H, steps=steps, gather="step", inflight=2, chunk=2,
                             gloo=True, stream=torch.cuda.current_stream().cuda_stream)
    shard.run(steps)
    assert not shard.finish("cpu")                 # no rank saw an incomplete frame
    assert shard.gathers == 2                      # one gather per chunk (2 + 1 frames)
    elapsed = multi.max_over_ranks(dist, 0.25 + rank, "cpu")
    if rank == 0:
        q.put((elapsed, [[f.numpy().copy() for f in shard.gathered(b)] for b in range(len(shard.outs))]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_hip_frames_gathered(gpu, orc, tmp_path):
    W, H, world, steps = 320, 240, 2, 3       # chunks of 2: buffers 0, 1 then 2 (second set)
    ply = str(tmp_path / "s.ply")
    gpu.write_synthetic_ply(ply, 10_000, 4)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ply, W, H, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        elapsed, recv = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert elapsed == pytest.approx(1.25)          # MAX over ranks
    soa = gpu.read_ply(ply)
    from gaussianrenderer_amd import multi
    wants = [orc.render(soa, multi.orbit_camera(r, W, H), W, H, 3.0).reshape(-1) for r in range(world)]
    assert not np.array_equal(wants[0], wants[1])
    for b in range(steps):                         # buffers 0, 1 (set 0) and 2 (set 1)
        for r in range(world):
            assert_frames(recv[b][r], wants[r])


def _validity_worker(rank, world, port, ply, W, H, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import gaussianrenderer_amd as gsr
    from gaussianrenderer_amd import multi
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    soa = gsr.read_ply(ply)
    near = gsr.Scene.from_soa(soa)                                   # view depth 3..5: keys < 2^24
    far_soa = soa.copy()
    far_soa[2] = np.linspace(-90.0, 1.0, soa.shape[1], dtype=np.float32)   # keys need all 4 passes
    far = gsr.Scene.from_soa(far_soa)
    r = gsr.Renderer()
    r.set_tuning(gsr.TUNE_BLEND_EXP, 0)      # exact blend: the gathered frames are checked bit for bit
    r.set_tuning(gsr.TUNE_DEPTH_BUCKETS, 0)  # the LSD passes' budget makes the incomplete frames
    r.set_frames_in_flight(2)
    cam = multi.orbit_camera(rank, W, H)
    got, measured = [], [False]

    def sink(cid, i0, frames):
        if measured[0]:
            got.append((cid, [f.cpu().numpy().copy() for f in frames]))

    # rank 1 renders the far scene in chunk 2 of the measured run only
    scene_of = (lambda i: far if (rank == 1 and measured[0] and i // 2 == 2) else near)
    shard = multi.FrameShard(dist, r, near, cam, W, H, steps=6, gather="step", inflight=2, chunk=2, gloo=True,
                             stream=torch.cuda.current_stream().cuda_stream, sink=sink, frame_scene=scene_of)
    for _ in range(8):                         # >= 4 clean checked frames per lane: budget 3 passes
        shard.run(4)
        assert not shard.finish("cpu")
    passes = r.depth_passes()
    measured[0] = True
    shard.run(6)
    first = shard.finish("cpu")
    agreed = list(shard.bad_chunks)
    shard.repair()
    second = shard.finish("cpu")
    q.put((rank, passes, first, agreed, second, shard.repaired, got if rank == 0 else None))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_validity_words_resend_flagged_chunk(gpu, orc, tmp_path):
    """Round-3 verdict item 4: every gathered frame carries its validity word
    (gsr_render_path_status).  Rank 1's lanes run at a 3-pass depth budget, then render
    a scene whose keys need four passes in chunk 2: those frames come out incomplete
    (GSR_FRAME_DEPTH_PASSES).  Both ranks agree on exactly chunk 2, re-render and
    re-gather it; rank 0 ends with every frame bit-exact against the oracle, and only
    chunk 2 was sent twice."""
    W, H, world = 160, 120, 2
    ply = str(tmp_path / "s.ply")
    gpu.write_synthetic_ply(ply, 10_000, 1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_validity_worker, args=(r, world, port, ply, W, H, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            out = q.get(timeout=150)
            res[out[0]] = out[1:]
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert res[1][0] == 3, "rank 1's pass budget was not lowered"
    for rank in range(world):
        _, first, agreed, second, repaired, _ = res[rank]
        assert first and agreed == [2] and not second and repaired == 1
    got = res[0][5]
    assert [c for c, _ in got] == [0, 1, 2, 2]
    soa = gpu.read_ply(ply)
    far_soa = soa.copy()
    far_soa[2] = np.linspace(-90.0, 1.0, soa.shape[1], dtype=np.float32)
    from gaussianrenderer_amd import multi
    npx = 3 * W * H
    cams = [multi.orbit_camera(r, W, H) for r in range(world)]
    want = {(r, f): orc.render(far_soa if f else soa, cams[r], W, H, 3.0).reshape(-1)
            for r in range(world) for f in (0, 1)}
    for k, (cid, frames) in enumerate(got):
        for r in range(world):
            words = frames[r][:, npx].view(np.int32)
            if k == 2 and r == 1:                # the first copy of chunk 2 from rank 1
                assert (words == 2).all(), words
                continue
            assert (words == 0).all(), (cid, r, words)
            for row in frames[r]:
                assert_frames(row[:npx], want[(r, int(r == 1 and cid == 2))], exact=True)


def _nccl_worker(port, ply, W, H, steps, chunk, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import gaussianrenderer_amd as gsr
    from gaussianrenderer_amd import multi
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    scene = gsr.Scene.from_ply(ply)
    r = gsr.Renderer()
    r.set_frames_in_flight(3)
    cam = multi.orbit_camera(0, W, H)
    shard = multi.FrameShard(dist, r, scene, cam, W, H, steps=steps, gather="step", inflight=3, chunk=chunk,
                             stream=torch.cuda.current_stream().cuda_stream)
    assert shard.frame_events is not None          # RCCL: per-frame events, no join
    for _ in range(3):                             # grow the lanes' pair buffers first
        if shard.path(0, 3, [0, 1, 2]) == 0 and r.sync() == 0:
            break
    torch.cuda.synchronize()
    for b in range(len(shard.outs)):
        shard.outs[b].fill_(-1.0)
    torch.cuda.synchronize()
    shard.overflowed = False
    shard.run(steps)
    ok = not shard.finish("cuda") and shard.gathers == (steps + chunk - 1) // chunk
    elapsed = multi.max_over_ranks(dist, 0.5, "cuda")
    q.put((ok, elapsed, [shard.gathered(b)[0].cpu().numpy().copy() for b in range(len(shard.outs))]))
    dist.destroy_process_group()


def test_rccl_world1_frame_events(gpu, orc, tmp_path):
    """The RCCL branch of FrameShard (what bench.py --gpus N runs on a node): one gather
    per chunk, waiting on the completion events of the chunk's frames
    (gsr_render_path_ex), and the lanes do not join between chunks.  World 1 (RCCL
    cannot put two ranks on one GPU): 7 frames in chunks of 3 over two buffer sets, so
    a set is re-used behind its pending gather; every gathered buffer must equal the
    oracle's render (bit for bit with the exact blend)."""
    W, H, steps, chunk = 320, 240, 7, 3
    ply = str(tmp_path / "s.ply")
    gpu.write_synthetic_ply(ply, 10_000, 4)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), ply, W, H, steps, chunk, q))
    p.start()
    try:
        ok, elapsed, recv = q.get(timeout=100)
    finally:
        p.join(timeout=60)
    assert p.exitcode == 0 and ok
    assert elapsed == pytest.approx(0.5)
    soa = gpu.read_ply(ply)
    from gaussianrenderer_amd import multi
    want = orc.render(soa, multi.orbit_camera(0, W, H), W, H, 3.0).reshape(-1)
    assert len(recv) == 2 * chunk
    for b, got in enumerate(recv):
        assert_frames(got, want)


def test_bench_launches_ranks(gpu, tmp_path):
    """bench.py --gpus 2 (no RANK in the environment) starts two ranks itself; gloo so
    both can share the one GPU of a test box.  Rank 0 prints n_gpus 2."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "1",
                          "--steps", "6", "--warmup", "2", "--dist-backend", "gloo", "--chunk", "3",
                          "--scene-dir", str(tmp_path)],
                         capture_output=True, text=True, timeout=110, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    res = lines[0]
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "frames2"
    assert res["value"] > 0 and res["steps"] == 6
    # the line explains itself (per-rank render-only rates, gather time per
    # chunk, DESIGN.md section 8's prediction); 6 frames in chunks of 3: two gathers per rank
    sc = res["scale"]
    fps = sc["per_rank_render_fps"]
    assert len(fps["per_rank"]) == 2 and 0 < fps["min"] <= fps["max"]
    assert all(c >= 2 for c in sc["gather_ms_per_chunk"]["chunks_per_rank"])
    assert sc["gather_ms_per_chunk"]["mean"] > 0
    assert sc["predicted_fps"] == pytest.approx(2 * fps["min"] * (1 - 0.038) * 0.95, rel=1e-3)
