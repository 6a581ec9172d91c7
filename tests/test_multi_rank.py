"""World-size-2 gloo test (CPU) of the multi-GPU frame-sharding path
(gaussianrenderer_amd/multi.py, used by bench.py --gpus N): each rank renders
its own orbit camera — here with the CPU oracle standing in for the GPU — the
frames are gathered to rank 0 and the elapsed time is max-reduced."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ply, W, H, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    import gaussianrenderer_amd as gsr
    from gaussianrenderer_amd import multi
    import _oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    info = multi.rank_info()
    assert (info.rank, info.world) == (rank, world)
    soa = gsr.read_ply(ply)
    cam = multi.orbit_camera(info.rank, W, H)
    frame = torch.from_numpy(_oracle.render(soa, cam, W, H, 3.0, threads=1)).reshape(-1)
    elapsed = multi.max_over_ranks(dist, 0.5 + rank, "cpu")
    # the overflow agreement behind FrameShard.finish: any rank's flag reaches every rank
    assert multi.any_over_ranks(dist, rank == 1, "cpu") is True
    assert multi.any_over_ranks(dist, False, "cpu") is False
    frames = multi.gather_frames(dist, frame)
    if info.is_root:
        q.put((elapsed, [f.numpy().copy() for f in frames]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_two_rank_orbit_gather(gsr, orc, tmp_path, world):
    """World 2 as before, and 4 and 8 ranks (the driver's scaling run): every rank's
    orbit frame reaches rank 0 in rank order, the elapsed time is the max over ranks."""
    W, H = 96, 64
    ply = str(tmp_path / "s.ply")
    gsr.write_synthetic_ply(ply, 3000, 4)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ply, W, H, q)) for r in range(world)]
    for p in procs:
        p.start()
    elapsed, frames = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert elapsed == pytest.approx(0.5 + world - 1)   # MAX over ranks
    soa = gsr.read_ply(ply)
    from gaussianrenderer_amd import multi
    for r in range(world):
        want = orc.render(soa, multi.orbit_camera(r, W, H), W, H, 3.0, threads=1).reshape(-1)
        assert np.array_equal(frames[r], want)
    for r in range(1, world):
        assert not np.array_equal(frames[0], frames[r])   # different orbit cameras


def _scale_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from gaussianrenderer_amd import multi
    dist.init_process_group("gloo", rank=rank, world_size=world)
    steps = 200
    render_el = 0.05 + 0.01 * rank                       # rank r renders 200 frames in 50 + 10 r ms
    headline_el = multi.max_over_ranks(dist, 0.08 + 0.005 * rank, "cpu")   # with gathers: slower
    gathers = [1.0 + rank, 2.0 + rank, 3.0 + rank]      # ms per chunk on this rank's side stream
    rep = multi.scale_report(dist, render_el, steps, gathers, world * steps / headline_el, "cpu")
    if rank == 0:
        q.put((rep, world * steps / headline_el))
    else:
        assert rep is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_scale_report_fields(world):
    """the N > 1 bench line's 'scale' object (multi.scale_report, a
    collective) on gloo ranks: per-rank render-only rates (min / max over ranks), the gather
    time per chunk, and DESIGN.md section 8's prediction, with value <= world * min rate."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scale_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    rep, value = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    fps = rep["per_rank_render_fps"]
    want = [200 / (0.05 + 0.01 * r) for r in range(world)]
    assert fps["per_rank"] == pytest.approx(want, rel=1e-6)
    assert fps["min"] == pytest.approx(min(want)) and fps["max"] == pytest.approx(max(want))
    g = rep["gather_ms_per_chunk"]
    assert g["chunks_per_rank"] == [3] * world
    assert g["per_rank_mean"] == pytest.approx([2.0 + r for r in range(world)])
    assert g["mean"] == pytest.approx(2.0 + (world - 1) / 2) and g["max"] == pytest.approx(3.0 + world - 1)
    assert rep["render_bound_fps"] == pytest.approx(world * min(want), rel=1e-6)
    assert value <= rep["render_bound_fps"]
    assert rep["value_over_render_bound"] == pytest.approx(value / (world * min(want)), rel=1e-3)
    assert rep["predicted_fps"] == pytest.approx(world * min(want) * (1 - 0.038) * 0.95, rel=1e-4)
