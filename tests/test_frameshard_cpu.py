"""CPU (gloo, world 2) test of FrameShard's per-frame validity protocol
(gaussianrenderer_amd/multi.py, the loop behind bench.py --gpus N, config 4): every
gathered frame carries its validity word (gsr_render_path_status) right after its
image; finish() agrees over ranks on the chunks that hold an incomplete frame, and
repair() re-renders and re-gathers exactly those.  A stand-in renderer writes the
oracle's frames through the same buffer addresses the HIP library would, and reports
one chunk of rank 1 incomplete once (as a depth sort short of passes does: code
GSR_E_OVERFLOW, word GSR_FRAME_DEPTH_PASSES, clean when rendered again).  The GPU
twin with the HIP renderer is tests/test_gpu_multi_rank.py."""
import ctypes
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


class _StandIn:
    """render_path with the library's buffer contract: image floats at each output
    address, the validity word at each status address."""

    def __init__(self, img):
        self.img = img
        self.calls = []

    def render_path(self, scene, cams, W, H, ptrs, status=None, **_):
        rc = 0
        for j, p in enumerate(ptrs):
            out = np.ctypeslib.as_array((ctypes.c_float * self.img.size).from_address(p))
            word = 0
            if scene.get("bad"):
                out[:] = -1.0                     # an incomplete frame: wrong pixels
                word = 2                          # GSR_FRAME_DEPTH_PASSES
            else:
                out[:] = self.img
            if status:
                ctypes.c_uint32.from_address(status[j]).value = word
        if scene.get("bad"):
            scene["bad"] = False                  # the pass budget is back at four
            rc = -5
        self.calls.append(len(ptrs))
        return rc

    def sync(self):
        return 0


def _worker(rank, world, port, imgs, W, H, steps, chunk, q, flags=None, every=1):
    """flags: {rank: [chunk ids]} whose frames come out incomplete once on that rank
    (default: chunk 2 of rank 1)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from gaussianrenderer_amd import multi
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got = []

    def sink(cid, i0, frames):
        got.append((cid, i0, [f.numpy().copy() for f in frames]))

    flags = {1: [2]} if flags is None else flags
    good = {"bad": False}
    scenes = {c: {"bad": True} for c in flags.get(rank, [])}
    r = _StandIn(imgs[rank])
    shard = multi.FrameShard(dist, r, good, None, W, H, steps=steps, gather="step", inflight=2, chunk=chunk,
                             gloo=True, device="cpu", sink=sink, gather_every=every,
                             frame_scene=lambda i: scenes.get(i // chunk, good))
    assert shard.validity
    shard.run(steps)
    first = shard.finish("cpu")
    agreed = list(shard.bad_chunks)
    shard.repair()
    second = shard.finish("cpu")
    q.put((rank, first, agreed, second, shard.repaired, shard.gathers, r.calls, got if rank == 0 else None))
    dist.barrier()
    dist.destroy_process_group()


def test_frameshard_resends_only_the_flagged_chunk(tmp_path):
    W, H, world, steps, chunk = 16, 12, 2, 7, 2          # chunks 0..3 (the last one of 1 frame)
    rng = np.random.default_rng(5)
    imgs = [rng.random(3 * W * H, dtype=np.float32) for _ in range(world)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, imgs, W, H, steps, chunk, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            out = q.get(timeout=120)
            res[out[0]] = out[1:]
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for rank in range(world):
        first, agreed, second, repaired, gathers, calls, _ = res[rank]
        assert first and agreed == [2], "both ranks agree on exactly chunk 2"
        assert not second and repaired == 1
        assert gathers == 4 + 1                          # four chunks, then chunk 2 once more
        assert calls == [2, 2, 2, 1, 2]                  # the re-render is chunk 2's two frames only
    got = res[0][6]
    assert [g[0] for g in got] == [0, 1, 2, 3, 2]        # rank 0's sink: every chunk, chunk 2 again
    npx = 3 * W * H
    for cid, i0, frames in got:
        assert i0 == chunk * cid
        for r in range(world):
            block = frames[r]
            words = block[:, npx].view(np.int32)
            if cid == 2 and r == 1 and (cid, i0) == (got[2][0], got[2][1]) and frames is got[2][2]:
                assert (words == 2).all()                # the incomplete frames, flagged as such
                assert (block[:, :npx] == -1.0).all()
            else:
                assert (words == 0).all()
                assert np.array_equal(block[:, :npx], np.broadcast_to(imgs[r], block[:, :npx].shape))


def _run_world(world, steps, chunk, flags, every=1, W=8, H=6):
    rng = np.random.default_rng(world)
    imgs = [rng.random(3 * W * H, dtype=np.float32) for _ in range(world)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, imgs, W, H, steps, chunk, q, flags, every))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            out = q.get(timeout=240)
            res[out[0]] = out[1:]
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    return imgs, res


@pytest.mark.parametrize("world,flags", [(8, {7: [1]}), (8, {3: [0], 5: [2]}), (4, {3: [1], 2: [3]})])
def test_frameshard_validity_at_world(world, flags):
    """Round-4 verdict item 3: the validity protocol at world 4 and 8.  Ranks flag one
    chunk (rank 7) or different chunks (ranks 3 and 5; 3 and 2): every rank agrees on the
    same bad_chunks (the union), re-renders and re-gathers exactly those; rank 0's sink
    sees each flagged chunk twice (first with the flagged rank's words set and its
    pixels wrong, then clean) and every other chunk once, every clean frame bit-equal to
    its rank's image."""
    steps, chunk = 8, 2                                  # chunks 0..3
    imgs, res = _run_world(world, steps, chunk, flags)
    want_bad = sorted({c for cs in flags.values() for c in cs})
    n_chunks = steps // chunk
    for rank in range(world):
        first, agreed, second, repaired, gathers, calls, _ = res[rank]
        assert first and agreed == want_bad, (rank, agreed)
        assert not second and repaired == len(want_bad)
        assert gathers == n_chunks + len(want_bad)
        assert calls == [chunk] * (n_chunks + len(want_bad))
    got = res[0][6]
    assert [g[0] for g in got] == list(range(n_chunks)) + want_bad
    npx = 3 * W_H(got)
    seen = {}
    for cid, i0, frames in got:
        assert i0 == chunk * cid
        k = seen.get(cid, 0)
        seen[cid] = k + 1
        for r in range(world):
            block = frames[r]
            words = block[:, npx].view(np.int32)
            if k == 0 and cid in flags.get(r, []):
                assert (words == 2).all() and (block[:, :npx] == -1.0).all()
            else:
                assert (words == 0).all(), (cid, r, words)
                assert np.array_equal(block[:, :npx], np.broadcast_to(imgs[r], block[:, :npx].shape))
    assert all(seen[c] == (2 if c in want_bad else 1) for c in range(n_chunks))


def W_H(got):
    """Pixels per frame (W * H) from the gathered rows (image + status pad)."""
    from gaussianrenderer_amd.multi import STATUS_PAD
    return (got[0][2][0].shape[1] - STATUS_PAD) // 3


def test_frameshard_gather_every_kth_chunk():
    """--gather-every K (rank 0's inbound xGMI budget): only every
    K-th chunk is gathered; the others stay on their rank, but their validity words still
    count, so a flagged chunk that is not gathered is re-rendered (and, not being a
    gathered chunk, still not sent)."""
    world, steps, chunk, every = 4, 8, 2, 2               # chunks 0..3: 0 and 2 gathered
    flags = {1: [1], 2: [2]}
    imgs, res = _run_world(world, steps, chunk, flags, every=every)
    for rank in range(world):
        first, agreed, second, repaired, gathers, calls, _ = res[rank]
        assert first and agreed == [1, 2]
        assert not second and repaired == 2
        assert gathers == 2 + 1                            # chunks 0 and 2, chunk 2 again
        assert calls == [chunk] * 6
    got = res[0][6]
    assert [g[0] for g in got] == [0, 2, 2]
