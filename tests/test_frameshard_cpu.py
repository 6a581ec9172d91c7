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


def _worker(rank, world, port, imgs, W, H, steps, chunk, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from gaussianrenderer_amd import multi
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got = []

    def sink(cid, i0, frames):
        got.append((cid, i0, [f.numpy().copy() for f in frames]))

    good = {"bad": False}
    bad_chunk2 = {"bad": rank == 1}              # rank 1's frames of chunk 2 come out incomplete once
    r = _StandIn(imgs[rank])
    shard = multi.FrameShard(dist, r, good, None, W, H, steps=steps, gather="step", inflight=2, chunk=chunk,
                             gloo=True, device="cpu", sink=sink,
                             frame_scene=lambda i: bad_chunk2 if i // chunk == 2 else good)
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
