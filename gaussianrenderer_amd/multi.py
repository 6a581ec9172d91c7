"""Multi-GPU frame sharding (BASELINE config 4): one process per GPU, one orbit
camera per rank, finished frames gathered to rank 0 over torch.distributed
(backend "nccl" = RCCL over xGMI on the MI355X node, "gloo" in CPU tests).

Frames are independent, so the render path has no collective; the only
exchange is the hand-off of finished images to rank 0 (the offline-render
consumer).  SURVEY.md section 8e.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass
class RankInfo:
    rank: int
    world: int
    local_rank: int

    @property
    def is_root(self) -> bool:
        return self.rank == 0


def rank_info() -> RankInfo:
    """RANK / WORLD_SIZE / LOCAL_RANK as set by torch.distributed.run."""
    return RankInfo(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                    int(os.environ.get("LOCAL_RANK", "0")))


def orbit_azimuth(rank: int) -> float:
    """Config 4: camera i orbits by 45 deg * i (Camera::orbit, camera.cpp:130-158)."""
    return 45.0 * rank


def orbit_camera(rank: int, W: int, H: int, position=(0.0, 0.0, 4.0), fov_y: float = 50.0):
    from . import make_camera, orbit
    cam = make_camera(position=position, fov_y=fov_y, aspect=W / H)
    if rank:
        orbit(cam, orbit_azimuth(rank), 0.0)
    return cam


def max_over_ranks(dist, value: float, device) -> float:
    """MAX of a per-rank scalar (the bench's elapsed time) over all ranks."""
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_frames(dist, frame, root: int = 0):
    """Gather every rank's finished frame (same shape) to `root`; returns the
    list of frames on root (index = rank) and None elsewhere."""
    import torch
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [frame]
    world = dist.get_world_size()
    out = [torch.empty_like(frame) for _ in range(world)] if dist.get_rank() == root else None
    dist.gather(frame, out, dst=root)
    return out


class FrameShard:
    """One rank's frame loop for bench.py --gpus N (config 4): K frames of this rank's
    camera through Renderer.render_path (F lanes in flight), and with gather="step"
    every finished frame handed to rank 0 — issued asynchronously (RCCL) right after
    its chunk is enqueued and overlapped with the next chunk's render.

    Buffers: with per-step gathers, two sets of `chunk` output buffers (one set
    renders while the other's gathers drain; a buffer is reused only after its
    pending gather completes); otherwise a ring of F.  On rank 0, `recv[b]` holds
    the last frame gathered from every rank into buffer b.  gloo (the CPU / shared-GPU
    rehearsal) gathers host copies synchronously."""

    def __init__(self, dist, renderer, scene, cam, W: int, H: int, k: float = 3.0, steps: int = 1,
                 gather: str = "step", inflight: int = 1, chunk: int = 8, gloo: bool = False,
                 frame_time=None, stream: int = 0, overlap: bool = True):
        import torch
        self.dist, self.r, self.scene, self.cam = dist, renderer, scene, cam
        self.W, self.H, self.k, self.stream = W, H, k, stream
        self.F = max(1, inflight)
        self.gloo = gloo
        self.frame_time = frame_time
        self.step_gather = dist is not None and gather == "step"
        self.chunk = max(1, chunk) if self.step_gather else max(1, steps)
        self.nsets = 2 if self.step_gather else 1
        self.per_set = self.chunk if self.step_gather else self.F
        self.outs = [torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
                     for _ in range(self.nsets * self.per_set)]
        rank = dist.get_rank() if dist is not None else 0
        world = dist.get_world_size() if dist is not None else 1
        self.recv = ([[torch.empty_like(self.outs[0], device="cpu" if gloo else self.outs[0].device)
                       for _ in range(world)] for _ in range(len(self.outs))]
                     if (self.step_gather and rank == 0) else None)
        if self.recv is not None and not gloo:
            # rank 0's own slot IS its output buffer: the gather's local copy of the
            # root's frame (torch copies input -> gather_list[root]) becomes a no-op,
            # which at world 1 was the whole gather cost (a 24.9-MB device copy per
            # frame competing with the blends).  Same lifetime as the other slots: a
            # buffer is rendered again only after its pending gather completed.
            for b in range(len(self.outs)):
                self.recv[b][0] = self.outs[b]
        self.pending = [None] * len(self.outs)
        # RCCL: each gather waits for its own frame's completion event (gsr_render_path_ex)
        # on a side stream, and render_path runs without the exit join, so the lanes keep
        # frames in flight across chunks instead of draining at every chunk boundary
        self.frame_events = (None if (gloo or not self.step_gather or not overlap)
                             else [torch.cuda.Event() for _ in range(len(self.outs))])
        self.gather_stream = torch.cuda.Stream() if self.frame_events else None
        # ... and buffer b's next frame waits on the completion of b's last gather
        # (recorded on the side stream) instead of the whole path waiting on the caller's
        # stream: the chunked calls skip the fork, which otherwise holds lanes 1.. behind
        # lane 0's frames of the previous call (~4 % of the rate)
        self.gathered = [torch.cuda.Event() for _ in range(len(self.outs))] if self.frame_events else None
        self.gathered_valid = [False] * len(self.outs)

    def _times(self, i0: int, m: int):
        return [self.frame_time(i0 + j) for j in range(m)] if self.frame_time else None

    def wait_pending(self, b: int):
        if self.pending[b] is not None:
            self.pending[b].wait()          # nccl: stream-wait until the gather of buffer b is done
            self.pending[b] = None

    def drain(self):
        for b in range(len(self.outs)):
            self.wait_pending(b)

    def gather(self, b: int):
        if self.frame_events:
            import torch
            # RCCL's stream waits on the current stream: the side stream, which waits
            # on buffer b's frame only
            with torch.cuda.stream(self.gather_stream):
                self.gather_stream.wait_event(self.frame_events[b])
                self.pending[b] = self.dist.gather(self.outs[b], self.recv[b] if self.recv else None, dst=0,
                                                   async_op=True)
                self.pending[b].wait()                       # side stream: after the gather
                self.gathered[b].record(self.gather_stream)
                self.gathered_valid[b] = True
            return
        src = self.outs[b].cpu() if self.gloo else self.outs[b]
        self.pending[b] = self.dist.gather(src, self.recv[b] if self.recv else None, dst=0,
                                           async_op=not self.gloo)

    def frame(self, i: int = 0, b: int = 0):
        """One frame on the caller's stream (sequential: the viewer's one-at-a-time use)."""
        self.r.render(self.scene, self.cam, self.W, self.H, self.outs[b].data_ptr(), k=self.k,
                      stream=self.stream, time=self.frame_time(i) if self.frame_time else None)

    def path(self, i0: int, m: int, bufs, overlap: bool = False, first: bool = True):
        """Frames i0 .. i0+m-1 through gsr_render_path into outs[bufs[j]]; returns its code
        (GSR_E_OVERFLOW: some frame of the call overflowed and must be re-rendered).
        overlap (run()): record each buffer's frame event, skip the exit join, wait per
        frame on the buffer's last gather, and fork from the caller's stream only on the
        first call of a run."""
        ov = overlap and self.frame_events is not None
        waits = [self.gathered[b] if self.gathered_valid[b] else None for b in bufs] if ov else None
        return self.r.render_path(self.scene, [self.cam] * m, self.W, self.H, [self.outs[b].data_ptr() for b in bufs],
                                  k=self.k, stream=self.stream, times=self._times(i0, m),
                                  events=[self.frame_events[b] for b in bufs] if ov else None, join=not ov,
                                  fork=not ov or first, wait_events=waits)

    def run(self, steps: int):
        """K frames in flight, gathered per step when enabled (not drained: call drain())."""
        if not self.step_gather:
            self.path(0, steps, [j % self.F for j in range(steps)])
            return
        for c0 in range(0, steps, self.chunk):
            m = min(self.chunk, steps - c0)
            base = ((c0 // self.chunk) % self.nsets) * self.per_set
            bufs = [base + j for j in range(m)]
            if not self.frame_events:                # gloo: the caller's stream orders reuse
                for b in bufs:
                    self.wait_pending(b)
            self.path(c0, m, bufs, overlap=True, first=c0 == 0)
            for b in bufs:
                self.gather(b)
