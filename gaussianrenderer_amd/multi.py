"""Multi-GPU frame sharding (BASELINE config 4): one process per GPU, one orbit
camera per rank, finished frames gathered to rank 0 over torch.distributed
(backend "nccl" = RCCL over xGMI on the MI355X node, "gloo" in CPU tests).

Frames are independent, so the render path has no collective; the exchanges are
the scene's replication at load (one broadcast of the device scene block from
rank 0) and the hand-off of finished images to rank 0 (the offline-render
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


def any_over_ranks(dist, flag: bool, device) -> bool:
    """True on every rank if `flag` is true on any rank (a collective: every rank calls it)."""
    return max_over_ranks(dist, 1.0 if flag else 0.0, device) > 0.0


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


def broadcast_scene(dist, scene, gloo: bool = False):
    """Replicate rank 0's device scene block on every rank (one
    broadcast at load instead of N ranks parsing the .ply).  `scene` is rank 0's
    loaded Scene (ignored elsewhere).  The block (header + SoA arrays, one
    allocation) travels whole; each rank gets a Scene over a torch-owned copy.
    gloo stages the block through host memory."""
    import torch
    from . import Scene, check, lib
    rank = dist.get_rank() if dist is not None and dist.is_initialized() else 0
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return scene
    dev = "cpu" if gloo else "cuda"
    meta = torch.tensor([scene.n, scene.narrays] if rank == 0 else [0, 0], dtype=torch.int64, device=dev)
    dist.broadcast(meta, 0)
    n, narrays = (int(v) for v in meta.tolist())
    nbytes = int(lib().gsr_scene_bytes(narrays, n))
    if nbytes <= 0:
        raise RuntimeError(f"broadcast_scene: bad scene size ({narrays} arrays, {n} Gaussians)")
    block = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    if rank == 0:
        check(lib().gsr_scene_copy(block.data_ptr(), scene.ptr, narrays, n,
                                   torch.cuda.current_stream().cuda_stream), "gsr_scene_copy")
    if gloo:
        host = block.cpu()
        dist.broadcast(host, 0)
        block.copy_(host)
    else:
        dist.broadcast(block, 0)
    torch.cuda.synchronize()
    out = Scene(block.data_ptr(), n, owned=False, narrays=narrays)
    out.storage = block          # the torch allocation backs the scene's pointer
    return out


# DESIGN.md section 8's prediction of the N-GPU rate: the per-chunk gathers cost one GPU
# 3.8 % at world 1 (profiles/r03_reh_chunks.txt), and rank 0's receive kernels beside its
# own render are budgeted at 5 %.
GATHER_COST_WORLD1 = 0.038
RANK0_RECEIVE_BUDGET = 0.95


def scale_report(dist, render_elapsed: float, render_steps: int, gather_ms, value: float, device) -> dict | None:
    """The self-explaining part of an N > 1 bench line (a collective: every rank calls it;
    rank 0 gets the dict, the others None).

    render_elapsed: this rank's wall time for render_steps frames in flight with no
    gathers (its render-only rate); gather_ms: this rank's per-chunk gather durations on
    the side stream during the headline region (from the frames being done to the gather's
    completion: the wire time plus the wait for the slowest rank); value: the headline
    whole-job rate.  Reports the per-rank render-only rates (min / max), the gather time
    per chunk, and DESIGN.md section 8's predicted rate from the slowest rank's render-only
    rate: world * R1 * 0.95 with R1 = that rate * (1 - 0.038)."""
    import torch
    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
    rank = dist.get_rank() if world > 1 else 0
    fps = render_steps / render_elapsed if render_elapsed > 0 else 0.0
    g = [float(x) for x in (gather_ms or [])]
    t = torch.tensor([fps, sum(g) / len(g) if g else 0.0, max(g) if g else 0.0, float(len(g))],
                     dtype=torch.float64, device=device)
    rows = [t]
    if world > 1:
        rows = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(rows, t)
    if rank != 0:
        return None
    per = [r.tolist() for r in rows]
    fmin = min(r[0] for r in per)
    r1 = fmin * (1.0 - GATHER_COST_WORLD1)
    predicted = world * r1 * RANK0_RECEIVE_BUDGET
    return {
        "per_rank_render_fps": {"min": round(fmin, 3), "max": round(max(r[0] for r in per), 3),
                                "per_rank": [round(r[0], 3) for r in per], "frames_per_rank": render_steps,
                                "note": "frames in flight with no gathers, untimed for the headline, after it"},
        "gather_ms_per_chunk": {"mean": round(sum(r[1] * r[3] for r in per) / max(1.0, sum(r[3] for r in per)), 4),
                                "max": round(max(r[2] for r in per), 4),
                                "per_rank_mean": [round(r[1], 4) for r in per],
                                "chunks_per_rank": [int(r[3]) for r in per],
                                "note": "side stream, from the chunk's frames done to its gather complete (wire "
                                        "time + the wait for the slowest rank), headline region"},
        "render_bound_fps": round(world * fmin, 3),
        "value_over_render_bound": round(value / (world * fmin), 4) if fmin > 0 else None,
        "predicted_fps": round(predicted, 1),
        "predicted_formula": (f"world * R1 * {RANK0_RECEIVE_BUDGET} with R1 = min per-rank render fps * "
                              f"(1 - {GATHER_COST_WORLD1}) (DESIGN.md section 8)"),
    }


# Floats after each image in a FrameShard buffer: word 0 is the frame's validity word
# (gsr_render_path_status: 0 complete, else GSR_FRAME_* bits); the pad keeps the next
# image 256-B aligned when the image is.
STATUS_PAD = 64


class FrameShard:
    """One rank's frame loop for bench.py --gpus N (config 4): K frames of this rank's
    camera through Renderer.render_path (F lanes in flight), and with gather="step"
    the finished frames handed to rank 0 — one gather per CHUNK of frames, issued
    asynchronously right after the chunk is enqueued and overlapped with the next
    chunk's render.

    Buffers: with per-step gathers, two SETS of `chunk` frames, each set one
    contiguous [chunk, 3*H*W + STATUS_PAD] tensor (one set renders while the other's
    gather drains; a set is rendered again only after its gather completed); otherwise
    a ring of F frames.  On rank 0, `recv[s][r]` is rank r's copy of set s
    (`gathered(b)` lists buffer b's frame from every rank).  gloo (the CPU /
    shared-GPU rehearsal) gathers host copies synchronously.

    Validity (per-step gathers): every frame's validity word (gsr_render_path_status)
    sits right after its image, so it travels in the same gather; each rank also logs
    its own words per frame.  finish() — a collective — drains, then agrees over ranks
    on the CHUNKS that hold an incomplete frame on any rank (GSR_E_OVERFLOW: pair buffer
    grown, a depth sort short of passes, a speculative depth-split miss), and repair()
    re-renders and re-gathers exactly those chunks on every rank (the gathers are
    collectives).  run_checked() does run + finish + repair until clean.  A consumer on
    rank 0 passes sink(chunk_id, first_frame, frames): frames[r] is rank r's
    [m, 3*H*W + STATUS_PAD] block of the chunk (word 3*H*W of a row: its status, int32
    view), called once per gather, repaired chunks again.

    Without per-step gathers the renderer's codes are the only signal: finish() reports
    whether any rank saw GSR_E_OVERFLOW since the last finish (re-run everything)."""

    def __init__(self, dist, renderer, scene, cam, W: int, H: int, k: float = 3.0, steps: int = 1,
                 gather: str = "step", inflight: int = 1, chunk: int = 8, gloo: bool = False,
                 frame_time=None, stream: int = 0, overlap: bool = True, sink=None, frame_scene=None,
                 device: str = "cuda", frame_cam=None, gather_every: int = 1):
        import torch
        self.dist, self.r, self.scene, self.cam = dist, renderer, scene, cam
        self.W, self.H, self.k, self.stream = W, H, k, stream
        self.F = max(1, inflight)
        self.gloo = gloo
        self.device = device
        self.frame_time = frame_time
        self.frame_scene = frame_scene
        self.frame_cam = frame_cam               # frame index -> camera (a moving viewer), else cam
        self.step_gather = dist is not None and gather == "step"
        # rank 0's inbound budget: gather only every k-th chunk; the
        # others stay on their rank, their validity words still count in finish()
        self.gather_every = max(1, int(gather_every))
        self.chunk = max(1, chunk) if self.step_gather else max(1, steps)
        self.nsets = 2 if self.step_gather else 1
        self.per_set = self.chunk if self.step_gather else self.F
        self.npx = npx = 3 * W * H
        self.validity = self.step_gather
        row = npx + STATUS_PAD if self.validity else npx
        self.sets = [torch.empty((self.per_set, row), dtype=torch.float32, device=device)
                     for _ in range(self.nsets)]
        self.outs = [self.sets[s][j, :npx] for s in range(self.nsets) for j in range(self.per_set)]
        self.status_ptrs = ([self.sets[s][j, npx:].data_ptr() for s in range(self.nsets) for j in range(self.per_set)]
                            if self.validity else None)
        self.rank = dist.get_rank() if dist is not None else 0
        self.world = dist.get_world_size() if dist is not None else 1
        self.recv = None
        if self.step_gather and self.rank == 0:
            # rank 0's own slot IS its set: torch's gather copies input -> gather_list[root],
            # a no-op when they alias (at world 1 that copy was the whole gather cost)
            self.recv = [[self.sets[s] if (r == 0 and not gloo) else
                          torch.empty_like(self.sets[s], device="cpu" if gloo else device)
                          for r in range(self.world)] for s in range(self.nsets)]
        self.pending = [None] * self.nsets
        # RCCL: a chunk's gather waits, on a side stream, for the completion events of the
        # chunk's frames (gsr_render_path_ex), and render_path runs without the exit
        # join, so the lanes keep frames in flight across chunks
        self.frame_events = (None if (gloo or not self.step_gather or not overlap or device != "cuda")
                             else [torch.cuda.Event() for _ in range(len(self.outs))])
        self.gather_stream = torch.cuda.Stream() if self.frame_events else None
        # ... and a set's next frames wait on the completion of the set's last gather
        # (recorded on the side stream) instead of the whole path waiting on the caller's
        # stream: the chunked calls skip the fork, which otherwise holds lanes 1.. behind
        # lane 0's frames of the previous call (~4 % of the rate)
        self.gathered_ev = [torch.cuda.Event() for _ in range(self.nsets)] if self.frame_events else None
        self.gathered_valid = [False] * self.nsets
        self.sink = sink if self.recv is not None else None
        self.undelivered = [None] * self.nsets          # (chunk id, first frame, m) gathered into set s
        self.chunks = []                                # (first frame, m) per chunk id, since run()
        self.status_log = None                          # this rank's validity word per frame index
        self.bad_chunks = []
        self.overflowed = False
        self.gathers = 0
        self.repaired = 0
        # per-chunk gather timing (time_gathers): (start, end) timing events on the side
        # stream (RCCL), or host milliseconds (synchronous gloo gathers)
        self.time_gathers = False
        self.gather_marks = []

    def _times(self, i0: int, m: int):
        return [self.frame_time(i0 + j) for j in range(m)] if self.frame_time else None

    def gathered(self, b: int):
        """Rank 0: buffer b's frame from every rank (index = rank), as device/host views."""
        s, j = divmod(b, self.per_set)
        return [self.recv[s][r][j][:self.npx] for r in range(self.world)]

    def _sync(self):
        if self.device == "cuda":
            import torch
            torch.cuda.synchronize()

    def wait_pending(self, s: int):
        if self.pending[s] is not None:
            self.pending[s].wait()          # nccl: stream-wait until the gather of set s is done
            self.pending[s] = None

    def _deliver(self, s: int):
        """Rank 0 with a sink: hand set s's last gathered chunk to it (stream-ordered after
        that gather)."""
        u = self.undelivered[s]
        if u is None:
            return
        self.undelivered[s] = None
        if self.frame_events:
            import torch
            torch.cuda.current_stream().wait_event(self.gathered_ev[s])
        else:
            self.wait_pending(s)
        cid, i0, m = u
        self.sink(cid, i0, [t[:m] for t in self.recv[s]])

    def gather_ms(self) -> list:
        """Milliseconds of every timed gather since time_gathers was set (synchronizes)."""
        out = []
        for m in self.gather_marks:
            if isinstance(m, tuple):
                m[1].synchronize()
                out.append(m[0].elapsed_time(m[1]))
            else:
                out.append(m)
        return out

    def drain(self):
        for s in range(self.nsets):
            self.wait_pending(s)
            if self.sink:
                self._deliver(s)

    def _log_status(self, s: int, i0: int, m: int):
        """This rank's validity words of frames i0..i0+m-1 (in set s) into status_log, on
        the current stream (after the frames: the side stream waited on their events, or
        the caller's stream joined the lanes)."""
        import torch
        if self.status_log is None or self.status_log.numel() < i0 + m:
            old = self.status_log
            self.status_log = torch.zeros(max(i0 + m, 2 * (old.numel() if old is not None else 0)),
                                          dtype=torch.int32, device=self.device)
            if old is not None:
                self.status_log[:old.numel()].copy_(old)
        self.status_log[i0:i0 + m].copy_(self.sets[s][:m, self.npx].view(torch.int32))

    def gather(self, s: int, m: int, cid: int = 0, i0: int = 0):
        """One gather of frames 0..m-1 of set s (chunk cid, first frame i0) to rank 0."""
        self.gathers += 1
        src = self.sets[s][:m]
        dst = None
        if self.recv:
            # rank 0's slot is the very tensor object it sends (torch then skips the copy)
            dst = [src if t is self.sets[s] else t[:m] for t in self.recv[s]]
        if self.frame_events:
            import torch
            # RCCL's stream waits on the current stream: the side stream, which waits on
            # the chunk's frames only (the last frame of each lane covers its lane)
            with torch.cuda.stream(self.gather_stream):
                for j in range(max(0, m - self.F), m):
                    self.gather_stream.wait_event(self.frame_events[s * self.per_set + j])
                self._log_status(s, i0, m)
                if self.time_gathers:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(self.gather_stream)
                self.pending[s] = self.dist.gather(src, dst, dst=0, async_op=True)
                self.pending[s].wait()                       # side stream: after the gather
                if self.time_gathers:
                    e1.record(self.gather_stream)
                    self.gather_marks.append((e0, e1))
                self.gathered_ev[s].record(self.gather_stream)
                self.gathered_valid[s] = True
        else:
            self._log_status(s, i0, m)
            import time
            t0 = time.perf_counter()
            if self.gloo:
                self.pending[s] = self.dist.gather(src.cpu(), dst, dst=0)
            else:
                self.pending[s] = self.dist.gather(src, dst, dst=0, async_op=True)
            if self.time_gathers and self.gloo:
                self.gather_marks.append((time.perf_counter() - t0) * 1e3)
        if self.sink:
            self.undelivered[s] = (cid, i0, m)
            if not self.frame_events:
                self._deliver(s)

    def keep_local(self, s: int, m: int, i0: int = 0):
        """A chunk that is not gathered (gather_every > 1): only its validity words are
        logged, after its frames, and the set's reuse waits on that like on a gather."""
        if self.frame_events:
            import torch
            with torch.cuda.stream(self.gather_stream):
                for j in range(max(0, m - self.F), m):
                    self.gather_stream.wait_event(self.frame_events[s * self.per_set + j])
                self._log_status(s, i0, m)
                self.gathered_ev[s].record(self.gather_stream)
                self.gathered_valid[s] = True
        else:
            self._log_status(s, i0, m)

    def frame(self, i: int = 0, b: int = 0):
        """One frame on the caller's stream (sequential: the viewer's one-at-a-time use)."""
        rc = self.r.render(self.frame_scene(i) if self.frame_scene else self.scene,
                           self.frame_cam(i) if self.frame_cam else self.cam, self.W, self.H,
                           self.outs[b].data_ptr(), k=self.k, stream=self.stream,
                           time=self.frame_time(i) if self.frame_time else None)
        self.overflowed |= rc != 0
        return rc

    def path(self, i0: int, m: int, bufs, overlap: bool = False, first: bool = True, wait_set=None):
        """Frames i0 .. i0+m-1 through gsr_render_path into outs[bufs[j]]; returns its code
        (GSR_E_OVERFLOW: some frame since the last clean check came out incomplete).
        overlap (run()): record each buffer's frame event, skip the exit join, wait on
        the last gather of set `wait_set`, and fork from the caller's stream only on the
        first call of a run.  Buffers with a validity word get it written."""
        ov = overlap and self.frame_events is not None
        waits = None
        if ov and wait_set is not None and self.gathered_valid[wait_set]:
            waits = [self.gathered_ev[wait_set]] * m
        scene = self.frame_scene(i0) if self.frame_scene else self.scene
        cams = [self.frame_cam(i0 + j) for j in range(m)] if self.frame_cam else [self.cam] * m
        rc = self.r.render_path(scene, cams, self.W, self.H, [self.outs[b].data_ptr() for b in bufs],
                                k=self.k, stream=self.stream, times=self._times(i0, m),
                                events=[self.frame_events[b] for b in bufs] if ov else None, join=not ov,
                                fork=not ov or first, wait_events=waits,
                                status=[self.status_ptrs[b] for b in bufs] if self.status_ptrs else None)
        self.overflowed |= rc != 0
        return rc

    def _chunk(self, cid: int, first: bool):
        i0, m = self.chunks[cid]
        s = cid % self.nsets
        if not self.frame_events:                # gloo / no overlap: the caller's stream orders reuse
            self.wait_pending(s)
        if self.sink:
            self._deliver(s)                     # the set's previous chunk, before it is overwritten
        self.path(i0, m, [s * self.per_set + j for j in range(m)], overlap=True, first=first, wait_set=s)
        if cid % self.gather_every == 0:
            self.gather(s, m, cid, i0)
        else:
            self.keep_local(s, m, i0)

    def run(self, steps: int):
        """K frames in flight, gathered per chunk when enabled (not drained: call drain())."""
        self.chunks = []
        self.bad_chunks = []
        if not self.step_gather:
            self.path(0, steps, [j % self.F for j in range(steps)])
            return
        for c0 in range(0, steps, self.chunk):
            self.chunks.append((c0, min(self.chunk, steps - c0)))
            self._chunk(len(self.chunks) - 1, c0 == 0)

    def finish(self, device) -> bool:
        """Drain the gathers and the renderer, then agree over ranks (a collective)
        whether any rank's frames since the last finish() were incomplete; with validity
        words, bad_chunks = the chunk ids (same list on every rank) that repair() must
        send again.  Clears the renderer's flag."""
        import torch
        self.drain()
        self._sync()
        rc = self.r.sync()                       # always: it also clears the context's reported overflow
        coarse = self.overflowed or rc != 0
        self.overflowed = False
        if not self.validity or not self.chunks:
            self.bad_chunks = []
            return any_over_ranks(self.dist, coarse, device)
        words = self.status_log.cpu() if self.status_log is not None else None
        local = [bool((words[i0:i0 + m] != 0).any()) for i0, m in self.chunks]
        if coarse and not any(local):
            local = [True] * len(self.chunks)   # an overflow no word names (frames outside the chunks)
        t = torch.tensor([1.0 if b else 0.0 for b in local], dtype=torch.float64, device=device)
        if self.dist is not None and self.dist.is_initialized() and self.dist.get_world_size() > 1:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        self.bad_chunks = [c for c, v in enumerate(t.tolist()) if v > 0]
        return bool(self.bad_chunks)

    def repair(self):
        """Render and gather again exactly the chunks finish() agreed on (every rank)."""
        for j, cid in enumerate(self.bad_chunks):
            self._chunk(cid, j == 0)
            self.repaired += 1

    def run_checked(self, steps: int, device, attempts: int = 3) -> bool:
        """run(steps), then finish() and repair() until no rank holds an incomplete frame
        (at most `attempts` repairs); True when clean.  Without validity words a bad
        region is run again whole."""
        self.run(steps)
        for _ in range(attempts):
            if not self.finish(device):
                return True
            if self.validity:
                self.repair()
            else:
                self.run(steps)
        return not self.finish(device)
