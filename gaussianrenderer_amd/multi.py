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
