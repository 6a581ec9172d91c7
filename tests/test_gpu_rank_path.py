"""Both digit-rank paths of the sort and binning kernels (GSR_TUNE_RANK_ATOMIC).

The depth sort's downsweeps and both binning scatters take stable ranks either from
returning LDS atomics (one ds_add_rtn per item; relies on same-address lanes of one
wave64 instruction returning in lane order, which the ISA does not document) or
from ballot matching.  The library takes the atomic path only after the device
self-check (gsr_rank_order_check) passed.  These tests run that check, then render
configs 2 and 3 at full size and a tie-heavy scene with each path and require the
same depth order, the same tile lists and images bit-exact against the oracle.
Reference contract: a stable sort (render.cu:1099-1118, CUB SortPairs), ties by
Gaussian index."""
import os

import numpy as np
import pytest

from conftest import scene_soa
from conftest import exact_blend
from test_gpu_parity import assert_image_parity, cam_for

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch(gpu):
    import torch as t
    assert t.cuda.is_available()
    return t


def test_rank_order_self_check(gpu):
    ops, bad = gpu.rank_order_check()
    assert ops > 10_000_000
    assert bad == 0, f"{bad} of {ops} same-address LDS atomic lanes returned out of lane order"
    r = gpu.Renderer()
    assert r.get_tuning(gpu.TUNE_RANK_ATOMIC) == 1
    assert r.get_tuning(gpu.TUNE_RANK_ATOMIC_ACTIVE) == 1
    r.set_tuning(gpu.TUNE_RANK_ATOMIC, 0)
    assert r.get_tuning(gpu.TUNE_RANK_ATOMIC_ACTIVE) == 0
    with pytest.raises(gpu.GsrError):
        r.set_tuning(gpu.TUNE_RANK_ATOMIC_ACTIVE, 1)


def render_both(gpu, torch, scene, n, cam, W, H):
    """Render with ballot ranks and with atomic ranks; return {path: (image, depth order, pairs)}."""
    out = {}
    for ra in (0, 1):
        r = exact_blend(gpu.Renderer())      # images bit-exact against the oracle
        r.set_tuning(gpu.TUNE_DEPTH_SPLIT, 0)  # whole-depth-order tile lists (config 3 splits by default)
        r.set_tuning(gpu.TUNE_RANK_ATOMIC, ra)
        assert r.get_tuning(gpu.TUNE_RANK_ATOMIC_ACTIVE) == ra
        img = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
        for _ in range(3):
            r.render(scene, cam, W, H, img.data_ptr())
            if r.sync() == 0:
                break
        assert r.row_item_count() > 0                     # the binning path ran
        out[ra] = (img.view(3, H, W).cpu().numpy(), r.read_depth_order(n), r.read_pairs())
        r.close()
    return out


def check_paths(out, want):
    (i0, d0, p0), (i1, d1, p1) = out[0], out[1]
    assert np.array_equal(d0, d1), "depth order differs between the rank paths"
    keys = (d0 >> np.uint64(32)).astype(np.uint32)
    idx = (d0 & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    tie = keys[1:] == keys[:-1]
    assert (idx[1:][tie] > idx[:-1][tie]).all(), "depth ties not in index order"
    assert p0.size == p1.size and np.array_equal(p0, p1), "tile lists differ between the rank paths"
    assert_image_parity(i0, want, exact=True)
    assert_image_parity(i1, want, exact=True)


def test_rank_paths_config2_full(gpu, orc, torch, tmp_path_factory):
    """Config 2: 1M Gaussians, 1920x1080."""
    path, soa = scene_soa(gpu, tmp_path_factory, 1_000_000, 2)
    W, H = 1920, 1080
    cam = cam_for(gpu, W, H)
    out = render_both(gpu, torch, gpu.Scene.from_ply(path), soa.shape[1], cam, W, H)
    want = orc.render(soa, cam, W, H, 3.0, threads=min(16, os.cpu_count() or 1))
    check_paths(out, want)


def test_rank_paths_config3_full(gpu, orc, torch, tmp_path_factory):
    """Config 3 stand-in: 5M Gaussians, 1600x1063 (16 items per thread in the depth sort:
    the downsweep ranks with ballots on both paths there, the binning scatters do not)."""
    path, soa = scene_soa(gpu, tmp_path_factory, 5_000_000, 3)
    W, H = 1600, 1063
    cam = cam_for(gpu, W, H)
    out = render_both(gpu, torch, gpu.Scene.from_ply(path), soa.shape[1], cam, W, H)
    want = orc.render(soa, cam, W, H, 3.0, threads=min(16, os.cpu_count() or 1))
    check_paths(out, want)


def test_rank_paths_tie_heavy(gpu, orc, torch, tmp_path_factory):
    """300k Gaussians on 7 depth planes (the camera looks down -z, so view depth is z - 4
    exactly): every depth key is shared by ~43k Gaussians, and each tile list is made
    of long tied runs whose order only the index tie-break decides."""
    path, soa = scene_soa(gpu, tmp_path_factory, 300_000, 11)
    soa = soa.copy()
    planes = np.linspace(-0.9, 0.9, 7, dtype=np.float32)
    soa[2] = planes[np.arange(soa.shape[1]) % 7]
    W, H = 1920, 1080
    cam = cam_for(gpu, W, H)
    scene = gpu.Scene.from_soa(soa)
    out = render_both(gpu, torch, scene, soa.shape[1], cam, W, H)
    keys = (out[0][1] >> np.uint64(32)).astype(np.uint32)
    live = keys[keys != 0xFFFFFFFF]
    assert np.unique(live).size <= 7 and live.size > 200_000
    want = orc.render(soa, cam, W, H, 3.0, threads=min(16, os.cpu_count() or 1))
    check_paths(out, want)


def test_depth_sort_16_items_one_tile_per_workgroup(gpu, orc, torch, tmp_path_factory):
    """The 16-items-per-thread downsweep sorts exactly one 4,096-item tile per workgroup
    (a straight-line kernel: 147 VGPRs instead of 207); launch_radix_pass sorts 8 per
    thread when the grid is too small for that (GSR_TUNE_DEPTH_SORT_GROUPS caps it).
    700k Gaussians (the last tile partial) with 16 per thread, 16 with the grid capped at
    64 workgroups (the 8-item fallback, several tiles per workgroup) and 8 per thread: the
    same depth order, ties by index, and the image bit-exact against the oracle."""
    path, soa = scene_soa(gpu, tmp_path_factory, 700_000, 5)
    n = soa.shape[1]
    W, H = 1280, 720
    cam = cam_for(gpu, W, H)
    scene = gpu.Scene.from_ply(path)
    want = orc.render(soa, cam, W, H, 3.0, threads=min(16, os.cpu_count() or 1))
    orders = []
    for knobs in ({gpu.TUNE_DEPTH_SORT_ITEMS: 16}, {gpu.TUNE_DEPTH_SORT_ITEMS: 16, gpu.TUNE_DEPTH_SORT_GROUPS: 64},
                  {gpu.TUNE_DEPTH_SORT_ITEMS: 8}):
        r = exact_blend(gpu.Renderer())
        r.set_tuning(gpu.TUNE_DEPTH_SPLIT, 0)
        r.set_tuning(gpu.TUNE_DEPTH_BUCKETS, 0)            # the LSD passes on every frame
        for k, v in knobs.items():
            r.set_tuning(k, v)
        img = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
        for _ in range(3):
            r.render(scene, cam, W, H, img.data_ptr())
            if r.sync() == 0:
                break
        orders.append(r.read_depth_order(n))
        assert_image_parity(img.view(3, H, W).cpu().numpy(), want, exact=True)
        r.close()
    assert all(np.array_equal(orders[0], o) for o in orders[1:])
    keys = (orders[0] >> np.uint64(32)).astype(np.uint32)
    idx = (orders[0] & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    tie = keys[1:] == keys[:-1]
    assert (keys[1:] >= keys[:-1]).all() and (idx[1:][tie] > idx[:-1][tie]).all()
