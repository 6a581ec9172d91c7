"""The bucket depth sort (GSR_TUNE_DEPTH_BUCKETS, gsr_kernels.hip "bucket depth sort").

A context's first frame of a scene size runs the LSD passes and takes depth quantiles
from their order; every later frame scatters the preprocess order stably into ~n/1024
buckets bounded by those quantiles and sorts each bucket in one workgroup (in LDS, or
through global memory when the bucket is over capacity).  The order must be exactly the
LSD passes' order: stable by depth key, ties in index order (render.cu:1099-1118, CUB
SortPairs).  Every test renders at least two frames per context,
so the second one is bucket-sorted, and compares the depth order with the oracle's
(tests/_oracle.py expected_depth_order), the tile lists with the LSD path's and the
image bit for bit with the oracle's (exact blend)."""
import os

import numpy as np
import pytest

from conftest import exact_blend, scene_soa
from test_gpu_parity import assert_image_parity, cam_for

pytestmark = pytest.mark.gpu

THREADS = min(16, len(os.sched_getaffinity(0)))


@pytest.fixture(scope="module")
def torch(gpu):
    import torch as t
    assert t.cuda.is_available()
    return t


# big buckets above 2M: 512 (default) or 1,024 (A/B env GSR_BIG_BUCKETS=1024), and their capacity
BIG = 1024 if os.environ.get("GSR_BIG_BUCKETS") == "1024" else 512
BIG_CAP = 16384 * 512 // BIG


def render_frames(gpu, torch, r, scene, cams, W, H):
    """Render each camera on r (re-rendered after an overflow); returns the last image."""
    out = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    for cam in cams:
        for _ in range(3):
            r.render(scene, cam, W, H, out.data_ptr())
            if r.sync() == 0:
                break
        else:
            raise AssertionError("frame kept overflowing")
    return out.view(3, H, W).cpu().numpy()


def renderer(gpu, buckets=1):
    r = exact_blend(gpu.Renderer())
    r.set_tuning(gpu.TUNE_DEPTH_SPLIT, 0)       # whole-order lists (5M scenes split by default)
    r.set_tuning(gpu.TUNE_DEPTH_BUCKETS, buckets)
    return r


def check_bucket_frame(gpu, orc, torch, scene, soa, cams, W, H, buckets=1, want_over=None, want_work=None):
    """Frames over cams on a bucket-sort renderer and on an LSD-only one; the last frame
    must be bucket-sorted on the first and equal the oracle (order, image) and the LSD
    renderer (order, tile lists)."""
    n = soa.shape[1]
    r = renderer(gpu, buckets)
    img = render_frames(gpu, torch, r, scene, cams, W, H)
    assert r.depth_passes() == 0, "the last frame was not bucket-sorted"
    order = r.read_depth_order(n)
    pairs = r.read_pairs()
    over = r.get_tuning(gpu.TUNE_DEPTH_BUCKETS_OVER)
    if want_work is not None:       # tied keys: the global path's buckets need (almost) no passes
        assert r.get_tuning(gpu.TUNE_DEPTH_BUCKETS_WORK) <= want_work
    ref = renderer(gpu, 0)
    img_lsd = render_frames(gpu, torch, ref, scene, cams[-1:], W, H)
    assert ref.depth_passes() >= 1
    want_spl = orc.preprocess(soa, cams[-1], W, H, 3.0)
    assert np.array_equal(order, orc.expected_depth_order(want_spl)), "bucket-sorted depth order differs"
    assert np.array_equal(order, ref.read_depth_order(n))
    assert np.array_equal(pairs, ref.read_pairs()), "tile lists differ from the LSD path's"
    want = orc.render(soa, cams[-1], W, H, 3.0, threads=THREADS)
    assert_image_parity(img, want, exact=True)
    assert np.array_equal(img.view(np.uint32), img_lsd.view(np.uint32))
    if want_over is not None:
        want_over(over)
    r.close()
    ref.close()
    return order


def no_over(o):
    assert o == 0, f"{o} items took the global path on a fixed camera"


def some_over(o):
    assert o > 0, "no bucket took the global path"


def test_bucket_sort_config1(gpu, orc, torch, tmp_path_factory):
    """Config 1 (10k Gaussians, 640x480): 256 buckets of ~40 items."""
    _, soa = scene_soa(gpu, tmp_path_factory, 10_000, 1)
    W, H = 640, 480
    cams = [cam_for(gpu, W, H)] * 2
    check_bucket_frame(gpu, orc, torch, gpu.Scene.from_soa(soa), soa, cams, W, H, want_over=no_over)


def test_bucket_sort_config2_full(gpu, orc, torch, tmp_path_factory):
    """Config 2 (1M, 1920x1080): 1,024 buckets of ~930 live items, all inside the local
    capacity on a fixed camera (no item takes the global path)."""
    path, soa = scene_soa(gpu, tmp_path_factory, 1_000_000, 2)
    W, H = 1920, 1080
    cams = [cam_for(gpu, W, H)] * 3
    check_bucket_frame(gpu, orc, torch, gpu.Scene.from_ply(path), soa, cams, W, H, want_over=no_over)


def test_bucket_sort_moving_camera(gpu, orc, torch, tmp_path_factory):
    """Quantiles from one view, frame from another (orbit steps of 10 and 90 degrees and a
    zoom): the buckets are unbalanced, some may overflow into the global path; the
    order stays exact."""
    from gaussianrenderer_amd import multi
    _, soa = scene_soa(gpu, tmp_path_factory, 200_000, 4)
    W, H = 960, 540
    n = soa.shape[1]
    cams = [multi.orbit_camera(0, W, H), multi.orbit_camera(1, W, H), multi.orbit_camera(3, W, H),
            cam_for(gpu, W, H, pos=(0.0, 0.0, 2.5))]
    scene = gpu.Scene.from_soa(soa)
    # every frame's order is exact; a frame after one whose global path ran over n / 8
    # item-passes reseeds the splitters (LSD passes), the others are bucket-sorted with the
    # previous frame's quantiles
    r = renderer(gpu)
    bucketed = 0
    for i, cam in enumerate(cams):
        render_frames(gpu, torch, r, scene, [cam], W, H)
        if i > 0:
            bucketed += r.depth_passes() == 0
        assert np.array_equal(r.read_depth_order(n), orc.expected_depth_order(orc.preprocess(soa, cam, W, H, 3.0)))
    assert bucketed >= 2, "stale splitters were not exercised"
    r.close()
    check_bucket_frame(gpu, orc, torch, scene, soa, cams[:2], W, H)


def test_bucket_sort_config2_orbit_bounded(gpu, orc, torch, tmp_path_factory):
    """config 2 (1M, 1920x1080) on a moving camera, 0.25 deg per frame (the
    bench's orbit object): every frame is bucket-sorted with the previous frame's quantiles,
    the buckets stay under the local capacity (largest live bucket <= 2,048 items and <= 2 x
    the mean; gsr_bucket_sizes; the open edge buckets take a quarter share for the drift), no
    item takes the global path, and the last frame's order and image equal the oracle's."""
    path, soa = scene_soa(gpu, tmp_path_factory, 1_000_000, 2)
    n = soa.shape[1]
    W, H = 1920, 1080
    scene = gpu.Scene.from_ply(path)
    cams = []
    for i in range(12):
        c = gpu.make_camera(position=(0, 0, 4), fov_y=50, aspect=W / H)
        cams.append(gpu.orbit(c, 0.25 * i, 0.0))
    r = renderer(gpu)
    render_frames(gpu, torch, r, scene, cams[:1], W, H)           # LSD: the first quantiles
    over0 = r.get_tuning(gpu.TUNE_DEPTH_BUCKETS_OVER)
    for cam in cams[1:]:
        img = render_frames(gpu, torch, r, scene, [cam], W, H)
        assert r.depth_passes() == 0
        sizes = r.bucket_sizes()
        assert sizes is not None and sizes.size == 1024 and int(sizes.sum()) == n
        live = sizes[:-1].astype(np.float64)
        # under the 2,048-item local capacity, the edge buckets' drift included
        assert live.max() <= 2048 and live.max() <= 2.0 * live.mean(), f"imbalance {live.max() / live.mean():.3f}"
    assert r.get_tuning(gpu.TUNE_DEPTH_BUCKETS_OVER) == over0, "an orbit frame took the global path"
    spl = orc.preprocess(soa, cams[-1], W, H, 3.0)
    assert int(sizes[-1]) == int((spl["status"] != 2).sum())      # the last bucket: the culled items
    assert np.array_equal(r.read_depth_order(n), orc.expected_depth_order(spl))
    assert_image_parity(img, orc.render(soa, cams[-1], W, H, 3.0, threads=THREADS), exact=True)
    r.close()


def test_bucket_splitters_reseed(gpu, orc, torch, tmp_path_factory):
    """The splitters belong to a scene and a view: another scene of the same size class, or
    a frame whose global path ran more than n / 8 item-passes (a camera cut), makes the
    next frame take the LSD passes and reseed them (one workgroup would otherwise
    sort most of the scene); the frame after is bucket-sorted again.  Every order exact."""
    _, soa_a = scene_soa(gpu, tmp_path_factory, 100_000, 15)
    _, soa_b = scene_soa(gpu, tmp_path_factory, 100_000, 16)
    soa_b = soa_b.copy()
    soa_b[2] *= 0.05                                   # a thin slab: B's depths fill few of A's buckets
    W, H = 640, 480
    n = soa_a.shape[1]
    cam = cam_for(gpu, W, H)
    a, b = gpu.Scene.from_soa(soa_a), gpu.Scene.from_soa(soa_b)
    r = renderer(gpu)
    seq = [(a, soa_a, None), (a, soa_a, 0), (b, soa_b, "lsd"), (b, soa_b, 0), (b, soa_b, 0)]
    for scene, soa, want in seq:
        render_frames(gpu, torch, r, scene, [cam], W, H)
        if want == "lsd":
            assert r.depth_passes() >= 1, "a new scene did not reseed the splitters"
        elif want == 0:
            assert r.depth_passes() == 0
        assert np.array_equal(r.read_depth_order(n), orc.expected_depth_order(orc.preprocess(soa, cam, W, H, 3.0)))
    assert r.get_tuning(gpu.TUNE_DEPTH_BUCKETS_OVER) == 0
    # a camera cut on one scene: from far behind to close in front, then hold
    far_cam = cam_for(gpu, W, H, pos=(0, 0, 40))
    near_cam = cam_for(gpu, W, H, pos=(0, 0, 1.2), fov=90)
    render_frames(gpu, torch, r, a, [far_cam, far_cam], W, H)
    assert r.depth_passes() == 0
    work0 = r.get_tuning(gpu.TUNE_DEPTH_BUCKETS_WORK)
    render_frames(gpu, torch, r, a, [near_cam], W, H)          # stale splitters: a spike
    assert r.depth_passes() == 0
    spike = r.get_tuning(gpu.TUNE_DEPTH_BUCKETS_WORK) - work0
    assert spike > n // 8, f"the cut sent only {spike} item-passes through the global path"
    render_frames(gpu, torch, r, a, [near_cam], W, H)
    assert r.depth_passes() >= 1, "the spike did not reseed the splitters"
    render_frames(gpu, torch, r, a, [near_cam], W, H)
    assert r.depth_passes() == 0
    assert np.array_equal(r.read_depth_order(n), orc.expected_depth_order(orc.preprocess(soa_a, near_cam, W, H, 3.0)))
    r.close()


def test_bucket_sort_global_path(gpu, orc, torch, tmp_path_factory):
    """Test hook 2: a local capacity of 64 items, so nearly every bucket of a 200k scene is
    sorted through global memory (stable 8-bit passes ping-ponging with the scratch
    buffer); the order and image are still exact."""
    _, soa = scene_soa(gpu, tmp_path_factory, 200_000, 5)
    W, H = 960, 540
    cams = [cam_for(gpu, W, H)] * 2

    def many_over(o):
        assert o > 150_000, f"only {o} items took the global path"

    check_bucket_frame(gpu, orc, torch, gpu.Scene.from_soa(soa), soa, cams, W, H, buckets=2, want_over=many_over)


def test_bucket_sort_tie_heavy(gpu, orc, torch, tmp_path_factory):
    """300k Gaussians on 7 depth planes: every live key is shared by ~43k Gaussians, so
    each plane fills one bucket far over capacity (the global path with no key bits to
    sort: the stable scatter's index order is the answer), ties in index order."""
    _, soa = scene_soa(gpu, tmp_path_factory, 300_000, 11)
    soa = soa.copy()
    soa[2] = np.linspace(-0.9, 0.9, 7, dtype=np.float32)[np.arange(soa.shape[1]) % 7]
    W, H = 1920, 1080
    cams = [cam_for(gpu, W, H)] * 2
    order = check_bucket_frame(gpu, orc, torch, gpu.Scene.from_soa(soa), soa, cams, W, H,
                               want_over=some_over, want_work=soa.shape[1] // 8)
    keys = (order >> np.uint64(32)).astype(np.uint32)
    assert np.unique(keys[keys != 0xFFFFFFFF]).size <= 7


def test_bucket_sort_ballot_ranks(gpu, orc, torch, tmp_path_factory):
    """The ballot-matching rank path (GSR_TUNE_RANK_ATOMIC 0) of the scatter and the local
    passes gives the same order."""
    _, soa = scene_soa(gpu, tmp_path_factory, 100_000, 6)
    W, H = 640, 480
    n = soa.shape[1]
    scene = gpu.Scene.from_soa(soa)
    cams = [cam_for(gpu, W, H)] * 2
    orders = []
    for ra in (0, 1):
        for hook in (1, 2):
            r = renderer(gpu, hook)
            r.set_tuning(gpu.TUNE_RANK_ATOMIC, ra)
            render_frames(gpu, torch, r, scene, cams, W, H)
            assert r.depth_passes() == 0
            orders.append(r.read_depth_order(n))
            r.close()
    want = orc.expected_depth_order(orc.preprocess(soa, cams[-1], W, H, 3.0))
    for o in orders:
        assert np.array_equal(o, want)


def test_bucket_sort_4d_replaces_partition(gpu, orc, torch, tmp_path_factory):
    """4D scenes (config 5 kind) take the live partition before the LSD passes; the bucket
    sort keeps culled items apart itself (its last bucket, index order).  Two times of a
    100k 4D scene: the second frame is bucket-sorted; its order equals the partitioned
    LSD path's (the temporal cull gives culled items key 0xFFFFFFFF, which the oracle's
    3D restatement of the scene at time t does not know) and its image the oracle's."""
    p = tmp_path_factory.mktemp("b4d") / "scene4d.ply"
    gpu.write_synthetic_ply4d(str(p), 100_000, 5)
    soa49 = gpu.read_ply(str(p), four_d=True)
    scene = gpu.Scene.from_ply(str(p))
    assert scene.is_4d
    W, H = 960, 540
    cam = cam_for(gpu, W, H)
    n = soa49.shape[1]
    got = {}
    for buckets in (1, 0):
        r = renderer(gpu, buckets)
        out = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
        for t in (0.0, 0.5):
            r.render(scene, cam, W, H, out.data_ptr(), time=t)
            assert r.sync() == 0
        assert (r.depth_passes() == 0) == (buckets == 1)
        got[buckets] = (r.read_depth_order(n), out.view(3, H, W).cpu().numpy(), r.read_pairs())
        r.close()
    order = got[1][0]
    assert np.array_equal(order, got[0][0]), "bucket-sorted 4D order differs from the partitioned LSD order"
    assert np.array_equal(got[1][2], got[0][2])
    keys = (order >> np.uint64(32)).astype(np.uint32)
    assert (keys == 0xFFFFFFFF).sum() > n // 4          # the temporal cull left many culled items
    want = orc.render(orc.temporal(soa49, 0.5), cam, W, H, 3.0, threads=THREADS)
    assert_image_parity(got[1][1], want, exact=True)


def test_bucket_sort_stage_api_repeated_sort(gpu, orc, torch, tmp_path_factory):
    """Stage API: preprocess, sort (bucket-sorted), sort again (LSD passes over the sorted
    order), blend: the same order both times and the oracle's image."""
    _, soa = scene_soa(gpu, tmp_path_factory, 50_000, 7)
    W, H = 640, 480
    cam = cam_for(gpu, W, H)
    scene = gpu.Scene.from_soa(soa)
    n = soa.shape[1]
    r = renderer(gpu)
    render_frames(gpu, torch, r, scene, [cam], W, H)      # quantiles
    out = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    r.preprocess(scene, cam, W, H)
    r.sort()
    assert r.depth_passes() == 0
    first = r.read_depth_order(n)
    r.sort()
    assert r.depth_passes() >= 1
    assert np.array_equal(r.read_depth_order(n), first)
    r.blend(out.data_ptr())
    assert r.sync() == 0
    want_spl = orc.preprocess(soa, cam, W, H, 3.0)
    assert np.array_equal(first, orc.expected_depth_order(want_spl))
    assert_image_parity(out.view(3, H, W).cpu().numpy(), orc.render(soa, cam, W, H, 3.0), exact=True)


def test_bucket_sort_frames_in_flight(gpu, orc, torch, tmp_path_factory):
    """Four lanes over an orbit (each lane's splitters come from its own previous frame):
    every frame equals the oracle's."""
    from gaussianrenderer_amd import multi
    _, soa = scene_soa(gpu, tmp_path_factory, 100_000, 8)
    W, H = 640, 480
    cams = [multi.orbit_camera(i % 8, W, H) for i in range(12)]
    scene = gpu.Scene.from_soa(soa)
    r = renderer(gpu)
    r.set_frames_in_flight(4)
    outs = [torch.empty(3 * W * H, device="cuda") for _ in cams]
    for _ in range(3):
        rc = r.render_path(scene, cams, W, H, [o.data_ptr() for o in outs])
        if r.sync() == 0 and rc == 0:
            break
    for cam, o in zip(cams, outs):
        assert_image_parity(o.view(3, H, W).cpu().numpy(), orc.render(soa, cam, W, H, 3.0), exact=True)


def test_bucket_sort_knob(gpu):
    r = gpu.Renderer()
    assert r.get_tuning(gpu.TUNE_DEPTH_BUCKETS) == 1
    with pytest.raises(gpu.GsrError):
        r.set_tuning(gpu.TUNE_DEPTH_BUCKETS, 4)
    with pytest.raises(gpu.GsrError):
        r.set_tuning(gpu.TUNE_DEPTH_BUCKETS_OVER, 0)
    assert r.get_tuning(gpu.TUNE_DEPTH_BUCKETS_OVER) == 0


def test_bucket_sort_all_culled_then_visible(gpu, orc, torch, tmp_path_factory):
    """A frame with every Gaussian culled (the camera looks away: every item in the last
    bucket, no live quantiles, so the frame keeps its splitters) between visible frames:
    each frame's order is exact, and every frame is bucket-sorted unless the frame before
    it ran more than n / 8 item-passes through the global path (then it reseeds)."""
    _, soa = scene_soa(gpu, tmp_path_factory, 20_000, 9)
    W, H = 320, 240
    n = soa.shape[1]
    scene = gpu.Scene.from_soa(soa)
    r = renderer(gpu)
    render_frames(gpu, torch, r, scene, [cam_for(gpu, W, H)], W, H)   # the LSD frame: first quantiles
    spike = False
    for i, cam in enumerate((cam_for(gpu, W, H), cam_for(gpu, W, H, pos=(0, 0, 40), look=(0, 0, 80)),
                             cam_for(gpu, W, H), cam_for(gpu, W, H, pos=(0, 0, 12), fov=90))):
        w0 = r.get_tuning(gpu.TUNE_DEPTH_BUCKETS_WORK)
        img = render_frames(gpu, torch, r, scene, [cam], W, H)
        assert (r.depth_passes() == 0) == (not spike), i
        if i == 2:   # after the look-away: its kept splitters are the visible frame's
            assert r.get_tuning(gpu.TUNE_DEPTH_BUCKETS_WORK) == w0
        spike = r.get_tuning(gpu.TUNE_DEPTH_BUCKETS_WORK) - w0 > n // 8
        want_spl = orc.preprocess(soa, cam, W, H, 3.0)
        assert np.array_equal(r.read_depth_order(n), orc.expected_depth_order(want_spl))
        assert_image_parity(img, orc.render(soa, cam, W, H, 3.0), exact=True)


def test_bucket_rows_fused_matches_row_count(gpu, orc, torch, tmp_path_factory):
    """GSR_TUNE_BUCKET_ROWS: the local sorts count the row pass per bucket (the bucket is the
    row chunk) and the row pass skips its count kernel; with 0 the row pass counts its own
    fixed chunks.  Same tile lists, same image, also with the global path (hook 2), whose
    buckets are larger than a row chunk."""
    _, soa = scene_soa(gpu, tmp_path_factory, 200_000, 12)
    W, H = 1280, 720
    scene = gpu.Scene.from_soa(soa)
    cams = [cam_for(gpu, W, H)] * 2
    got = {}
    for hook in (1, 2):
        for fused in (1, 0):
            r = renderer(gpu, hook)
            r.set_tuning(gpu.TUNE_BUCKET_ROWS, fused)
            img = render_frames(gpu, torch, r, scene, cams, W, H)
            assert r.depth_passes() == 0
            got[(hook, fused)] = (img, r.read_pairs(), r.read_tile_ranges())
            r.close()
    base = got[(1, 0)]
    for key, (img, pairs, ranges) in got.items():
        assert np.array_equal(pairs, base[1]), key
        assert np.array_equal(ranges, base[2]), key
        assert np.array_equal(img.view(np.uint32), base[0].view(np.uint32)), key
    assert_image_parity(base[0], orc.render(soa, cams[-1], W, H, 3.0, threads=THREADS), exact=True)


def test_bucket_rows_fused_saturated_keys(gpu, orc, torch, tmp_path_factory):
    """Live Gaussians whose depth key saturates (depth >= ~4295: gsr_f2u_sat(-Z * 1e6) =
    0xFFFFFFFF, render.cu:850) under a far clip of 1e4 share the last bucket with the culled
    items.  The fused row count must bin them like the unfused row pass, the LSD passes and
    the oracle (the fused row pass used to stop at the last bucket's start)."""
    _, soa = scene_soa(gpu, tmp_path_factory, 200_000, 14)
    soa = soa.copy()
    n = soa.shape[1]
    far = np.arange(n) % 20 == 7                      # 5 %: large Gaussians ~5,000 units away
    rng = np.random.default_rng(14)
    m = int(far.sum())
    soa[0, far] = rng.uniform(-800, 800, m)
    soa[1, far] = rng.uniform(-450, 450, m)
    soa[2, far] = -rng.uniform(4996, 5400, m)
    soa[4:7, far] = rng.uniform(12, 30, (3, m))
    W, H = 1280, 720
    cam = gpu.make_camera(position=(0, 0, 4), look_at=(0, 0, 0), fov_y=50, aspect=W / H, far=1e4)
    spl = orc.preprocess(soa, cam, W, H, 3.0)
    sat = int(((spl["status"] == 2) & (spl["depth_key"] == 0xFFFFFFFF)).sum())
    assert sat > m // 2, f"only {sat} live Gaussians with a saturated key"
    scene = gpu.Scene.from_soa(soa)
    got = {}
    for buckets, fused in ((1, 1), (1, 0), (0, 1)):
        r = renderer(gpu, buckets)
        r.set_tuning(gpu.TUNE_BUCKET_ROWS, fused)
        img = render_frames(gpu, torch, r, scene, [cam] * 2, W, H)
        assert (r.depth_passes() == 0) == (buckets == 1)
        assert np.array_equal(r.read_depth_order(n), orc.expected_depth_order(spl))
        got[(buckets, fused)] = (img, r.read_pairs(), r.read_tile_ranges())
        r.close()
    base = got[(0, 1)]
    for key, (img, pairs, ranges) in got.items():
        assert np.array_equal(pairs, base[1]), key
        assert np.array_equal(ranges, base[2]), key
        assert np.array_equal(img.view(np.uint32), base[0].view(np.uint32)), key
    assert_image_parity(base[0], orc.render(soa, cam, W, H, 3.0, threads=THREADS), exact=True)


@pytest.mark.parametrize("hook", [1, 2])
def test_big_buckets(gpu, orc, torch, tmp_path_factory, hook):
    """Knob 28 = 1 (default) above 2M Gaussians: 512 buckets of ~n / 512 items, each sorted by
    one 1,024-thread workgroup in LDS (gsr_kernels.hip k_bbk_local), the scatter writing each
    tile in bucket order as 12-B records; 2 = the same with a 64-item capacity, so nearly every
    bucket goes to the second launch (k_bkt_local's paths).  2.3M Gaussians on a moving camera (stale splitters):
    the order equals the oracle's and the LSD passes', the tile lists and image too."""
    from gaussianrenderer_amd import multi
    _, soa = scene_soa(gpu, tmp_path_factory, 2_300_000, 18)
    n = soa.shape[1]
    W, H = 960, 540
    scene = gpu.Scene.from_soa(soa)
    cams = [multi.orbit_camera(0, W, H), gpu.orbit(multi.orbit_camera(0, W, H), 0.5, 0.0),
            gpu.orbit(multi.orbit_camera(0, W, H), 1.0, 0.0)]
    r = renderer(gpu, hook)
    img = render_frames(gpu, torch, r, scene, cams, W, H)
    assert r.depth_passes() == 0
    sizes = r.bucket_sizes()
    assert sizes is not None and sizes.size == BIG and int(sizes.sum()) == n
    over = r.get_tuning(gpu.TUNE_DEPTH_BUCKETS_OVER)
    if hook == 2:
        assert over > n // 2
    order, pairs = r.read_depth_order(n), r.read_pairs()
    r.close()
    ref = renderer(gpu, 0)
    img_lsd = render_frames(gpu, torch, ref, scene, cams[-1:], W, H)
    assert ref.depth_passes() >= 1
    spl = orc.preprocess(soa, cams[-1], W, H, 3.0)
    assert np.array_equal(order, orc.expected_depth_order(spl)), "big-bucket depth order differs"
    assert np.array_equal(order, ref.read_depth_order(n))
    assert np.array_equal(pairs, ref.read_pairs())
    assert np.array_equal(img.view(np.uint32), img_lsd.view(np.uint32))
    assert_image_parity(img, orc.render(soa, cams[-1], W, H, 3.0, threads=THREADS), exact=True)
    ref.close()


def test_big_buckets_tie_heavy(gpu, orc, torch, tmp_path_factory):
    """Big buckets (the default above 2M) on 2.2M Gaussians on 5 depth planes: each plane's bucket is far over the
    capacity (the second launch's global path, no key bits to sort: index order), ties in
    index order."""
    _, soa = scene_soa(gpu, tmp_path_factory, 2_200_000, 19)
    soa = soa.copy()
    soa[2] = np.linspace(-0.9, 0.9, 5, dtype=np.float32)[np.arange(soa.shape[1]) % 5]
    n = soa.shape[1]
    W, H = 640, 480
    cam = cam_for(gpu, W, H)
    r = renderer(gpu)
    render_frames(gpu, torch, r, gpu.Scene.from_soa(soa), [cam] * 2, W, H)
    assert r.depth_passes() == 0
    assert np.array_equal(r.read_depth_order(n), orc.expected_depth_order(orc.preprocess(soa, cam, W, H, 3.0)))
    r.close()


def test_bucket_kind_by_size(gpu, orc, torch, tmp_path_factory):
    """Above 2,097,152 Gaussians the default sorts 512 big buckets; knob 28 = 3 keeps the
    small-bucket kind (~n / 1,024 buckets, up to 4,096) there.  Both orders exact."""
    _, soa = scene_soa(gpu, tmp_path_factory, 2_100_000, 13)
    n = soa.shape[1]
    W, H = 320, 240
    scene = gpu.Scene.from_soa(soa)
    cam = cam_for(gpu, W, H)
    want = orc.expected_depth_order(orc.preprocess(soa, cam, W, H, 3.0))
    for knob, buckets in ((1, BIG), (3, gpu.MAX_BUCKETS)):
        r = renderer(gpu, knob)
        render_frames(gpu, torch, r, scene, [cam] * 2, W, H)
        assert r.depth_passes() == 0
        assert r.bucket_sizes().size == buckets, knob
        assert np.array_equal(r.read_depth_order(n), want), knob
        r.close()


def test_big_buckets_config3_orbit(gpu, orc, torch, tmp_path_factory):
    """Config 3 (5M, 1600x1063) on a 0.25-deg orbit with the default
    bucket sort: the first frame runs the LSD passes, the next three sort 512 big buckets
    bounded by the previous frame's quantiles.  Every live bucket fits one workgroup's 16,384
    items and no item takes the global path; the last frame's depth order equals the oracle's,
    and its order, tile lists and image (exact blend) equal the LSD passes', bit for bit."""
    path, soa = scene_soa(gpu, tmp_path_factory, 5_000_000, 3)
    n = soa.shape[1]
    W, H = 1600, 1063
    scene = gpu.Scene.from_ply(path)
    cams = [gpu.orbit(gpu.make_camera(position=(0, 0, 4), fov_y=50, aspect=W / H), 0.25 * i, 0.0)
            for i in range(4)]
    r = renderer(gpu)
    over0 = r.get_tuning(gpu.TUNE_DEPTH_BUCKETS_OVER)
    img = render_frames(gpu, torch, r, scene, cams, W, H)
    assert r.depth_passes() == 0
    sizes = r.bucket_sizes()
    assert sizes.size == BIG and int(sizes.sum()) == n
    assert int(sizes[:-1].max()) <= BIG_CAP, int(sizes[:-1].max())
    assert r.get_tuning(gpu.TUNE_DEPTH_BUCKETS_OVER) == over0
    order, pairs = r.read_depth_order(n), r.read_pairs()
    r.close()
    ref = renderer(gpu, 0)
    img_lsd = render_frames(gpu, torch, ref, scene, cams[-1:], W, H)
    assert ref.depth_passes() >= 1
    assert np.array_equal(order, ref.read_depth_order(n))
    assert np.array_equal(pairs, ref.read_pairs())
    assert np.array_equal(img.view(np.uint32), img_lsd.view(np.uint32))
    ref.close()
    spl = orc.preprocess(soa, cams[-1], W, H, 3.0)
    assert np.array_equal(order, orc.expected_depth_order(spl)), "config 3 orbit depth order differs"


def test_big_buckets_camera_cut_reseeds(gpu, orc, torch, tmp_path_factory):
    """A camera cut above 2M (big buckets): from far behind the scene to close in front, the
    stale splitters put most items into a few buckets over the 16,384-item capacity; the
    second launch's global path sorts them (more than n / 8 item-passes), the next frame
    reseeds from the LSD passes and the one after is bucket-sorted again.  Orders exact."""
    _, soa = scene_soa(gpu, tmp_path_factory, 2_200_000, 21)
    n = soa.shape[1]
    W, H = 640, 480
    scene = gpu.Scene.from_soa(soa)
    far_cam = cam_for(gpu, W, H, pos=(0, 0, 40))
    near_cam = cam_for(gpu, W, H, pos=(0, 0, 1.2), fov=90)
    r = renderer(gpu)
    render_frames(gpu, torch, r, scene, [far_cam, far_cam], W, H)
    assert r.depth_passes() == 0 and r.bucket_sizes().size == BIG
    work0 = r.get_tuning(gpu.TUNE_DEPTH_BUCKETS_WORK)
    render_frames(gpu, torch, r, scene, [near_cam], W, H)          # stale splitters: a spike
    assert r.depth_passes() == 0
    spike = r.get_tuning(gpu.TUNE_DEPTH_BUCKETS_WORK) - work0
    assert spike > n // 8, f"the cut sent only {spike} item-passes through the global path"
    want = orc.expected_depth_order(orc.preprocess(soa, near_cam, W, H, 3.0))
    assert np.array_equal(r.read_depth_order(n), want)
    render_frames(gpu, torch, r, scene, [near_cam], W, H)
    assert r.depth_passes() >= 1, "the spike did not reseed the splitters"
    render_frames(gpu, torch, r, scene, [near_cam], W, H)
    assert r.depth_passes() == 0
    assert np.array_equal(r.read_depth_order(n), want)
    r.close()
