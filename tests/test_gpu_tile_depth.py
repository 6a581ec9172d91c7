"""Per-tile depth order (GSR_TUNE_DEPTH_ORDER, gsr_kernels.hip "per-tile depth
order"): binning in index order followed by a stable depth sort of every tile's
list must give exactly the (tile, Gaussian) pairs of the global depth sort +
binning and of the pair sort (render.cu:1099-1118 order: tile, then depth key,
then index), and images bit-equal to the oracle.  Covers the LDS path (lists up
to 4096), the chunked global path (dense clusters, lists over 4096), every pass
count the key span can need (0 = all keys equal, 2, 3, 4), and the depth-order
readback of a per-tile frame."""
import numpy as np
import pytest

from test_gpu_parity import assert_image_parity, cam_for, render_gpu

pytestmark = pytest.mark.gpu

KNOB_BINNING, KNOB_DEPTH_ORDER = 7, 15


@pytest.fixture(scope="module")
def torch(gpu):
    import torch as t
    assert t.cuda.is_available()
    return t


def cluster(n, z_lo, z_hi, spread, seed):
    """n small Gaussians around the optical axis; z uniform in [z_lo, z_hi]."""
    rng = np.random.default_rng(seed)
    soa = np.zeros((38, n), np.float32)
    soa[0] = rng.normal(0, spread, n)
    soa[1] = rng.normal(0, spread, n)
    soa[2] = rng.uniform(z_lo, z_hi, n) if z_hi > z_lo else z_lo
    soa[3] = rng.uniform(0.05, 0.6, n)
    soa[4:7] = rng.uniform(0.004, 0.02, (3, n))
    soa[7:11] = rng.normal(0, 1, (4, n))
    soa[11:38] = rng.normal(0, 0.3, (27, n))
    return soa


def max_list(r):
    rg = r.read_tile_ranges().astype(np.int64)
    return int((rg[:, 1] - rg[:, 0]).max())


# (z range) -> depth-key span from the camera at z = 4: 0 (flat layer), < 2^16,
# < 2^24, >= 2^24 — 0, 2, 3 and 4 LSD passes in each tile
SPANS = [(0.0, 0.0), (0.0, 0.03), (-1.0, 1.0), (-20.0, 2.0)]


@pytest.mark.parametrize("z", SPANS)
@pytest.mark.parametrize("dense", [False, True])
def test_tile_depth_order_matches_global_and_pair_sort(gpu, orc, torch, z, dense):
    n = 40_000 if dense else 8_000
    soa = cluster(n, z[0], z[1], 0.05 if dense else 0.8, seed=11)
    W, H = 640, 480
    cam = cam_for(gpu, W, H)
    scene = gpu.Scene.from_soa(soa)
    rs = {}
    for name, knobs in (("tile", {KNOB_DEPTH_ORDER: 1}), ("global", {KNOB_DEPTH_ORDER: 0}),
                        ("pairs", {KNOB_BINNING: 0})):
        r = gpu.Renderer()
        for kn, v in knobs.items():
            r.set_tuning(kn, v)
        img, _ = render_gpu(gpu, torch, scene, cam, W, H, renderer=r)
        rs[name] = (r, img)
    r_tile = rs["tile"][0]
    assert r_tile.depth_passes() == 0                 # the frame used the per-tile order
    assert rs["global"][0].depth_passes() >= 1
    longest = max_list(r_tile)
    assert (longest > 4096) == dense, longest         # dense clusters exercise the chunked path
    pt = r_tile.read_pairs()
    assert pt.shape[0] > 1000
    assert np.array_equal(pt, rs["global"][0].read_pairs())
    assert np.array_equal(pt, rs["pairs"][0].read_pairs())
    want = orc.render(soa, cam, W, H, 3.0)
    for name in rs:
        assert_image_parity(rs[name][1], want)


def test_read_depth_order_after_tile_frame(gpu, orc, torch):
    """The depth-order readback of a per-tile frame is computed on demand and equals
    the oracle's stable (key, index) order."""
    soa = cluster(8_000, -1.0, 1.0, 0.8, seed=14)
    W, H = 320, 240
    cam = cam_for(gpu, W, H)
    r = gpu.Renderer()
    r.set_tuning(KNOB_DEPTH_ORDER, 1)
    render_gpu(gpu, torch, gpu.Scene.from_soa(soa), cam, W, H, renderer=r)
    assert r.depth_passes() == 0
    want = orc.preprocess(soa, cam, W, H, 3.0)
    assert np.array_equal(r.read_depth_order(soa.shape[1]), orc.expected_depth_order(want))
