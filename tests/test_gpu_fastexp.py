"""The fast-exp blend (GSR_TUNE_BLEND_EXP 1, the default since round 4) against the oracle.

The exact blend evaluates the reference's expf (render.cu:333) as gsr_blend_expf, a
15-VALU polynomial per pixel-splat pair, and is bit-identical to the oracle.  The
fast blend uses the hardware exp (v_exp_f32) for alpha and keeps every DECISION of
the reference (render.cu:328, 335) exact:

* the alpha test `alpha < 1e-3` is taken on the exp argument against the record's
  xs = gsr_alpha_take_min_x(opacity) — exact because gsr_blend_expf is monotone on every
  float (checked exhaustively below) and xs is the smallest passing argument
  (checked on the device against the host restatement below);
* the transmittance test `T < 1e-3` is guarded: T differs from the exact chain by a
  relative amount bounded from the exhaustively measured exp error (checked below
  against the kernel's constants), and a block where T crosses 1e-3 inside that band
  is blended again exactly.

So every pixel composites the same splats as the oracle in the same order (take
maps equal, pixel by pixel), and the colours differ only by the alpha rounding: the
north-star gate L-inf <= 1e-4 holds with orders of magnitude to spare."""
import os

import numpy as np
import pytest

from conftest import KNOB_BLEND_EXP, assert_frames, scene_soa

KNOB_DEPTH_SPLIT = 23
from test_gpu_parity import CAMS, cam_for, render_gpu

pytestmark = pytest.mark.gpu

# gsr_kernels.hip: kFxEps3 / kFxEps2 / kFxEps1, bounds on |alpha_fast / alpha_exact - 1|
# for composited lanes / alpha > 0.5 / alpha > 0.9
K_FX_EPS = {-6.95: 6.6e-7, -0.70: 4.8e-7, -0.11: 4.8e-7}
ULP_PRODUCT = 2.0 ** -23          # the two roundings of op * e
ORC_THREADS = min(16, len(os.sched_getaffinity(0)))


@pytest.fixture(scope="module")
def torch(gpu):
    import torch as t
    assert t.cuda.is_available()
    return t


def test_exact_exp_is_monotone_on_every_float(gpu):
    """gsr_blend_expf(x) <= gsr_blend_expf(next float after x) for every float in
    [-2e7, 88.75] (outside [-104, 88.75] the clamp makes it constant): the alpha test is
    a threshold on the exp argument.  Over the same floats, the compositing loop's
    packed exp (gsr_blend_expf_x2: no clamp, for the fast-path proof's in-box range
    [-2e7, 5]) equals the scalar function on both halves."""
    viol, pk_bad, _, _ = gpu.exp_probe(-2e7, 88.75, 0.0)
    assert viol == 0
    assert pk_bad == 0


def test_fast_exp_error_within_kernel_bounds(gpu):
    """Every float exp argument a composited lane can have: alpha_exact >= 1e-3 with
    opacity <= 1 means gsr_blend_expf(x) >= 1e-3, x >= ln(1e-3) = -6.9078; the fast-path
    proof bounds md2 >= -10, x <= 5.  alpha > 0.5 means x > ln 0.5 = -0.6931, alpha >
    0.9 means x > ln 0.9 = -0.1054."""
    for lo, eps in K_FX_EPS.items():
        viol, pk_bad, e_all, e_big = gpu.exp_probe(-6.95, 5.0, lo)
        assert viol == 0 and pk_bad == 0
        print(f"fast exp vs gsr_blend_expf: max rel {e_all:.4e} (x >= -6.95), {e_big:.4e} (x >= {lo})")
        assert e_big + ULP_PRODUCT <= eps


def test_alpha_cut_device_matches_host(gpu, orc):
    """xs on the device equals the host restatement bit for bit, and it is the least
    float argument that passes the reference's alpha test."""
    rng = np.random.default_rng(11)
    ops = np.concatenate([rng.uniform(0, 1, 50_000), rng.uniform(0, 2e-3, 5_000), 10.0 ** rng.uniform(-44, 3, 5_000),
                          [0.0, -0.0, -1.0, 1.0, 0.99, 1e-3, 1e-3 * 0.999, np.inf, -np.inf, np.nan, 1e-45,
                           3.4e38]]).astype(np.float32)
    dev = gpu.alpha_cut_probe(ops)
    L = orc.lib()
    host = np.array([L.orc_alpha_take_min_x(float(o)) for o in ops], dtype=np.float32)
    same = (dev.view(np.uint32) == host.view(np.uint32))
    assert same.all(), f"{(~same).sum()} mismatches, e.g. op={ops[~same][:3]} dev={dev[~same][:3]} host={host[~same][:3]}"
    for o, x in zip(ops[:2000], host[:2000]):
        assert np.isfinite(x)
        assert L.orc_alpha_taken(float(o), float(x))
        below = np.nextafter(x, np.float32(-np.inf), dtype=np.float32)
        assert not L.orc_alpha_taken(float(o), float(below))
    assert np.isneginf(host[ops.size - 3])          # NaN opacity: fminf(NaN, 0.99) always passes
    assert np.isposinf(host[ops.size - 12]) and np.isposinf(host[ops.size - 10])   # op <= 0: never


def take_parity(gpu, torch, scene, cam, W, H, want, takes_want, mode=None, renderer=None, **kw):
    """Render with the given blend mode (None: the library default), without and with
    diagnostics; the diagnostics kernel must give the same image (so its take map
    describes the shipped kernel's composite).  Returns (L-inf, blend counters)."""
    r = renderer or gpu.Renderer()
    if mode is not None:
        r.set_tuning(KNOB_BLEND_EXP, mode)
    if r.get_tuning(KNOB_BLEND_EXP) != 0:
        # depth-split frames (scenes above 1.5M Gaussians) run the exact blend whatever the
        # mode (tests/test_gpu_depth_split.py); here every frame must be the fast blend's
        r.set_tuning(KNOB_DEPTH_SPLIT, 0)
    img, _ = render_gpu(gpu, torch, scene, cam, W, H, renderer=r, **kw)
    r.set_diagnostics(True)
    img_d, _ = render_gpu(gpu, torch, scene, cam, W, H, renderer=r, **kw)
    takes = r.take_map(W, H)
    counters = r.blend_counters_ex()
    r.set_diagnostics(False)
    assert np.array_equal(img.view(np.uint32), img_d.view(np.uint32))
    exact = r.get_tuning(KNOB_BLEND_EXP) == 0
    linf = assert_frames(img, want, exact=exact)
    bad = takes != takes_want
    assert not bad.any(), (f"{int(bad.sum())} pixels composited other splats, e.g. "
                           f"{np.argwhere(bad)[:3].tolist()}: {takes[bad][:3]} vs {takes_want[bad][:3]}")
    return linf, counters


@pytest.fixture(scope="module")
def c1(gpu, tmp_path_factory):
    return scene_soa(gpu, tmp_path_factory, 10_000, 1)


@pytest.mark.parametrize("ci", range(len(CAMS)))
def test_take_maps_config1(gpu, orc, torch, c1, ci):
    path, soa = c1
    W, H = 640, 480
    cam = cam_for(gpu, W, H, **CAMS[ci])
    scene = gpu.Scene.from_soa(soa)
    want, takes_want = orc.render_takes(soa, cam, W, H, 3.0)
    assert (takes_want & np.uint64(0xFFFFFFFF)).max() > 3
    linf_fast, cf = take_parity(gpu, torch, scene, cam, W, H, want, takes_want, mode=1)
    assert linf_fast < 1e-5
    linf_exact, ce = take_parity(gpu, torch, scene, cam, W, H, want, takes_want, mode=0)
    assert linf_exact == 0.0 and ce["reblended_blocks"] == 0
    assert cf["taken_lanes"] >= ce["taken_lanes"] - 0      # same decisions (re-blends count twice)


@pytest.fixture(scope="module")
def dense(gpu, tmp_path_factory):
    """200k Gaussians at 640x480: most pixels saturate (T < 1e-3)."""
    return scene_soa(gpu, tmp_path_factory, 200_000, 6)


def test_reblend_hook_full_band(gpu, orc, torch, dense):
    """Mode 2 (test hook): a 100 % guard band, so every pixel that saturates is handed
    to the exact re-blend — that path itself must produce the oracle's composite, for
    the suspect pixels it re-blends and the fast pixels beside them."""
    path, soa = dense
    W, H = 640, 480
    cam = cam_for(gpu, W, H, **CAMS[1])
    want, takes_want = orc.render_takes(soa, cam, W, H, 3.0, threads=ORC_THREADS)
    saturated = int(((takes_want & np.uint64(0xFFFFFFFF)) > 0).sum())
    linf, c = take_parity(gpu, torch, gpu.Scene.from_soa(soa), cam, W, H, want, takes_want, mode=2)
    print(f"hook: re-blended blocks {c['reblended_blocks']}, suspect pixels {c['suspect_pixels']} "
          f"of {saturated} covered")
    assert c["reblended_blocks"] > 1000 and c["suspect_pixels"] > 20_000
    _, c1_ = take_parity(gpu, torch, gpu.Scene.from_soa(soa), cam, W, H, want, takes_want, mode=1)
    print(f"default band: re-blended blocks {c1_['reblended_blocks']}, suspect pixels {c1_['suspect_pixels']}")
    assert c1_["suspect_pixels"] < c["suspect_pixels"] // 20


@pytest.mark.parametrize("W,H,k", [(1, 1, 3.0), (37, 23, 3.0), (640, 480, 8.0), (17, 300, 2.0)])
def test_take_maps_odd_sizes(gpu, orc, torch, c1, W, H, k):
    path, soa = c1
    cam = cam_for(gpu, W, H, fov=60)
    want, takes_want = orc.render_takes(soa, cam, W, H, k)
    take_parity(gpu, torch, gpu.Scene.from_soa(soa), cam, W, H, want, takes_want, mode=1, k=k)


def test_take_maps_partial_tiling(gpu, orc, torch, c1):
    """A reference tiling that covers only part of the image (uncovered pixels stay 0)."""
    path, soa = c1
    W, H = 640, 480
    cam = cam_for(gpu, W, H)
    t = gpu.TilingInformation(1, 1, H, W)
    t.num_tile_x, t.num_tile_y, t.width_stride, t.height_stride = (7, 3, 92, 160)
    want, takes_want = orc.render_takes(soa, cam, W, H, 3.0, tiling=(7, 3, 92, 160))
    take_parity(gpu, torch, gpu.Scene.from_soa(soa), cam, W, H, want, takes_want, mode=1, tiling=t)


def test_take_maps_config5_full(gpu, orc, torch, tmp_path_factory):
    """Config 5 at full size (2M 4D Gaussians, 1080p) at t = 0.5: the temporal cull and
    the fast blend together composite exactly the uncut oracle's splats."""
    d = tmp_path_factory.mktemp("c5fx")
    p = str(d / "scene4d.ply")
    gpu.write_synthetic_ply4d(p, 2_000_000, 5)
    soa49 = gpu.read_ply(p, four_d=True)
    scene = gpu.Scene.from_ply(p)
    W, H = 1920, 1080
    cam = gpu.make_camera(position=(0.0, 0.0, 4.0), fov_y=50.0, aspect=W / H)
    want, takes_want = orc.render_takes(orc.temporal(soa49, 0.5), cam, W, H, 3.0, threads=ORC_THREADS)
    r = gpu.Renderer()
    r.set_time(0.5)
    linf, c = take_parity(gpu, torch, scene, cam, W, H, want, takes_want, mode=1, renderer=r)
    print(f"config 5 t=0.5: L-inf {linf:.3g}, re-blended blocks {c['reblended_blocks']} of {(W // 8) * (H // 8)}")
