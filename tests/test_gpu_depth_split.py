"""Depth split (GSR_TUNE_DEPTH_SPLIT) against the oracle.

Phase A bins only the nearest part of the depth order and blends it; a block whose
pixels are not all saturated at the end of its phase-A list saves its transmittance.
Phase B bins the rest of the depth order and resumes those blocks from the saved
transmittance and the colours phase A wrote.  The reference blend walks each tile's
depth-ordered list front to back and stops a pixel at T < 1e-3 (render.cu:323-341), so
a pixel composites the same splats in the same order with the same operations either
way: images are bit-exact against the oracle and the per-pixel take maps (which splats
each pixel composited) equal the oracle's.  The split points below cover phase B doing
nothing (config 3: every block saturates within the nearest ~10 % of the visible
splats, tools/sim/depth_split.py), part of the work, and nearly all of it."""
import os

import numpy as np
import pytest

from conftest import assert_frames, exact_blend, scene_soa
from test_gpu_parity import CAMS, cam_for, render_gpu

pytestmark = pytest.mark.gpu

KNOB_SPLIT, KNOB_PM, KNOB_UNSAT, KNOB_STATE = 23, 24, 25, 26
ORC_THREADS = min(16, len(os.sched_getaffinity(0)))


@pytest.fixture(scope="module")
def torch(gpu):
    import torch as t
    assert t.cuda.is_available()
    return t


@pytest.fixture(scope="module")
def c3(gpu, orc, tmp_path_factory):
    path, soa = scene_soa(gpu, tmp_path_factory, 5_000_000, 3)
    W, H = 1600, 1063
    cam = cam_for(gpu, W, H)
    want, takes = orc.render_takes(soa, cam, W, H, 3.0, threads=ORC_THREADS)
    return gpu.Scene.from_ply(path), soa, cam, W, H, want, takes


def split_renderer(gpu, split, pm=None):
    r = exact_blend(gpu.Renderer())
    r.set_tuning(KNOB_SPLIT, split)
    if pm is not None:
        r.set_tuning(KNOB_PM, pm)
    return r


def check_takes(gpu, torch, r, scene, cam, W, H, want, takes_want, **kw):
    """Diagnostics render (the same kernels with counters and the take map): same image
    as the plain render, take map equal to the oracle's.  Returns the counters."""
    r.set_diagnostics(True)
    img, _ = render_gpu(gpu, torch, scene, cam, W, H, renderer=r, **kw)
    takes = r.take_map(W, H)
    counters = r.blend_counters_ex()
    r.set_diagnostics(False)
    assert_frames(img, want, exact=True)
    bad = takes != takes_want
    assert not bad.any(), (f"{int(bad.sum())} pixels composited other splats, e.g. "
                           f"{np.argwhere(bad)[:3].tolist()}")
    return counters


def test_depth_split_knobs(gpu):
    r = gpu.Renderer()
    assert r.get_tuning(KNOB_SPLIT) == 2 and r.get_tuning(KNOB_PM) == 250
    r.set_tuning(KNOB_PM, 40)
    assert r.get_tuning(KNOB_PM) == 40
    assert r.get_tuning(KNOB_STATE) == 0
    for bad in ((KNOB_SPLIT, 3), (KNOB_PM, 0), (KNOB_PM, 1000), (KNOB_UNSAT, 1), (KNOB_STATE, 1)):
        with pytest.raises(gpu.GsrError):
            r.set_tuning(*bad)


@pytest.mark.parametrize("pm", [20, 60, 250])
def test_config3_split_points(gpu, orc, torch, c3, pm):
    """Config 3 stand-in (5M Gaussians, 1600x1063).  At 2 % of the depth order phase A
    leaves most blocks unsaturated and phase B does most of the work; at 6 % part of it;
    at 25 % (the starting point) phase B does nothing.  Bit-exact with the oracle and the
    same take maps in every case."""
    scene, soa, cam, W, H, want, takes = c3
    r = split_renderer(gpu, 1, pm)
    img, _ = render_gpu(gpu, torch, scene, cam, W, H, renderer=r)
    unsat = r.get_tuning(KNOB_UNSAT)
    nblocks = 4 * ((W + 15) // 16) * ((H + 15) // 16)
    if pm == 20:
        assert unsat > nblocks // 2
    elif pm == 60:
        assert 0 < unsat < nblocks
    else:
        assert unsat == 0
    assert_frames(img, want, exact=True)
    r.set_tuning(KNOB_PM, pm)
    check_takes(gpu, torch, r, scene, cam, W, H, want, takes)
    r.close()


@pytest.mark.parametrize("pm", [20, 60, 250])
def test_config3_key_mode(gpu, orc, torch, c3, pm):
    """Key mode: after the first split frame (which sorts the whole order and sets the
    threshold), each frame partitions its items by a depth threshold and sorts only the
    near part; phase B sorts the far part on its own, only when blocks are left
    unsaturated.  Frames 2 and 3 at each split point: bit-exact, the oracle's take maps;
    the whole depth order is then not readable."""
    scene, soa, cam, W, H, want, takes = c3
    r = split_renderer(gpu, 1, pm)
    for _ in range(2):
        img, _ = render_gpu(gpu, torch, scene, cam, W, H, renderer=r)
        assert_frames(img, want, exact=True)
    unsat = r.get_tuning(KNOB_UNSAT)
    assert (unsat > 0) if pm < 100 else (unsat == 0)
    check_takes(gpu, torch, r, scene, cam, W, H, want, takes)
    with pytest.raises(gpu.GsrError):
        r.read_depth_order(soa.shape[1])
    r.close()


def test_key_mode_records(gpu, orc, torch, c3):
    """In key mode the preprocess writes records only for the Gaussians nearer than the
    threshold; phase B (or gsr_read_splats) writes the far ones.  The records read back
    after a key-mode frame equal those of a frame without the split."""
    scene, soa, cam, W, H, want, _ = c3
    n = soa.shape[1]
    r0 = split_renderer(gpu, 0)
    render_gpu(gpu, torch, scene, cam, W, H, renderer=r0)
    ref = r0.read_splats(n)
    r = split_renderer(gpu, 1, 250)
    for _ in range(3):
        img, _ = render_gpu(gpu, torch, scene, cam, W, H, renderer=r)
    assert r.get_tuning(KNOB_STATE) in (2, 3)
    assert_frames(img, want, exact=True)
    got = r.read_splats(n)
    vis = ref["depth_key"] != 0xFFFFFFFF
    assert vis.sum() > 4_000_000 and got[vis].tobytes() == ref[vis].tobytes()
    for x in (r0, r):
        x.close()


def test_config3_key_mode_camera_change(gpu, orc, torch, c3):
    """The threshold comes from the previous frame; with another camera it is only a
    worse guess (any threshold gives the same image): alternate two cameras."""
    scene, soa, cam, W, H, want, _ = c3
    cam2 = cam_for(gpu, W, H, **CAMS[2])
    want2 = orc.render(soa, cam2, W, H, 3.0, threads=ORC_THREADS)
    r = split_renderer(gpu, 1, 100)
    for i in range(4):
        img, _ = render_gpu(gpu, torch, scene, cam if i % 2 == 0 else cam2, W, H, renderer=r)
        assert_frames(img, want if i % 2 == 0 else want2, exact=True)
    r.close()


def test_config3_speculation_and_miss(gpu, orc, torch, c3):
    """From a split point too small for the scene the controller grows it (phase B runs),
    then shrinks it to 5/4 of the last point that needed phase B and, when it cannot
    shrink further, renders without phase B (state 3) — only while the camera stays the
    one its threshold came from.  A moved camera queues phase B again (state 2, no miss).
    A speculative frame that leaves a block unsaturated — here the same camera on a
    scene with 30 % of the opacity, which the previous frame's threshold does not cover —
    is reported by gsr_sync as GSR_E_OVERFLOW; rendered again it is bit-exact."""
    scene, soa, cam, W, H, want, _ = c3
    r = split_renderer(gpu, 2, 30)
    out = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    states, misses = [], 0
    for i in range(120):
        r.render(scene, cam, W, H, out.data_ptr())
        while r.sync() != 0:                        # the re-render contract (pair buffer, misses)
            misses += 1
            assert misses < 10
            r.render(scene, cam, W, H, out.data_ptr())
        states.append(r.get_tuning(KNOB_STATE))
        if states[-1] == 3 and states.count(3) >= 4:
            break
    assert 2 in states and states[-1] == 3, str(states)
    assert_frames(out.view(3, H, W).cpu().numpy(), want, exact=True)
    far = cam_for(gpu, W, H, pos=(0, 0, 7))
    want_far = orc.render(soa, far, W, H, 3.0, threads=ORC_THREADS)
    r.render(scene, far, W, H, out.data_ptr())
    assert r.sync() == 0 and r.get_tuning(KNOB_STATE) == 2     # a moved camera: phase B queued
    assert_frames(out.view(3, H, W).cpu().numpy(), want_far, exact=True)
    for _ in range(60):                                         # back to speculation on `cam`
        r.render(scene, cam, W, H, out.data_ptr())
        while r.sync() != 0:
            r.render(scene, cam, W, H, out.data_ptr())
        if r.get_tuning(KNOB_STATE) == 3:
            break
    assert r.get_tuning(KNOB_STATE) == 3
    thin = soa.copy()
    thin[3] *= 0.3                                              # opacity (sigmoid applied)
    thin_scene = gpu.Scene.from_soa(thin)
    want_thin = orc.render(thin, cam, W, H, 3.0, threads=ORC_THREADS)
    word = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    # through gsr_render_path_status: the frame's own validity word names the miss
    r.render_path(thin_scene, [cam], W, H, [out.data_ptr()], status=[word.data_ptr()])
    assert r.sync() != 0, "a speculative frame that needed phase B was not reported"
    assert int(word.item()) == 4, "GSR_FRAME_SPEC_MISS not set in the frame's validity word"
    r.render_path(thin_scene, [cam], W, H, [out.data_ptr()], status=[word.data_ptr()])
    assert r.sync() == 0 and r.get_tuning(KNOB_STATE) == 2
    assert int(word.item()) == 0
    assert_frames(out.view(3, H, W).cpu().numpy(), want_thin, exact=True)
    # with completion events off (frames captured into a graph) no frame is
    # queued without phase B — a captured graph would replay that choice — so the same
    # miss cannot happen unreported: back to speculation (a fresh context: the thin
    # scene's unsaturated blocks may have turned this one's split off for good, since the
    # camera never moves), events off, the thin scene
    r.close()
    r = split_renderer(gpu, 2, 30)
    for _ in range(120):
        r.render(scene, cam, W, H, out.data_ptr())
        while r.sync() != 0:
            r.render(scene, cam, W, H, out.data_ptr())
        if r.get_tuning(KNOB_STATE) == 3:
            break
    assert r.get_tuning(KNOB_STATE) == 3
    r.set_tuning(11, 0)
    r.render(scene, cam, W, H, out.data_ptr())
    assert r.get_tuning(KNOB_STATE) == 2, "a frame speculated with completion events off"
    r.render(thin_scene, cam, W, H, out.data_ptr())
    assert r.sync() == 0
    assert_frames(out.view(3, H, W).cpu().numpy(), want_thin, exact=True)
    r.close()


def test_dropin_config3_split(gpu, orc, torch, c3):
    """The drop-in preprocessCUDAGaussians (synchronous, host image, one process-wide
    context) at config-3 size: its frames go through the split too (count mode, then
    the depth threshold, later speculation; it re-renders what it must), every call
    bit-exact.  The reference viewer's tiling (50 x 50 tiles)."""
    scene, soa, cam, W, H, want, _ = c3
    t = gpu.TilingInformation(50, 50, H, W)
    want_t = orc.render(soa, cam, W, H, 3.0, tiling=(t.num_tile_x, t.num_tile_y, t.width_stride, t.height_stride),
                        threads=ORC_THREADS)
    out = None
    for _ in range(12):
        out = gpu.preprocessCUDAGaussians(scene.ptr, scene.n, cam, t.num_tile_y, t.num_tile_x, t.width_stride,
                                          t.height_stride, W, H, 3.0, out=out)
        assert_frames(out, want_t, exact=True)


def test_config3_background_masked_phase_b(gpu, orc, torch, c3):
    """The camera turned off the scene's centre: 15 % of the tiles see past it and never
    saturate, so phase B has blocks to resume on every frame.  In key mode its far sort
    keeps only the far splats whose rect touches an unsaturated tile (summed-area table
    of phase A's block flags).  Frames at a forced split are bit-exact with the oracle's
    take maps; by default the controller grows the split point to 1000, which turns the
    split off (no gain to be had), and the frames stay bit-exact."""
    scene, soa, _, W, H, _, _ = c3
    cam = cam_for(gpu, W, H, look=(1.2, 0, 0))
    want, takes = orc.render_takes(soa, cam, W, H, 3.0, threads=ORC_THREADS)
    r = split_renderer(gpu, 1, 250)
    for _ in range(3):
        img, _ = render_gpu(gpu, torch, scene, cam, W, H, renderer=r)
        assert_frames(img, want, exact=True)
    assert r.get_tuning(KNOB_STATE) == 2 and r.get_tuning(KNOB_UNSAT) > 0
    check_takes(gpu, torch, r, scene, cam, W, H, want, takes)
    r.close()
    r = split_renderer(gpu, 2)
    out = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    checked = 0
    while r.get_tuning(KNOB_PM) < 1000:
        # at the starting point 15 % of the blocks stay unsaturated: the controller turns
        # the split off after the first checked frame (no growth steps)
        r.render(scene, cam, W, H, out.data_ptr())
        while r.sync() != 0:
            r.render(scene, cam, W, H, out.data_ptr())
        checked += 1
        assert checked <= 2, f"split point {r.get_tuning(KNOB_PM)} after {checked} checked frames"
    for i in range(16):
        r.render(scene, cam, W, H, out.data_ptr())
        while r.sync() != 0:
            r.render(scene, cam, W, H, out.data_ptr())
    assert r.get_tuning(KNOB_PM) == 1000 and r.get_tuning(KNOB_STATE) == 0
    assert_frames(out.view(3, H, W).cpu().numpy(), want, exact=True)
    # the same camera never retries the split (nothing in its view can change)
    for i in range(300):
        r.render(scene, cam, W, H, out.data_ptr())
        if i % 16 == 15:
            assert r.sync() == 0
            assert r.get_tuning(KNOB_PM) == 1000 and r.get_tuning(KNOB_STATE) == 0
    assert r.sync() == 0
    # the camera turns back to a view whose tiles all saturate: 256 frames after the split
    # was turned off, on another camera, it is tried again, and it stays on
    centred, want_c = c3[2], c3[5]
    for i in range(300):
        r.render(scene, centred, W, H, out.data_ptr())
        if i % 16 == 15:
            while r.sync() != 0:
                r.render(scene, centred, W, H, out.data_ptr())
    while r.sync() != 0:
        r.render(scene, centred, W, H, out.data_ptr())
    assert r.get_tuning(KNOB_STATE) in (1, 2, 3) and r.get_tuning(KNOB_PM) < 1000
    assert_frames(out.view(3, H, W).cpu().numpy(), want_c, exact=True)
    r.close()


def test_moving_camera_never_retries_the_split(gpu, orc, torch, c3):
    """A camera that keeps moving (an orbit, 0.5 deg per frame) never retries the split
    once background turned it off: its threshold would always come from another view.
    Stopped on a view whose tiles all saturate, it retries (256 frames after the turn-off)
    and stays on.  Frames stay bit-exact."""
    scene, soa, centred, W, H, want_c, _ = c3
    r = split_renderer(gpu, 2)
    out = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")

    def orbit_cam(deg):
        c = cam_for(gpu, W, H)
        gpu.orbit(c, deg, 0.0)
        return c
    pms = []
    for i in range(700):
        c = orbit_cam(40.0 + 0.5 * i)
        r.render(scene, c, W, H, out.data_ptr())
        if i % 8 == 7:
            while r.sync() != 0:
                r.render(scene, c, W, H, out.data_ptr())
            pms.append(r.get_tuning(KNOB_PM))
    off = pms.index(1000)
    assert off < 20, f"the split did not turn off on the orbit: {pms[:20]}"
    assert all(p == 1000 for p in pms[off:]), "the split was retried while the camera kept moving"
    assert r.sync() == 0
    want = orc.render(soa, c, W, H, 3.0, threads=ORC_THREADS)
    assert_frames(out.view(3, H, W).cpu().numpy(), want, exact=True)
    for i in range(300):
        r.render(scene, centred, W, H, out.data_ptr())
        if i % 16 == 15:
            while r.sync() != 0:
                r.render(scene, centred, W, H, out.data_ptr())
    while r.sync() != 0:
        r.render(scene, centred, W, H, out.data_ptr())
    assert r.get_tuning(KNOB_STATE) in (1, 2, 3) and r.get_tuning(KNOB_PM) < 1000
    assert_frames(out.view(3, H, W).cpu().numpy(), want_c, exact=True)
    r.close()


def test_config3_split_off_same_lists(gpu, orc, torch, c3):
    """With the split off the tile lists are the whole depth order's; the default (on
    for this size) renders the same image, and so does the stage API, which never
    splits (gsr_sort lists every pair)."""
    scene, soa, cam, W, H, want, _ = c3
    r0 = split_renderer(gpu, 0)
    img0, _ = render_gpu(gpu, torch, scene, cam, W, H, renderer=r0)
    assert_frames(img0, want, exact=True)
    full = r0.read_pairs()
    r1 = exact_blend(gpu.Renderer())
    assert r1.get_tuning(KNOB_SPLIT) == 2
    img1, _ = render_gpu(gpu, torch, scene, cam, W, H, renderer=r1)
    assert np.array_equal(img1.view(np.uint32), img0.view(np.uint32))
    assert r1.get_tuning(KNOB_UNSAT) == 0
    assert r1.read_pairs().size < full.size // 2           # phase A listed a prefix only
    out = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    for _ in range(3):     # the whole lists overflow the pair buffer sized by phase A's: grown, again
        r1.preprocess(scene, cam, W, H)
        r1.sort()
        r1.blend(out.data_ptr())
        if r1.sync() == 0:
            break
    assert np.array_equal(r1.read_pairs(), full)
    assert np.array_equal(out.view(3, H, W).cpu().numpy().view(np.uint32), img0.view(np.uint32))
    for r in (r0, r1):
        r.close()


def test_reblend_after_split_frame(gpu, orc, torch, c3):
    """gsr_blend again after a split gsr_render (phase B's lists replaced phase A's):
    the library bins phase A again, same image."""
    scene, soa, cam, W, H, want, _ = c3
    r = split_renderer(gpu, 1, 40)
    img, _ = render_gpu(gpu, torch, scene, cam, W, H, renderer=r)
    assert r.get_tuning(KNOB_UNSAT) > 0
    out = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    r.blend(out.data_ptr())
    assert r.sync() == 0
    assert np.array_equal(out.view(3, H, W).cpu().numpy().view(np.uint32), img.view(np.uint32))
    assert_frames(img, want, exact=True)
    r.close()


def test_split_point_adapts(gpu, orc, torch, c3):
    """The split point grows by half after a frame whose phase B had work and shrinks by
    an eighth after 8 checked frames in a row that had none (never below 5/4 of the last
    point that needed phase B); every frame stays bit-exact."""
    scene, soa, cam, W, H, want, _ = c3
    r = split_renderer(gpu, 2, 20)
    out = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    r.render(scene, cam, W, H, out.data_ptr())
    if r.sync() != 0:      # first frame: the pair buffer grew for phase B's lists
        r.set_tuning(KNOB_PM, 20)
        r.render(scene, cam, W, H, out.data_ptr())
        assert r.sync() == 0
    assert r.get_tuning(KNOB_UNSAT) > 0                     # gsr_sync checked the frame: 20 -> 31
    assert r.get_tuning(KNOB_PM) == 31
    r.set_tuning(KNOB_PM, 400)
    for _ in range(20):
        r.render(scene, cam, W, H, out.data_ptr())
        assert r.sync() == 0
    assert r.get_tuning(KNOB_PM) < 400
    assert r.get_tuning(KNOB_UNSAT) == 0
    assert_frames(out.view(3, H, W).cpu().numpy(), want, exact=True)
    r.close()


def test_config3_render_path_split(gpu, orc, torch, c3):
    """Frames in flight (gsr_render_path, 4 lanes) with the split: each lane splits on
    its own workspace; every frame bit-exact."""
    scene, soa, cam, W, H, want, _ = c3
    cam2 = cam_for(gpu, W, H, **CAMS[1])
    want2 = orc.render(soa, cam2, W, H, 3.0, threads=ORC_THREADS)
    r = split_renderer(gpu, 1, 60)
    r.set_frames_in_flight(4)
    cams = [cam, cam2] * 4
    outs = [torch.empty(3 * W * H, dtype=torch.float32, device="cuda") for _ in cams]
    for _ in range(3):
        r.render_path(scene, cams, W, H, [o.data_ptr() for o in outs])
        if r.sync() == 0:
            break
    for i, o in enumerate(outs):
        assert_frames(o.view(3, H, W).cpu().numpy(), want if i % 2 == 0 else want2, exact=True)
    r.close()


def test_config2_split_with_unsaturated_background(gpu, orc, torch, tmp_path_factory):
    """Config 2 (1M, 1080p): 13 % of its tiles never saturate, so phase B always has
    blocks to resume whatever the split point.  Forced split at 30 %, bit-exact, same
    take maps as the oracle."""
    path, soa = scene_soa(gpu, tmp_path_factory, 1_000_000, 2)
    W, H = 1920, 1080
    cam = cam_for(gpu, W, H)
    want, takes = orc.render_takes(soa, cam, W, H, 3.0, threads=ORC_THREADS)
    scene = gpu.Scene.from_ply(path)
    r = split_renderer(gpu, 1, 300)
    img, _ = render_gpu(gpu, torch, scene, cam, W, H, renderer=r)
    assert r.get_tuning(KNOB_UNSAT) > 0
    assert_frames(img, want, exact=True)
    r.set_tuning(KNOB_PM, 300)
    check_takes(gpu, torch, r, scene, cam, W, H, want, takes)
    r.close()


@pytest.mark.parametrize("ci", range(len(CAMS)))
def test_split_odd_sizes_partial_tiling(gpu, orc, torch, tmp_path_factory, ci):
    """Odd image size, a tiling that covers only part of it (pixels outside stay 0), four
    cameras, split points 5 % and 50 %: bit-exact and the oracle's take maps."""
    path, soa = scene_soa(gpu, tmp_path_factory, 200_000, 7)
    W, H = 333, 197
    t = gpu.TilingInformation(1, 1, H, W)
    t.num_tile_x, t.num_tile_y, t.width_stride, t.height_stride = (4, 3, 70, 50)   # 280 x 150 of 333 x 197
    cam = cam_for(gpu, W, H, **CAMS[ci])
    scene = gpu.Scene.from_soa(soa)
    want, takes = orc.render_takes(soa, cam, W, H, 3.0, tiling=(4, 3, 70, 50), threads=ORC_THREADS)
    for pm in (50, 500):
        r = split_renderer(gpu, 1, pm)
        img, _ = render_gpu(gpu, torch, scene, cam, W, H, renderer=r, tiling=t)
        assert_frames(img, want, exact=True)
        r.set_tuning(KNOB_PM, pm)
        check_takes(gpu, torch, r, scene, cam, W, H, want, takes, tiling=t)
        r.close()
