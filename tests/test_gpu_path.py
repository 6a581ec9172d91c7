"""Camera paths with frames in flight (gsr_render_path, include/gsr.h): frames
dealt round-robin to F lanes (private workspaces, own streams) must each equal
the oracle's render of that camera bit for bit — the concurrency changes only
when a frame runs, never what it computes.  Covers distinct outputs, a ring of
outputs shared across lanes (the alias wait), 4D times, F = 1, stream ordering
against the caller's stream, and pair-buffer overflow on a child lane."""
import numpy as np
import pytest

from conftest import scene_soa
from test_gpu_parity import assert_image_parity, cam_for

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch(gpu):
    import torch as t
    assert t.cuda.is_available()
    return t


@pytest.fixture(scope="module")
def c1(gpu, tmp_path_factory):
    return scene_soa(gpu, tmp_path_factory, 10_000, 1)


def orbit_cams(gsr, W, H, m):
    from gaussianrenderer_amd import multi
    return [multi.orbit_camera(i % 8, W, H) for i in range(m)]


def render_path_checked(r, scene, cams, W, H, ptrs, **kw):
    """render_path, re-rendered once if an earlier frame overflowed (as the bench warmup does)."""
    for _ in range(3):
        rc = r.render_path(scene, cams, W, H, ptrs, **kw)   # overflow of an earlier frame of the call
        if r.sync() == 0 and rc == 0:                         # ... or of the last ones, seen at sync
            return
    raise AssertionError("render_path kept overflowing")


@pytest.mark.parametrize("F", [1, 2, 3, 4, 8])
def test_path_distinct_outputs_match_oracle(gpu, orc, torch, c1, F):
    path, soa = c1
    W, H = 320, 240
    cams = orbit_cams(gpu, W, H, 8)
    scene = gpu.Scene.from_soa(soa)
    r = gpu.Renderer()
    r.set_frames_in_flight(F)
    assert r.frames_in_flight() == F
    outs = [torch.empty(3 * W * H, device="cuda") for _ in cams]
    render_path_checked(r, scene, cams, W, H, [o.data_ptr() for o in outs])
    for cam, o in zip(cams, outs):
        assert_image_parity(o.view(3, H, W).cpu().numpy(), orc.render(soa, cam, W, H, 3.0))


def test_path_ring_outputs_shared_across_lanes(gpu, orc, torch, c1):
    """Two buffers, three lanes: frames 0 and 2 (lanes 0 and 2) both write buffer A,
    so frame 2 must wait for frame 0; every buffer ends with its LAST frame's image."""
    path, soa = c1
    W, H = 320, 240
    m = 7
    cams = orbit_cams(gpu, W, H, m)
    scene = gpu.Scene.from_soa(soa)
    r = gpu.Renderer()
    r.set_frames_in_flight(3)
    bufs = [torch.full((3 * W * H,), -1.0, device="cuda") for _ in range(2)]
    render_path_checked(r, scene, cams, W, H, [bufs[i % 2].data_ptr() for i in range(m)])
    for b in range(2):
        last = max(i for i in range(m) if i % 2 == b)
        assert_image_parity(bufs[b].view(3, H, W).cpu().numpy(), orc.render(soa, cams[last], W, H, 3.0))


@pytest.mark.parametrize("F,ring,m", [(2, 3, 9), (4, 5, 13), (3, 4, 10)])
def test_path_ring_longer_than_lanes(gpu, orc, torch, c1, F, ring, m):
    """A ring of more buffers than lanes: frame i and frame i + ring write the same
    buffer from lanes that are not ordered with each other (and more than F - 1 frames
    apart), so the later frame must still wait for the earlier writer."""
    path, soa = c1
    W, H = 320, 240
    cams = orbit_cams(gpu, W, H, m)
    scene = gpu.Scene.from_soa(soa)
    r = gpu.Renderer()
    r.set_frames_in_flight(F)
    bufs = [torch.full((3 * W * H,), -1.0, device="cuda") for _ in range(ring)]
    render_path_checked(r, scene, cams, W, H, [bufs[i % ring].data_ptr() for i in range(m)])
    for b in range(ring):
        last = max(i for i in range(m) if i % ring == b)
        assert_image_parity(bufs[b].view(3, H, W).cpu().numpy(), orc.render(soa, cams[last], W, H, 3.0))


def test_path_is_stream_ordered(gpu, orc, torch, c1):
    """Work queued on the caller's stream after the call sees every frame (join), and
    the frames see work queued before it (fork): clear, render, reduce on one stream."""
    path, soa = c1
    W, H = 320, 240
    cams = orbit_cams(gpu, W, H, 6)
    scene = gpu.Scene.from_soa(soa)
    r = gpu.Renderer()
    r.set_frames_in_flight(3)
    s = torch.cuda.Stream()
    outs = [torch.empty(3 * W * H, device="cuda") for _ in cams]
    render_path_checked(r, scene, cams, W, H, [o.data_ptr() for o in outs], stream=s.cuda_stream)
    with torch.cuda.stream(s):
        for o in outs:
            o.fill_(7.0)                        # queued before the frames: must be overwritten
    r.render_path(scene, cams, W, H, [o.data_ptr() for o in outs], stream=s.cuda_stream)
    with torch.cuda.stream(s):
        sums = torch.stack([o.double().sum() for o in outs])  # queued after: must see the images
    s.synchronize()
    assert r.sync() == 0
    for cam, o, sm in zip(cams, outs, sums.cpu().numpy()):
        want = orc.render(soa, cam, W, H, 3.0)
        img = o.view(3, H, W).cpu().numpy()
        assert_image_parity(img, want)
        assert sm == pytest.approx(float(img.astype(np.float64).sum()), rel=1e-12)


def test_path_frame_events_without_join(gpu, orc, torch, c1):
    """gsr_render_path_ex as the multi-GPU frame loop drives it: per-frame completion
    events, no exit join, three chained calls over the same five buffers.  A consumer
    stream waits on each frame's event and copies the image out; the caller's stream
    waits on the consumer before the next call reuses the buffers.  Every copy equals
    its frame's oracle image (a copy taken before its frame finished, or a buffer
    overwritten before its copy, would not)."""
    path, soa = c1
    W, H = 320, 240
    F, chunk, calls = 4, 5, 3
    cams = orbit_cams(gpu, W, H, chunk * calls)
    scene = gpu.Scene.from_soa(soa)
    r = gpu.Renderer()
    r.set_frames_in_flight(F)
    bufs = [torch.empty(3 * W * H, device="cuda") for _ in range(chunk)]
    ptrs = [b.data_ptr() for b in bufs]
    # every lane renders every orbit camera once first (pair buffers at their high-water mark)
    warm = [torch.empty(3 * W * H, device="cuda") for _ in range(4 * 8)]
    render_path_checked(r, scene, [orbit_cams(gpu, W, H, 8)[(i // F) % 8] for i in range(4 * 8)], W, H,
                        [w.data_ptr() for w in warm])
    torch.cuda.synchronize()
    evs = [torch.cuda.Event() for _ in range(chunk)]
    S = torch.cuda.current_stream()
    cons = torch.cuda.Stream()
    snaps = []
    for c in range(calls):
        S.wait_stream(cons)                       # the buffers' previous copies are done
        rc = r.render_path(scene, cams[c * chunk:(c + 1) * chunk], W, H, ptrs, events=evs, join=False,
                           stream=S.cuda_stream)
        assert rc == 0
        with torch.cuda.stream(cons):
            for j in range(chunk):
                cons.wait_event(evs[j])
                snaps.append(bufs[j].clone())
    torch.cuda.synchronize()
    assert r.sync() == 0
    for cam, snap in zip(cams, snaps):
        assert_image_parity(snap.view(3, H, W).cpu().numpy(), orc.render(soa, cam, W, H, 3.0))


def test_path_ex_rejects_unknown_flags(gpu, torch, c1):
    import ctypes
    from gaussianrenderer_amd import _native
    r = gpu.Renderer()
    rc = _native.lib().gsr_render_path_ex(r.ctx, None, 0, 0, None, None, 0, 64, 64, 1, 1, 64, 64, 3.0, None,
                                          None, None, None, ctypes.c_int(4))
    assert rc == _native.GSR_E_ARG


def test_path_4d_times(gpu, orc, torch, tmp_path_factory):
    p = tmp_path_factory.mktemp("p4d") / "scene4d.ply"
    gpu.write_synthetic_ply4d(str(p), 20_000, 5)
    soa49 = gpu.read_ply(str(p), four_d=True)
    scene = gpu.Scene.from_ply(str(p))
    assert scene.is_4d
    W, H = 320, 240
    times = [0.0, 0.3, 0.55, 0.8, 1.0]
    cams = [cam_for(gpu, W, H)] * len(times)
    r = gpu.Renderer()
    r.set_frames_in_flight(3)
    outs = [torch.empty(3 * W * H, device="cuda") for _ in times]
    render_path_checked(r, scene, cams, W, H, [o.data_ptr() for o in outs], times=times)
    for t, o in zip(times, outs):
        want = orc.render(orc.temporal(soa49, t), cams[0], W, H, 3.0)
        assert_image_parity(o.view(3, H, W).cpu().numpy(), want)


def test_path_overflow_on_child_lane(gpu, orc, torch):
    """Huge splats overflow every lane's initial pair buffer: the call reports it (now or
    at sync), the lanes grow, and the re-rendered path is exact."""
    n = 3000
    rng = np.random.default_rng(9)
    soa = np.zeros((38, n), np.float32)
    soa[0:3] = rng.uniform(-0.2, 0.2, (3, n))
    soa[3] = rng.uniform(0.01, 0.05, n)
    soa[4:7] = rng.uniform(1.0, 2.0, (3, n))
    soa[7] = 1.0
    soa[11:38] = rng.normal(0, 0.3, (27, n))
    W, H = 640, 480
    cams = orbit_cams(gpu, W, H, 3)
    scene = gpu.Scene.from_soa(soa)
    r = gpu.Renderer()
    r.set_frames_in_flight(3)
    outs = [torch.empty(3 * W * H, device="cuda") for _ in cams]
    ptrs = [o.data_ptr() for o in outs]
    rc = r.render_path(scene, cams, W, H, ptrs)
    assert rc == -5 or r.sync() == -5
    render_path_checked(r, scene, cams, W, H, ptrs)
    for cam, o in zip(cams, outs):
        assert_image_parity(o.view(3, H, W).cpu().numpy(), orc.render(soa, cam, W, H, 3.0))


def test_overflow_reported_with_completion_events_off(gpu, orc, torch):
    """with GSR_TUNE_COMPLETION_EVENTS 0 (frames captured into a graph) no
    completion event marks finished work, so the render calls cannot report an incomplete
    frame — gsr_sync must: it drains the device and reads the sticky words.  Huge splats
    overflow the initial pair buffer; the re-render after the sync is exact."""
    n = 3000
    rng = np.random.default_rng(11)
    soa = np.zeros((38, n), np.float32)
    soa[0:3] = rng.uniform(-0.2, 0.2, (3, n))
    soa[3] = rng.uniform(0.01, 0.05, n)
    soa[4:7] = rng.uniform(1.0, 2.0, (3, n))
    soa[7] = 1.0
    soa[11:38] = rng.normal(0, 0.3, (27, n))
    W, H = 640, 480
    cam = cam_for(gpu, W, H)
    scene = gpu.Scene.from_soa(soa)
    r = gpu.Renderer()
    r.set_tuning(11, 0)
    out = torch.empty(3 * W * H, device="cuda")
    assert r.render(scene, cam, W, H, out.data_ptr()) == 0        # nothing to report yet
    assert r.sync() == -5, "gsr_sync did not report the overflow with completion events off"
    assert r.sync() == 0                                          # reported once
    r.render(scene, cam, W, H, out.data_ptr())
    assert r.sync() == 0
    assert_image_parity(out.view(3, H, W).cpu().numpy(), orc.render(soa, cam, W, H, 3.0))


def test_path_status_words(gpu, orc, torch):
    """gsr_render_path_status: each frame's validity word names exactly the frames that
    came out incomplete (here: huge splats overflow every lane's initial pair buffer, so
    the first frame of each lane is incomplete), and is 0 for complete frames."""
    n = 3000
    rng = np.random.default_rng(9)
    soa = np.zeros((38, n), np.float32)
    soa[0:3] = rng.uniform(-0.2, 0.2, (3, n))
    soa[3] = rng.uniform(0.01, 0.05, n)
    soa[4:7] = rng.uniform(1.0, 2.0, (3, n))
    soa[7] = 1.0
    soa[11:38] = rng.normal(0, 0.3, (27, n))
    W, H = 640, 480
    cams = orbit_cams(gpu, W, H, 3)
    scene = gpu.Scene.from_soa(soa)
    r = gpu.Renderer()
    r.set_frames_in_flight(3)
    outs = [torch.empty(3 * W * H, device="cuda") for _ in cams]
    words = torch.full((len(cams),), -1, dtype=torch.int32, device="cuda")
    st = [words.data_ptr() + 4 * i for i in range(len(cams))]
    rc = r.render_path(scene, cams, W, H, [o.data_ptr() for o in outs], status=st)
    rc2 = r.sync()
    assert rc == -5 or rc2 == -5
    w = words.cpu().numpy()
    assert ((w & 1) == 1).all(), f"pair overflow not flagged per frame: {w}"
    r.render_path(scene, cams, W, H, [o.data_ptr() for o in outs], status=st)
    assert r.sync() == 0
    assert (words.cpu().numpy() == 0).all()
    for cam, o in zip(cams, outs):
        assert_image_parity(o.view(3, H, W).cpu().numpy(), orc.render(soa, cam, W, H, 3.0))


def test_path_status_word_released_after_error(gpu, orc, torch, c1):
    """a gsr_render_path_status call that fails inside the frame (here the
    image size is refused after the lane took the frame's validity word) must not leave
    the word with the context: a later plain gsr_render on the same context would have
    its column scan write the frame's overflow bits through a pointer the caller may
    since have freed.  The old word keeps its sentinel through both calls."""
    _, soa = c1
    W, H = 64, 48
    cam = cam_for(gpu, W, H)
    scene = gpu.Scene.from_soa(soa)
    r = gpu.Renderer()
    word = torch.full((1,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    out = torch.empty(3 * W * H, device="cuda")
    with pytest.raises(gpu.GsrError):
        r.render_path(scene, [cam], 0, H, [out.data_ptr()], status=[word.data_ptr()])
    r.render(scene, cam, W, H, out.data_ptr())
    assert r.sync() == 0
    assert int(word.cpu()[0]) == 0x5A5A5A5A, "a later frame wrote through the failed call's status word"
    assert_image_parity(out.view(3, H, W).cpu().numpy(), orc.render(soa, cam, W, H, 3.0))


def test_path_error_after_fork_joins_lanes(gpu, orc, torch, tmp_path_factory):
    """a frame failing after the fork (GSR_TUNE_FAIL_FRAME fails frame 3
    of 6 on three lanes, so frames 1 and 2 are still running on lanes 1 and 2) must still
    join those lanes to the caller's stream: a copy queued there right after the error sees
    frames 0-2 complete (outputs pre-filled with NaN), and the next gsr_render on the
    context is correct."""
    _, soa = scene_soa(gpu, tmp_path_factory, 300_000, 21)
    W, H = 1280, 720
    cams = orbit_cams(gpu, W, H, 6)
    scene = gpu.Scene.from_soa(soa)
    r = gpu.Renderer()
    r.set_tuning(gpu.TUNE_DEPTH_SPLIT, 0)
    r.set_frames_in_flight(3)
    outs = [torch.empty(3 * W * H, device="cuda") for _ in cams]
    s = torch.cuda.Stream()
    # warm every lane (workspace high-water marks, bucket splitters) so the failing call
    # queues real frames, not first-frame allocations
    for _ in range(2):
        r.render_path(scene, cams, W, H, [o.data_ptr() for o in outs], stream=s.cuda_stream)
        assert r.sync() == 0
    with torch.cuda.stream(s):
        for o in outs:
            o.fill_(float("nan"))
    r.set_tuning(gpu.TUNE_FAIL_FRAME, 3)
    with pytest.raises(gpu.GsrError):
        r.render_path(scene, cams, W, H, [o.data_ptr() for o in outs], stream=s.cuda_stream)
    assert r.get_tuning(gpu.TUNE_FAIL_FRAME) == 0
    with torch.cuda.stream(s):
        snap = torch.stack(outs[:3]).clone()      # queued on the caller's stream after the error
    s.synchronize()
    for i in range(3):
        img = snap[i].view(3, H, W).cpu().numpy()
        assert np.isfinite(img).all(), f"frame {i}'s lane was not joined: the copy saw its output unfinished"
        assert_image_parity(img, orc.render(soa, cams[i], W, H, 3.0, threads=16))
    torch.cuda.synchronize()
    assert r.sync() == 0
    r.render(scene, cams[4], W, H, outs[4].data_ptr(), stream=s.cuda_stream)
    assert r.sync() == 0
    assert_image_parity(outs[4].view(3, H, W).cpu().numpy(), orc.render(soa, cams[4], W, H, 3.0, threads=16))


def test_path_bad_arguments(gpu, torch, c1):
    r = gpu.Renderer()
    with pytest.raises(gpu.GsrError):
        r.set_frames_in_flight(0)
    with pytest.raises(gpu.GsrError):
        r.set_frames_in_flight(9)
    assert r.render_path(gpu.Scene.from_soa(c1[1]), [], 64, 64, []) == 0


def test_frameshard_reports_depth_budget_overflow(gpu, orc, torch, c1):
    """the adaptive depth-pass budget makes GSR_E_OVERFLOW a steady-state
    event.  Lower every lane's budget to 3 passes on a scene whose keys fit 3 digits,
    then render a scene whose depth keys need all 4 through FrameShard.run: finish()
    must report the incomplete frames (even when a non-blocking check inside a render
    call consumed the flag first), and the re-run must match the oracle."""
    from gaussianrenderer_amd import multi
    path, soa = c1
    W, H, F = 320, 240, 2
    near = gpu.Scene.from_soa(soa)                       # view depth 3..5: keys < 2^24
    far_soa = soa.copy()
    far_soa[2] = np.linspace(-90.0, 1.0, soa.shape[1], dtype=np.float32)   # keys up to ~9.4e7 > 2^24
    far = gpu.Scene.from_soa(far_soa)
    r = gpu.Renderer()
    r.set_tuning(gpu.TUNE_DEPTH_BUCKETS, 0)              # the LSD passes' budget (the bucket sort has none)
    r.set_frames_in_flight(F)
    cam = cam_for(gpu, W, H)
    shard = multi.FrameShard(None, r, near, cam, W, H, steps=4, gather="none", inflight=F)
    for _ in range(8):                                   # >= 4 clean checked frames per lane
        shard.run(4)
        assert not shard.finish("cuda")
    assert r.depth_passes() == 3
    shard.scene = far
    shard.run(4)
    assert shard.finish("cuda"), "frames sorted with too few passes were not reported"
    shard.run(4)                                         # budget back at four passes
    assert not shard.finish("cuda")
    assert r.depth_passes() == 4
    want = orc.render(far_soa, cam, W, H, 3.0)
    for o in shard.outs:
        assert_image_parity(o.view(3, H, W).cpu().numpy(), want)
