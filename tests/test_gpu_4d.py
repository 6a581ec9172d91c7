"""Config 5 (own spec): 4D Spacetime-Gaussian-style scenes rendered
at time t with the per-frame temporal cull, against the oracle rendering the
same scene at t with NO cull (oracle/gsr_oracle.c orc_temporal + orc_render).
The cull only drops Gaussians that provably cannot composite, so the images
must be within the parity gate (bit-identical with the exact blend); the test
also checks the cull did drop Gaussians.
Parity vs any reference is unpinned (the reference has no 4D path)."""
import numpy as np
import pytest

from conftest import assert_frames

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch(gpu):
    import torch as t
    assert t.cuda.is_available()
    return t


@pytest.fixture(scope="module")
def s4d(gpu, tmp_path_factory):
    p = tmp_path_factory.mktemp("s4d") / "scene4d.ply"
    gpu.write_synthetic_ply4d(str(p), 30_000, 5)
    return p, gpu.read_ply(str(p), four_d=True)


def render(gsr, torch, scene, cam, W, H, t, renderer=None):
    r = renderer or gsr.Renderer()
    out = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    for _ in range(3):
        r.render(scene, cam, W, H, out.data_ptr(), time=t)
        if r.sync() == 0:
            break
    return out.view(3, H, W).cpu().numpy(), r


@pytest.mark.parametrize("t", [0.0, 0.25, 0.5, 0.9, 1.0])
def test_4d_frame_matches_uncut_oracle(gpu, orc, torch, s4d, t):
    path, soa49 = s4d
    W, H = 640, 480
    cam = gpu.make_camera(position=(0.0, 0.0, 4.0), fov_y=50.0, aspect=W / H)
    scene = gpu.Scene.from_ply(str(path))
    assert scene.is_4d
    got, r = render(gpu, torch, scene, cam, W, H, t)
    at_t = orc.temporal(soa49, t)
    want = orc.render(at_t, cam, W, H, 3.0)
    assert (want != 0).sum() > 1000
    assert_frames(got, want)
    # the temporal cull removed Gaussians the oracle keeps alive (status 2 = visible)
    spl = r.read_splats(soa49.shape[1])
    live_gpu = int((spl["depth_key"] != 0xFFFFFFFF).sum())
    live_orc = int((orc.preprocess(at_t, cam, W, H, 3.0)["status"] == 2).sum())
    assert live_gpu < live_orc


def test_4d_scene_from_soa_and_orbit(gpu, orc, torch, s4d):
    path, soa49 = s4d
    W, H = 320, 200
    cam = gpu.make_camera(position=(0.0, 0.0, 4.0), fov_y=50.0, aspect=W / H)
    gpu.orbit(cam, 60.0, 10.0)
    scene = gpu.Scene.from_soa(soa49)
    r = gpu.Renderer()
    for t in (0.1, 0.7):
        got, _ = render(gpu, torch, scene, cam, W, H, t, renderer=r)
        want = orc.render(orc.temporal(soa49, t), cam, W, H, 3.0)
        assert_frames(got, want)


def test_4d_dropin_renders_first_frame(gpu, orc, s4d):
    """preprocessCUDAGaussians on a 4D scene block (the viewer's ABI has no time
    argument): the block is recognised from its header and rendered at t = 0."""
    path, soa49 = s4d
    W, H = 200, 150
    cam = gpu.make_camera(position=(0.0, 0.0, 4.0), fov_y=50.0, aspect=W / H)
    scene = gpu.Scene.from_ply(str(path))
    t = gpu.TilingInformation(50, 50, H, W)
    got = gpu.preprocessCUDAGaussians(scene.ptr, scene.n, cam, t.num_tile_y, t.num_tile_x, t.width_stride,
                                      t.height_stride, W, H, 3.0)
    want = orc.render(orc.temporal(soa49, 0.0), cam, W, H, 3.0)
    assert_frames(got, want)
    # the reference loader symbol keeps the reference's semantics: a 3D scene
    ptr, n = gpu.loadGaussianCudaFromPly(str(path))
    try:
        got3 = gpu.preprocessCUDAGaussians(ptr, n, cam, t.num_tile_y, t.num_tile_x, t.width_stride,
                                           t.height_stride, W, H, 3.0)
    finally:
        from gaussianrenderer_amd._native import lib
        lib().gsr_scene_free(ptr)
    assert_frames(got3, orc.render(soa49[:38].copy(), cam, W, H, 3.0))
