"""Live partition before the global depth sort (GSR_TUNE_DEPTH_COMPACT,
gsr_kernels.hip "live partition"): visible Gaussians first, the passes sort only
those.  The depth order (render.cu:1099-1118: key, ties by index; culled last),
every (tile, Gaussian) pair, the splat records and the image must equal the
unpartitioned sort and the oracle — for scenes with most, some, none and all of
the Gaussians culled, and for a repeated sort of the same preprocessed frame."""
import numpy as np
import pytest

from test_gpu_parity import CAMS, assert_image_parity, c1, cam_for, render_gpu  # noqa: F401 (c1: fixture)

pytestmark = pytest.mark.gpu

KNOB_COMPACT = 18


@pytest.fixture(scope="module")
def torch(gpu):
    import torch as t
    assert t.cuda.is_available()
    return t


def frame(gpu, torch, soa, cam, W, H, compact):
    r = gpu.Renderer()
    r.set_tuning(KNOB_COMPACT, compact)
    img, _ = render_gpu(gpu, torch, gpu.Scene.from_soa(soa), cam, W, H, renderer=r)
    return r, img


@pytest.mark.parametrize("ci", range(len(CAMS)))
def test_partitioned_sort_matches_full_sort_and_oracle(gpu, orc, torch, c1, ci):
    _, soa = c1
    n = soa.shape[1]
    W, H = 640, 480
    cam = cam_for(gpu, W, H, **CAMS[ci])
    r1, img1 = frame(gpu, torch, soa, cam, W, H, 1)
    r0, img0 = frame(gpu, torch, soa, cam, W, H, 0)
    want = orc.preprocess(soa, cam, W, H, 3.0)
    order = r1.read_depth_order(n)
    assert np.array_equal(order, orc.expected_depth_order(want))
    assert np.array_equal(order, r0.read_depth_order(n))
    assert np.array_equal(r1.read_pairs(), r0.read_pairs())
    s1, s0 = r1.read_splats(n), r0.read_splats(n)
    assert np.array_equal(s1["depth_key"], s0["depth_key"])
    assert_image_parity(img1, orc.render(soa, cam, W, H, 3.0))
    assert np.array_equal(img1.view(np.uint32), img0.view(np.uint32))


def test_partition_none_and_all_culled(gpu, orc, torch, c1):
    _, soa = c1
    n = soa.shape[1]
    W, H = 320, 240
    for cam in (cam_for(gpu, W, H, pos=(0, 0, 12), fov=90),      # everything in view
                cam_for(gpu, W, H, pos=(0, 0, 40), look=(0, 0, 80))):   # everything behind
        r, img = frame(gpu, torch, soa, cam, W, H, 1)
        want = orc.preprocess(soa, cam, W, H, 3.0)
        assert np.array_equal(r.read_depth_order(n), orc.expected_depth_order(want))
        assert_image_parity(img, orc.render(soa, cam, W, H, 3.0))


def test_repeated_sort_of_partitioned_frame(gpu, orc, torch, c1):
    _, soa = c1
    n = soa.shape[1]
    W, H = 640, 480
    cam = cam_for(gpu, W, H, **CAMS[2])
    r = gpu.Renderer()
    r.set_tuning(KNOB_COMPACT, 1)
    r.preprocess(gpu.Scene.from_soa(soa), cam, W, H, k=3.0)
    r.sort()
    first = r.read_depth_order(n)
    r.sort()
    assert np.array_equal(r.read_depth_order(n), first)
    want = orc.preprocess(soa, cam, W, H, 3.0)
    assert np.array_equal(first, orc.expected_depth_order(want))
