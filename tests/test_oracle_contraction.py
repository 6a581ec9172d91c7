"""The parity hole the blend's FMA contraction leaves (round-3 verdict, weak #1).

renderGaussians computes md2 = dx*(i0*dx + i1*dy) + dy*(i2*dx + i3*dy) and
rgb += color*alpha*T in fp32 (render.cu:331, 337) under nvcc's default contraction;
which products it fuses cannot be observed (the CUDA path cannot be built here).  The
oracle and the kernels share one choice (gsr_detmath.h gsr_blend_md2), so the GPU tests,
which demand bits equal to the oracle, cannot see whether the choice matters.  This test
renders config 1 under every other plausible contraction — none, the second products,
the inner or outer sums only, the accumulation unfused — and with the host libm expf or
round 3's Cephes gsr_expf in place of gsr_blend_expf, and measures each against the shipped choice: the images must stay
within the north-star gate (L-inf <= 1e-4) and every pixel must composite the same
splats (take maps equal).  tools/contraction_parity.py runs the same table at configs 2
and 3 (profiles/r04_contraction_parity.txt)."""
import numpy as np
import pytest

from conftest import LINF_TOL

VARIANTS = [(0, 0, 0), (0, 1, 0), (1, 0, 0), (2, 1, 0), (2, 0, 0), (3, 1, 0), (4, 1, 0), (1, 1, 1), (0, 0, 1),
            (1, 1, 2)]


@pytest.fixture(scope="module")
def config1(gsr, orc, tmp_path_factory):
    p = str(tmp_path_factory.mktemp("c1") / "s.ply")
    gsr.write_synthetic_ply(p, 10_000, 1)
    soa = orc.ply_read(p)
    cam = gsr.make_camera(position=(0, 0, 4), fov_y=50, aspect=640 / 480)
    img, takes = orc.render_takes(soa, cam, 640, 480, 3.0)
    return soa, cam, img, takes


@pytest.mark.parametrize("variant", VARIANTS)
def test_contraction_variant_within_gate(orc, config1, variant):
    soa, cam, base, btakes = config1
    with orc.blend_variant(*variant):
        img, takes = orc.render_takes(soa, cam, 640, 480, 3.0)
    diff = np.abs(img.astype(np.float64) - base.astype(np.float64))
    linf = float(diff.max())
    print(f"variant {variant}: L-inf {linf:.3g}, pixels differing {int((diff.max(axis=0) > 0).sum())}, "
          f"take maps differing {int((takes != btakes).sum())}")
    assert (diff.max(axis=0) > 0).any(), "the variant did not change the arithmetic"
    assert linf <= LINF_TOL
    assert np.array_equal(takes, btakes), "a contraction variant composited other splats on some pixel"


def test_shipped_variant_is_the_default(orc, config1):
    soa, cam, base, _ = config1
    with orc.blend_variant(1, 1, 0):
        img, _ = orc.render_takes(soa, cam, 640, 480, 3.0)
    assert np.array_equal(img.view(np.uint32), base.view(np.uint32))


@pytest.fixture(scope="module")
def config2(gsr, orc, tmp_path_factory):
    import os
    p = str(tmp_path_factory.mktemp("c2") / "s.ply")
    gsr.write_synthetic_ply(p, 1_000_000, 2)
    soa = orc.ply_read(p)
    cam = gsr.make_camera(position=(0, 0, 4), fov_y=50, aspect=1920 / 1080)
    threads = min(8, len(os.sched_getaffinity(0)))
    img, takes = orc.render_takes(soa, cam, 1920, 1080, 3.0, threads=threads)
    return soa, cam, img, takes, threads


# measured (profiles/r04_blend_exp_parity.txt): config 1 L-inf 1.19e-7 and no take-map
# difference; config 2 L-inf 7.09e-6 and one pixel whose take decision flips
LIBM_BOUND = {1: (5e-7, 0), 2: (1e-5, 2)}


def _libm_exp_distance(orc, soa, cam, W, H, base, btakes, threads=None):
    kw = {"threads": threads} if threads else {}
    with orc.blend_variant(1, 1, 1):
        img, takes = orc.render_takes(soa, cam, W, H, 3.0, **kw)
    linf = float(np.abs(img.astype(np.float64) - base.astype(np.float64)).max())
    return linf, int((takes != btakes).sum())


def test_libm_exp_bound_config1(orc, config1):
    """the exact blend's exp is gsr_blend_expf (fitted here), not CUDA's
    expf (<= 2 ulp), and no fixture the reference holds pins that choice (parity
    unpinned for the exp).  The oracle with the host libm expf in its place bounds how
    far a correctly rounded exp moves the image: asserted at the measured bound."""
    soa, cam, base, btakes = config1
    linf, flips = _libm_exp_distance(orc, soa, cam, 640, 480, base, btakes)
    print(f"config 1, libm expf: L-inf {linf:.3g}, take-map pixels differing {flips}")
    assert linf <= LIBM_BOUND[1][0] and flips <= LIBM_BOUND[1][1]


def test_libm_exp_bound_config2(orc, config2):
    """The same at BASELINE config 2 (1M Gaussians, 1920x1080): within 1e-5 (measured
    7.09e-6), at most two pixels composite another splat set, well inside the 1e-4 gate."""
    soa, cam, base, btakes, threads = config2
    linf, flips = _libm_exp_distance(orc, soa, cam, 1920, 1080, base, btakes, threads)
    print(f"config 2, libm expf: L-inf {linf:.3g}, take-map pixels differing {flips}")
    assert linf <= LIBM_BOUND[2][0] and flips <= LIBM_BOUND[2][1]
    assert linf <= LINF_TOL
