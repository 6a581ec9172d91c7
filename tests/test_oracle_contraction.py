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
