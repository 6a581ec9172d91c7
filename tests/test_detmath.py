"""The deterministic elementary functions shared by the kernels and the oracle
(include/gsr_detmath.h): accuracy against float64 and the C99 special cases.
Their GPU twins are compared bit-for-bit in test_gpu_parity.py."""
import math

import numpy as np
import pytest


def ulp_err(got: np.ndarray, ref: np.ndarray) -> np.ndarray:
    ref32 = ref.astype(np.float32)
    spacing = np.spacing(np.abs(ref32)).astype(np.float64)
    spacing = np.maximum(spacing, np.float64(np.finfo(np.float32).smallest_subnormal))
    return np.abs(got.astype(np.float64) - ref) / spacing


def vec(f, *xs):
    return np.array([f(*args) for args in zip(*xs)], dtype=np.float32)


@pytest.fixture(scope="module")
def L(orc):
    return orc.lib()


def test_expf_accuracy(L):
    x = np.linspace(-103.0, 88.7, 200_001, dtype=np.float32)
    got = vec(L.orc_expf, x)
    ref = np.exp(x.astype(np.float64))
    assert ulp_err(got, ref).max() <= 2.0


def test_expf_blend_range_accuracy(L):
    # the blend evaluates exp(-0.5 md2), md2 >= 0 in practice
    x = -np.random.default_rng(0).exponential(3.0, 100_000).astype(np.float32)
    got = vec(L.orc_expf, x)
    assert ulp_err(got, np.exp(x.astype(np.float64))).max() <= 1.0


def test_blend_expf_exhaustive(L):
    """gsr_blend_expf, the blend's exp (render.cu:333), over EVERY float of [-104, 88.75]
    (constant outside, by its clamp): monotone non-decreasing — the alpha test is then a
    threshold on the exp argument (gsr_alpha_take_min_x, the blend's cull) — and within
    1.006 ulp of exp, the accuracy of the Cephes gsr_expf it replaced (1.0103 ulp)."""
    import ctypes
    viol, mu = ctypes.c_int64(0), ctypes.c_double(0)
    L.orc_blend_exp_sweep(-104.0, 88.75, ctypes.byref(viol), ctypes.byref(mu))
    print(f"gsr_blend_expf: {viol.value} monotonicity violations, max {mu.value:.4f} ulp")
    assert viol.value == 0
    assert mu.value <= 1.006


def test_blend_expf_special_cases(L):
    f = L.orc_blend_expf
    assert f(float("-inf")) == 0.0 and f(-104.0) == 0.0 and f(-200.0) == 0.0
    assert f(float("inf")) == float("inf") and f(88.75) == float("inf")
    assert math.isnan(f(float("nan")))
    assert f(0.0) == 1.0 and f(-0.0) == 1.0
    # denormal results keep IEEE rounding (ldexp on the device, two products here)
    assert 0.0 < f(-100.0) < 1.2e-38


def test_sincos_accuracy(L):
    x = np.linspace(-math.pi, math.pi, 200_001, dtype=np.float32)
    for f, r in ((L.orc_sinf, np.sin), (L.orc_cosf, np.cos)):
        got = vec(f, x)
        ref = r(x.astype(np.float64))
        err = np.abs(got.astype(np.float64) - ref)
        # ulp bound away from zeros, absolute bound near them
        assert (err <= np.maximum(2.0 * np.spacing(np.abs(ref.astype(np.float32))).astype(np.float64), 1e-9)).all()


def test_atan2_accuracy(L):
    rng = np.random.default_rng(1)
    y = (rng.standard_normal(200_000) * np.exp(rng.uniform(-20, 20, 200_000))).astype(np.float32)
    x = (rng.standard_normal(200_000) * np.exp(rng.uniform(-20, 20, 200_000))).astype(np.float32)
    got = vec(L.orc_atan2f, y, x)
    ref = np.arctan2(y.astype(np.float64), x.astype(np.float64))
    assert ulp_err(got, ref).max() <= 3.0


def test_atan2_special_cases(L):
    inf, nan = float("inf"), float("nan")
    cases = [(0.0, 0.0), (-0.0, 0.0), (0.0, -0.0), (-0.0, -0.0), (0.0, -1.0), (-0.0, -1.0), (1.0, 0.0),
             (-1.0, -0.0), (inf, inf), (-inf, inf), (inf, -inf), (-inf, -inf), (1.0, inf), (1.0, -inf),
             (-1.0, -inf), (inf, 1.0), (-inf, -5.0)]
    for y, x in cases:
        got = L.orc_atan2f(y, x)
        ref = np.float32(math.atan2(y, x))
        assert got == ref and math.copysign(1, got) == math.copysign(1, ref), (y, x, got, ref)
    assert math.isnan(L.orc_atan2f(nan, 1.0)) and math.isnan(L.orc_atan2f(1.0, nan))


def test_exp_sin_special_cases(L):
    assert L.orc_expf(float("-inf")) == 0.0
    assert L.orc_expf(float("inf")) == float("inf")
    assert L.orc_expf(89.0) == float("inf")
    assert math.isnan(L.orc_expf(float("nan")))
    assert math.isnan(L.orc_sinf(float("inf"))) and math.isnan(L.orc_cosf(float("nan")))
    assert L.orc_expf(0.0) == 1.0 and L.orc_sinf(0.0) == 0.0 and L.orc_cosf(0.0) == 1.0
