"""The reference's standalone sort entry points (render.cuh:8-11,
onesweep.cuh:8) on the GPU.  test_onesweep_reference_harness restates the
reference's only pass/fail check (src/projects/test/onesweep.cpp:120-218:
consecutive sizes 2048..4096, seeds 12345+, keys uniform in [0, 2^24-1],
output must equal a correct sort and be non-decreasing) with numpy's sort in
place of CUB."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def one_sweep_sort(L, keys: np.ndarray, max_val: int):
    keys = np.ascontiguousarray(keys, dtype=np.int32)
    out = np.zeros_like(keys)
    ms = ctypes.c_float(-1.0)
    L.oneSweepSort(keys.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                   out.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), keys.size, max_val, ctypes.byref(ms))
    return out, ms.value


def test_onesweep_reference_harness(gpu):
    L = gpu.lib()
    max_val = (1 << 24) - 1
    for N in range(2048, 4097, 7):
        rng = np.random.default_rng(12345 + N % 3)
        keys = rng.integers(0, max_val + 1, N).astype(np.int32)
        out, ms = one_sweep_sort(L, keys, max_val)
        assert np.all(out[1:] >= out[:-1]), N
        assert np.array_equal(out, np.sort(keys)), N
        assert ms > 0


@pytest.mark.parametrize("N", [1, 2, 255, 256, 257, 4095, 4096, 4097, 65537, 1 << 20, 1 << 22])
def test_onesweep_sizes(gpu, N):
    rng = np.random.default_rng(N)
    keys = rng.integers(0, 1 << 24, N).astype(np.int32)
    out, _ = one_sweep_sort(gpu.lib(), keys, (1 << 24) - 1)
    assert np.array_equal(out, np.sort(keys))


def test_onesweep_full_32bit_and_duplicates(gpu):
    rng = np.random.default_rng(7)
    keys = rng.integers(-2**31, 2**31, 100_000, dtype=np.int64).astype(np.int32)
    keys[::3] = 42
    out, _ = one_sweep_sort(gpu.lib(), keys, 2**31 - 1)
    # the reference sorts 4 unsigned 8-bit digits (onesweep.cu:197-198): unsigned order
    assert np.array_equal(out.view(np.uint32), np.sort(keys.view(np.uint32)))


@pytest.mark.parametrize("num_bits", [48, 44, 32, 13, 8])
def test_gaussian_pair_sort_stable(gpu, num_bits):
    """oneSweep3DGaussianSort: host lightWeightGaussian[] sorted in place, stably,
    by the low 8*ceil(num_bits/8) bits of radix_id (render.cu:194-264)."""
    from gaussianrenderer_amd._native import Lwg
    rng = np.random.default_rng(num_bits)
    N = 300_000
    tiles = rng.integers(0, 2500, N).astype(np.uint64)
    depth = rng.integers(3_000_000, 3_000_400, N).astype(np.uint64)      # many ties
    radix = (tiles << np.uint64(32)) | depth
    arr = (Lwg * N)()
    raw = np.frombuffer(arr, dtype=np.dtype([("radix_id", "<u8"), ("gaussian_id", "<u4"), ("pad", "<u4")]))
    raw["radix_id"] = radix
    raw["gaussian_id"] = np.arange(N, dtype=np.uint32)
    ms = ctypes.c_float(-1.0)
    gpu.lib().oneSweep3DGaussianSort(arr, N, num_bits, ctypes.byref(ms))
    nb = 8 * ((num_bits + 7) // 8)
    mask = np.uint64((1 << nb) - 1) if nb < 64 else np.uint64(0xFFFFFFFFFFFFFFFF)
    order = np.argsort(radix & mask, kind="stable")
    assert np.array_equal(raw["gaussian_id"], order.astype(np.uint32))
    assert np.array_equal(raw["radix_id"], radix[order])
    assert ms.value > 0
