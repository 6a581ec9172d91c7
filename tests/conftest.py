import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running (full-size configs)")


@pytest.fixture(scope="session")
def gsr():
    # torch first (if present) so libgsr binds to the same HIP runtime as torch
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    import gaussianrenderer_amd
    gaussianrenderer_amd.lib()
    return gaussianrenderer_amd


@pytest.fixture(scope="session")
def orc():
    import _oracle
    _oracle.lib()
    return _oracle


@pytest.fixture(scope="session")
def gpu(gsr):
    if not gsr.device_available():
        pytest.fail("GPU test selected but no HIP device is available")
    return gsr


def scene_soa(gsr, tmp_path_factory, n: int, seed: int):
    d = tmp_path_factory.mktemp(f"scene{n}_{seed}")
    p = os.path.join(str(d), "s.ply")
    gsr.write_synthetic_ply(p, n, seed)
    return p, gsr.read_ply(p)
