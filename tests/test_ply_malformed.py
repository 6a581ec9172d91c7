"""Malformed and hostile .ply files through both PLY readers (CPU).

The reference's loader (misc.cu:21-105) trusts its input: counts, property lists and
data lengths come straight from the file.  gsr_ply_read_host_ex (both modes: the
reference-exact reader and the typed one) and the oracle's orc_ply_read_ex must turn
every malformed file into an error code — never a crash, a hang, an out-of-bounds
access or undefined behaviour.  tests/test_sanitizers.py runs this file again against
the ASan + UBSan builds of both libraries (tools/asan.mk), where any out-of-bounds
read or write, overflow or bad float-to-int conversion aborts the run."""
import ctypes
import os
import struct

import numpy as np
import pytest

PROPS = (["x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"] + [f"f_rest_{i}" for i in range(45)]
         + ["opacity", "scale_0", "scale_1", "scale_2", "rot_0", "rot_1", "rot_2", "rot_3"])
MAX_N = 1 << 20           # the tests never allocate arrays for more Gaussians than this


def header(n, fmt="binary_little_endian 1.0", props=PROPS, ptype="float", extra="", end=True):
    h = f"ply\nformat {fmt}\n{extra}element vertex {n}\n" + "".join(f"property {ptype} {p}\n" for p in props)
    return (h + ("end_header\n" if end else "")).encode()


def rows(n, nprop=len(PROPS), seed=0):
    return np.random.default_rng(seed).normal(0, 1, (n, nprop)).astype("<f4").tobytes()


def gsr_read(gsr, path, flags, narrays):
    """Count call, then (for a sane count) the read: the first nonzero code, else 0."""
    L = gsr.lib()
    n = ctypes.c_int64(-1)
    rc = L.gsr_ply_read_host_ex(path.encode(), None, narrays, 0, ctypes.byref(n), flags, None)
    if rc:
        return rc
    if not 0 <= n.value <= MAX_N:
        return -100                     # the count call accepted an absurd count
    soa = np.zeros((narrays, max(1, n.value)), np.float32)
    return L.gsr_ply_read_host_ex(path.encode(), soa.ctypes.data, narrays, n.value, ctypes.byref(n), flags, None)


def orc_read(orc, path, narrays):
    L = orc.lib()
    n = ctypes.c_int64(-1)
    rc = L.orc_ply_read_ex(path.encode(), None, narrays, 0, ctypes.byref(n))
    if rc:
        return rc
    if not 0 <= n.value <= MAX_N:
        return -100
    soa = np.zeros((narrays, max(1, n.value)), np.float32)
    return L.orc_ply_read_ex(path.encode(), soa.ctypes.data, narrays, n.value, ctypes.byref(n))


MODES = [(0, 38), (0, 49), (1, 38), (1, 49), (2, 59), (3, 59)]    # (flags, narrays): reference / typed / SH-3


def malformed_cases():
    """name -> (bytes, which readers must refuse it: 'all', 'typed' or 'none' (any code,
    but it must return))."""
    good = header(8) + rows(8)
    cases = {
        "empty": (b"", "all"),
        "magic_only": (b"ply\n", "all"),
        "truncated_rows": (header(100) + rows(50), "all"),
        "truncated_mid_row": (header(8) + rows(8)[:-7], "all"),
        "count_beyond_file": (header(1_000_000_000) + rows(4), "all"),
        "count_int32_overflow": (header(2 ** 31) + rows(4), "all"),
        "count_int64_overflow": (header("99999999999999999999") + rows(4), "all"),
        "count_negative": (header(-5) + rows(4), "all"),
        "count_not_a_number": (header("lots") + rows(4), "all"),
        "no_end_header": (header(8, end=False), "all"),
        "no_vertex_element": (b"ply\nformat binary_little_endian 1.0\nelement face 3\nproperty float x\nend_header\n",
                              "all"),
        "unsupported_format": (header(8, fmt="binary_middle_endian 1.0") + rows(8), "all"),
        # typed reader only (the reference reads every property as a 4-B float by design)
        "list_float_count": (b"ply\nformat binary_little_endian 1.0\nelement vertex 2\nproperty float x\n"
                             b"property list float int idx\nend_header\n" + struct.pack("<ff", 1, 2) * 2, "typed"),
        "list_bad_type": (b"ply\nformat binary_little_endian 1.0\nelement vertex 2\nproperty float x\n"
                          b"property list uchar quux idx\nend_header\n" + b"\0" * 16, "typed"),
        "list_count_past_eof": (b"ply\nformat binary_little_endian 1.0\nelement vertex 2\nproperty float x\n"
                                b"property list uint int idx\nend_header\n" + struct.pack("<fI", 1.0, 2 ** 31), "typed"),
        "list_negative_count": (b"ply\nformat binary_little_endian 1.0\nelement vertex 2\nproperty float x\n"
                                b"property list int int idx\nend_header\n" + struct.pack("<fi", 1.0, -3) * 2, "typed"),
        "property_before_element": (b"ply\nformat binary_little_endian 1.0\nproperty float x\nelement vertex 1\n"
                                    b"end_header\n" + b"\0" * 4, "typed"),
        "bad_property_type": (header(2, ptype="quad") + rows(2), "typed"),
        "ascii_short_row": (b"ply\nformat ascii 1.0\nelement vertex 3\nproperty float x\nproperty float y\n"
                            b"end_header\n1 2\n3\n5 6\n", "typed"),
        "ascii_missing_rows": (b"ply\nformat ascii 1.0\nelement vertex 5\nproperty float x\nend_header\n1\n2\n", "typed"),
        "ascii_list_nan_count": (b"ply\nformat ascii 1.0\nelement vertex 1\nproperty float x\n"
                                 b"property list uchar int idx\nend_header\n1 nan 2 3\n", "typed"),
        "ascii_list_huge_count": (b"ply\nformat ascii 1.0\nelement vertex 1\nproperty float x\n"
                                  b"property list uint int idx\nend_header\n1 4000000000 1 2\n", "typed"),
        "ascii_list_short": (b"ply\nformat ascii 1.0\nelement vertex 1\nproperty float x\n"
                             b"property list uchar int idx\nend_header\n1 5 1 2\n", "typed"),
        # valid (an element without properties holds no data), but it used to loop ~1e11 times
        "empty_element_huge_count": (b"ply\nformat binary_little_endian 1.0\nelement junk 4000000000000000000\n"
                                     b"element vertex 1\nproperty float x\nend_header\n" + b"\0" * 4, "none"),
        "big_endian_truncated": (header(8, fmt="binary_big_endian 1.0") + rows(3), "typed"),
    }
    return cases, good


@pytest.fixture(scope="module")
def corpus(tmp_path_factory):
    d = tmp_path_factory.mktemp("plyfuzz")
    cases, good = malformed_cases()
    out = {}
    for name, (data, who) in cases.items():
        p = str(d / f"{name}.ply")
        with open(p, "wb") as f:
            f.write(data)
        out[name] = (p, who)
    p = str(d / "good.ply")
    with open(p, "wb") as f:
        f.write(good)
    out["good"] = (p, None)
    return out


def test_good_file_reads_in_every_mode(gsr, orc, corpus):
    p, _ = corpus["good"]
    for flags, na in MODES:
        assert gsr_read(gsr, p, flags, na) == 0
    for na in (38, 49, 59):
        assert orc_read(orc, p, na) == 0


@pytest.mark.parametrize("name", sorted(malformed_cases()[0]))
def test_malformed_file_is_an_error(gsr, orc, corpus, name):
    p, who = corpus[name]
    for flags, na in MODES:
        typed = flags & 1
        rc = gsr_read(gsr, p, flags, na)
        assert rc != -100, f"{name}: count accepted (flags {flags})"
        if who == "all" or (who == "typed" and typed):
            assert rc < 0, f"{name}: accepted (flags {flags}, {na} arrays)"
    rc = orc_read(orc, p, 38)
    assert rc != -100
    if who == "all":
        assert rc < 0, f"{name}: the oracle's reader accepted it"


def test_negative_f_rest_index_is_skipped(gsr, orc, tmp_path):
    """f_rest_-15 would index the array before sh[0] (misc.cu:76 checks only j < 24):
    both readers skip it."""
    props = PROPS + ["f_rest_-15", "f_rest_-1"]
    p = str(tmp_path / "neg.ply")
    with open(p, "wb") as f:
        f.write(header(4, props=props) + rows(4, len(props)))
    for flags, na in MODES:
        assert gsr_read(gsr, p, flags, na) == 0
    ref = gsr.read_ply(p)
    clean = str(tmp_path / "clean.ply")
    data = np.frombuffer(rows(4, len(props)), "<f4").reshape(4, len(props))[:, :len(PROPS)]
    with open(clean, "wb") as f:
        f.write(header(4) + data.tobytes())
    assert np.array_equal(ref, gsr.read_ply(clean))
    assert orc_read(orc, p, 38) == 0 and np.array_equal(orc.ply_read(p), orc.ply_read(clean))


def test_mutated_files_never_crash(gsr, orc, tmp_path):
    """Seeded byte mutations of a valid file (header and data): any code is allowed, but
    every read returns (under the sanitizer builds: with no memory error)."""
    base = bytearray(header(16) + rows(16))
    hdr_len = len(header(16))
    rng = np.random.default_rng(1234)
    for k in range(120):
        b = bytearray(base)
        for _ in range(int(rng.integers(1, 6))):
            pos = int(rng.integers(0, hdr_len if k % 2 == 0 else len(b)))
            b[pos] = int(rng.integers(0, 256))
        if k % 7 == 0:
            b = b[:int(rng.integers(1, len(b)))]
        p = str(tmp_path / f"m{k}.ply")
        with open(p, "wb") as f:
            f.write(bytes(b))
        for flags, na in MODES:
            assert gsr_read(gsr, p, flags, na) != -100
        assert orc_read(orc, p, 38) != -100
        os.remove(p)
