"""Pin the CPU oracle and the product's host helpers against the reference's
OWN host code (fixtures in tests/golden/, produced by make_golden.py from
utils/gaussians.cpp, scene/camera.cpp and math/math.cpp compiled in place),
and prove the oracle's splat-major blend equals the reference-literal tiled
blend (tile invariance)."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


def ref_soa(name):
    raw = open(os.path.join(GOLDEN, name), "rb").read()
    n = int(np.frombuffer(raw[:8], "<i8")[0])
    return np.frombuffer(raw[8:], "<f4").reshape(38, n)


@pytest.mark.parametrize("ply,ref", [("synth64.ply", "ref_synth64_soa.bin"), ("weird32.ply", "ref_weird32_soa.bin")])
def test_loaders_match_reference_loader(gsr, orc, ply, ref):
    want = ref_soa(ref)
    path = os.path.join(GOLDEN, ply)
    got_product = gsr.read_ply(path)
    got_oracle = orc.ply_read(path)
    assert got_product.shape == want.shape
    assert np.array_equal(got_product.view(np.uint32), want.view(np.uint32))
    assert np.array_equal(got_oracle.view(np.uint32), want.view(np.uint32))


CAM_FIELDS = ["position", "lookAt", "w_up", "fovY", "aspectRatio", "nearClip", "farClip", "up_vec", "P_matrix",
              "V_matrix", "M_matrix", "f_axis", "r_axis", "u_axis", "r_cam", "r_cam_T", "plane_normals"]


def cam_bytes(gsr, cam):
    return bytes(cam)


def test_camera_matches_reference(gsr):
    manifest = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    for ci, c in enumerate(manifest["cameras"]):
        raw = open(os.path.join(GOLDEN, f"ref_camera_{ci}.bin"), "rb").read()
        snaps = [raw[i:i + 484] for i in range(0, len(raw), 484)]
        cam = gsr.make_camera(position=c["pos"], look_at=c["look"], up=c["up"], fov_y=c["fov"],
                              aspect=c["aspect"], near=c["near"], far=c["far"])
        states = [gsr.Camera.from_buffer_copy(bytes(cam))]
        for op, a, b in c["ops"]:
            if op == "o":
                gsr.orbit(cam, a, b)
            else:
                gsr.lib().gsr_camera_zoom(ctypes.byref(cam), a)
            states.append(gsr.Camera.from_buffer_copy(bytes(cam)))
        assert len(states) == len(snaps)
        for got, snap in zip(states, snaps):
            want = gsr.Camera.from_buffer_copy(snap)
            for f in CAM_FIELDS:
                g = np.array(getattr(got, f), dtype=np.float32).view(np.uint32)
                w = np.array(getattr(want, f), dtype=np.float32).view(np.uint32)
                assert np.array_equal(g, w), (ci, f, getattr(got, f), getattr(want, f))


def test_covariance_chain_matches_reference_math(orc):
    rec = np.fromfile(os.path.join(GOLDEN, "chain_in.bin"), "<f4").reshape(-1, 21)
    want = np.fromfile(os.path.join(GOLDEN, "ref_chain_out.bin"), "<f4").reshape(-1, 4)
    L = orc.lib()
    for r, w in zip(rec, want):
        q = np.ascontiguousarray(r[0:4]); s = np.ascontiguousarray(r[4:7]); xyz = np.ascontiguousarray(r[7:10])
        rc = np.ascontiguousarray(r[12:21]); rct = np.ascontiguousarray(rc.reshape(3, 3).T.ravel())
        out = np.zeros(4, np.float32)
        L.orc_covariance_chain(q.ctypes.data, s.ctypes.data, xyz.ctypes.data, float(r[10]), float(r[11]),
                               rc.ctypes.data, rct.ctypes.data, out.ctypes.data)
        assert np.array_equal(out.view(np.uint32), w.view(np.uint32))


def test_projection_matches_reference_math(orc):
    pin = np.fromfile(os.path.join(GOLDEN, "project_in.bin"), "<f4")
    V, P, pts = pin[:16].copy(), pin[16:32].copy(), pin[32:].reshape(-1, 3)
    want = np.fromfile(os.path.join(GOLDEN, "ref_project_out.bin"), "<f4").reshape(-1, 8)
    L = orc.lib()
    for p, w in zip(pts, want):
        p = np.ascontiguousarray(p)
        tmp = np.zeros(4, np.float32); ndc = np.zeros(4, np.float32)
        L.orc_project(V.ctypes.data, P.ctypes.data, p.ctypes.data, tmp.ctypes.data, ndc.ctypes.data)
        assert np.array_equal(np.concatenate([tmp, ndc]).view(np.uint32), w.view(np.uint32))


@pytest.fixture(scope="module")
def config1(gsr, tmp_path_factory):
    d = tmp_path_factory.mktemp("c1")
    p = os.path.join(str(d), "c1.ply")
    gsr.write_synthetic_ply(p, 10_000, 1)
    return gsr.read_ply(p)


def test_oracle_config1_digest(gsr, orc, config1):
    """Pins the oracle (and the synthetic generator) across machines."""
    manifest = json.load(open(os.path.join(GOLDEN, "manifest.json")))["oracle_config1"]
    cam = gsr.make_camera(position=(0, 0, 4), fov_y=50, aspect=640 / 480)
    img = orc.render(config1, cam, 640, 480, 3.0)
    assert hashlib.sha256(img.tobytes()).hexdigest() == manifest["sha256"]
    crop = np.load(os.path.join(GOLDEN, "oracle_config1_crop.npy"))
    assert np.array_equal(img[:, 180:300, 240:400], crop)


@pytest.mark.parametrize("tiling", [(50, 50, 13, 10), (7, 3, 92, 160), (8, 8, 40, 30), (1, 1, 640, 480)])
def test_tile_invariance(gsr, orc, config1, tiling):
    """Splat-major oracle == reference-literal tiled oracle, bit for bit, for tilings
    that cover the image and ones that do not (8x8x40x30 covers 320x240 only)."""
    cam = gsr.make_camera(position=(0.2, -0.1, 4), fov_y=55, aspect=640 / 480)
    soa = config1[:, :3000]
    a = orc.render(soa, cam, 640, 480, 3.0, tiling=tiling)
    b = orc.render_tiled(soa, cam, 640, 480, 3.0, tiling)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_oracle_multithread_deterministic(gsr, orc, config1):
    cam = gsr.make_camera(position=(0, 0, 4), fov_y=50, aspect=640 / 480)
    a = orc.render(config1, cam, 640, 480, 3.0, threads=1)
    b = orc.render(config1, cam, 640, 480, 3.0, threads=4)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
