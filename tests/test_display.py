"""Display interop (include/gsr_gl.h): the frame is written
straight into the viewer's colour SSBO instead of the reference's
device -> host vector -> glBufferSubData round trip (canvas.cpp:337-351).

No GL context can exist in this image (no display, no EGL / OSMesa), so the GL
registration itself is exercised only up to its refusal; the render-into-target
path is exercised with device-memory targets on the GPU, bit-exact against the
plain render and the oracle."""
import ctypes
import os

import numpy as np
import pytest

from conftest import assert_frames

from conftest import scene_soa
from gaussianrenderer_amd import _native


# ---------------------------------------------------------------- CPU (no GL, no device)

def test_no_gl_context_is_refused_cleanly(gsr):
    L = gsr.lib()
    assert gsr.display_gl_current() is False
    p = ctypes.c_void_p(1)
    assert L.gsr_display_register_gl(7, ctypes.byref(p)) == _native.GSR_E_DISPLAY
    assert p.value is None
    assert b"no GL context" in L.gsr_last_error()
    with pytest.raises(_native.GsrError) as e:
        gsr.DisplayTarget.from_gl(7)
    assert e.value.code == _native.GSR_E_DISPLAY
    assert L.gsr_display_register_gl(0, ctypes.byref(p)) == _native.GSR_E_ARG
    assert L.gsr_display_register_gl(7, None) == _native.GSR_E_ARG


def test_dropin_gl_without_context_reports_and_returns(gsr, capfd):
    cam = gsr.make_camera(aspect=4 / 3)
    gsr.preprocessCUDAGaussiansGL(0, 3, 0, cam, 50, 50, 13, 10, 640, 480, 3.0)
    err = capfd.readouterr().err
    assert "preprocessCUDAGaussiansGL: register" in err and "no GL context" in err
    gsr.preprocessCUDAGaussiansGL(0, 3, 0, cam, 50, 50, 13, 10, 0, 480, 3.0)
    assert "preprocessCUDAGaussiansGL: argument" in capfd.readouterr().err


def test_device_target_arguments(gsr):
    L = gsr.lib()
    p = ctypes.c_void_p()
    assert L.gsr_display_wrap_device(None, 100, ctypes.byref(p)) == _native.GSR_E_ARG
    assert L.gsr_display_wrap_device(ctypes.c_void_p(4096), 0, ctypes.byref(p)) == _native.GSR_E_ARG
    # wrapping never dereferences the pointer
    t = gsr.DisplayTarget.from_device(4096, 12 * 64 * 48)
    assert t.ptr
    r = gsr.Renderer()
    cam = gsr.make_camera(aspect=4 / 3)
    # size checks come before any device work
    rc = L.gsr_render_display(r.ctx, t.ptr, None, 0, 0, ctypes.byref(cam), 0, 48, 1, 1, 64, 48, 3.0, None)
    assert rc == _native.GSR_E_ARG
    assert L.gsr_render_display(None, t.ptr, None, 0, 0, ctypes.byref(cam), 64, 48, 1, 1, 64, 48, 3.0,
                                None) == _native.GSR_E_ARG
    assert L.gsr_render_display(r.ctx, None, None, 0, 0, ctypes.byref(cam), 64, 48, 1, 1, 64, 48, 3.0,
                                None) == _native.GSR_E_ARG
    t.free()
    assert t.ptr == 0
    assert L.gsr_display_free(None) == _native.GSR_OK


# ---------------------------------------------------------------- GPU

@pytest.fixture(scope="module")
def torch(gpu):
    import torch as t
    assert t.cuda.is_available()
    return t


@pytest.fixture(scope="module")
def d1(gpu, tmp_path_factory):
    return scene_soa(gpu, tmp_path_factory, 8_000, 21)


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,extra", [(640, 480, 0), (333, 217, 4096), (64, 48, 1)])
def test_render_display_device_target_bit_exact(gpu, orc, torch, d1, W, H, extra):
    """A target larger than the image (an SSBO sized for a bigger window) is
    written in its first 3*W*H floats and left alone after them."""
    path, soa = d1
    scene = gpu.Scene.from_soa(soa)
    cam = gpu.make_camera(position=(0.3, -0.2, 4.0), fov_y=50.0, aspect=W / H)
    r = gpu.Renderer()
    buf = torch.full((3 * W * H + extra,), 7.0, dtype=torch.float32, device="cuda")
    t = gpu.DisplayTarget.from_device(buf.data_ptr(), buf.numel() * 4)
    for _ in range(3):
        r.render_display(t, scene, cam, W, H)
        if r.sync() == 0:
            break
    got = buf[: 3 * W * H].view(3, H, W).cpu().numpy()
    assert (buf[3 * W * H:] == 7.0).all()
    want = orc.render(soa, cam, W, H, 3.0)
    assert (want != 0).sum() > 100
    assert_frames(got, want)
    plain = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    r.render(scene, cam, W, H, plain.data_ptr())
    r.sync()
    assert torch.equal(plain, buf[: 3 * W * H])
    t.free()


@pytest.mark.gpu
def test_render_display_undersized_target_untouched(gpu, torch, d1):
    path, soa = d1
    scene = gpu.Scene.from_soa(soa)
    W, H = 320, 240
    cam = gpu.make_camera(aspect=W / H)
    buf = torch.full((3 * W * H - 1,), 5.0, dtype=torch.float32, device="cuda")
    t = gpu.DisplayTarget.from_device(buf.data_ptr(), buf.numel() * 4)
    r = gpu.Renderer()
    with pytest.raises(_native.GsrError) as e:
        r.render_display(t, scene, cam, W, H)
    assert e.value.code == _native.GSR_E_ARG
    torch.cuda.synchronize()
    assert (buf == 5.0).all()


@pytest.mark.gpu
def test_render_display_4d_scene(gpu, orc, torch, tmp_path):
    p = str(tmp_path / "s4d.ply")
    gpu.write_synthetic_ply4d(p, 6000, 3)
    soa49 = gpu.read_ply(p, four_d=True)
    scene = gpu.Scene.from_ply(p)
    W, H = 256, 192
    cam = gpu.make_camera(aspect=W / H)
    buf = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    t = gpu.DisplayTarget.from_device(buf.data_ptr(), buf.numel() * 4)
    r = gpu.Renderer()
    for _ in range(3):
        r.render_display(t, scene, cam, W, H, time=0.4)
        if r.sync() == 0:
            break
    want = orc.render(orc.temporal(soa49, 0.4), cam, W, H, 3.0)
    assert_frames(buf.view(3, H, W).cpu().numpy(), want)
