// gsr_gl.cpp — display interop (include/gsr_gl.h): the
// frame is rendered straight into the viewer's colour SSBO (canvas.cpp:118-121,
// read by canvas.hpp:83-106) instead of the reference's device -> host vector
// -> glBufferSubData round trip (canvas.cpp:337-351).  The SSBO layout is our
// image layout (planar float32 [3][H][W]), so the render writes it unchanged.
//
// GL is resolved with dlopen at run time: libgsr keeps no GL link dependency,
// and without a current context every GL call is refused with GSR_E_DISPLAY
// before HIP's interop is touched.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
// after hip_runtime.h: the interop header uses its types
#include <hip/hip_gl_interop.h>

#include <cstdio>
#include <mutex>

#include "gsr.h"
#include "gsr_gl.h"
#include "gsr_internal.h"

using gsr::set_error;

struct gsr_display_target {
    hipGraphicsResource_t res = nullptr;   // registered GL buffer (null: device memory)
    unsigned int gl_buffer = 0;
    void* dev = nullptr;                   // wrapped device memory
    size_t bytes = 0;
};

namespace {

#define HIP_OR(code, expr)                                                                            \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess) return set_error(code, "%s failed: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

using CurrentFn = void* (*)();

CurrentFn lookup(const char* lib, const char* sym) {
    void* h = dlopen(lib, RTLD_LAZY | RTLD_LOCAL);
    return h ? reinterpret_cast<CurrentFn>(dlsym(h, sym)) : nullptr;
}

bool gl_current() {
    static const CurrentFn glx = lookup("libGL.so.1", "glXGetCurrentContext");
    static const CurrentFn egl = lookup("libEGL.so.1", "eglGetCurrentContext");
    return (glx && glx()) || (egl && egl());
}

// Map the target on `s`; *ptr / *bytes describe the writable image memory.
int map_target(gsr_display_target* t, hipStream_t s, float** ptr, size_t* bytes) {
    if (!t->res) {
        *ptr = static_cast<float*>(t->dev);
        *bytes = t->bytes;
        return GSR_OK;
    }
    HIP_OR(GSR_E_DISPLAY, hipGraphicsMapResources(1, &t->res, s));
    void* p = nullptr;
    size_t sz = 0;
    if (hipGraphicsResourceGetMappedPointer(&p, &sz, t->res) != hipSuccess) {
        (void)hipGraphicsUnmapResources(1, &t->res, s);
        return set_error(GSR_E_DISPLAY, "hipGraphicsResourceGetMappedPointer failed for GL buffer %u",
                         t->gl_buffer);
    }
    *ptr = static_cast<float*>(p);
    *bytes = sz;
    return GSR_OK;
}

int unmap_target(gsr_display_target* t, hipStream_t s) {
    if (t->res) HIP_OR(GSR_E_DISPLAY, hipGraphicsUnmapResources(1, &t->res, s));
    return GSR_OK;
}

}  // namespace

extern "C" int gsr_display_gl_current(void) { return gl_current() ? 1 : 0; }

extern "C" int gsr_display_register_gl(unsigned int gl_buffer, gsr_display_target** out) {
    if (!out) return set_error(GSR_E_ARG, "gsr_display_register_gl: null output");
    *out = nullptr;
    if (gl_buffer == 0) return set_error(GSR_E_ARG, "gsr_display_register_gl: buffer 0 is not a GL buffer");
    if (!gl_current())
        return set_error(GSR_E_DISPLAY, "gsr_display_register_gl: no GL context is current on this thread");
    auto* t = new gsr_display_target();
    t->gl_buffer = gl_buffer;
    const hipError_t e = hipGraphicsGLRegisterBuffer(&t->res, gl_buffer, hipGraphicsRegisterFlagsWriteDiscard);
    if (e != hipSuccess) {
        delete t;
        return set_error(GSR_E_DISPLAY, "hipGraphicsGLRegisterBuffer(%u) failed: %s", gl_buffer,
                         hipGetErrorString(e));
    }
    *out = t;
    return GSR_OK;
}

extern "C" int gsr_display_wrap_device(void* d_ptr, size_t bytes, gsr_display_target** out) {
    if (!out) return set_error(GSR_E_ARG, "gsr_display_wrap_device: null output");
    *out = nullptr;
    if (!d_ptr || bytes == 0) return set_error(GSR_E_ARG, "gsr_display_wrap_device: null or empty buffer");
    auto* t = new gsr_display_target();
    t->dev = d_ptr;
    t->bytes = bytes;
    *out = t;
    return GSR_OK;
}

extern "C" int gsr_display_free(gsr_display_target* t) {
    if (!t) return GSR_OK;
    int rc = GSR_OK;
    if (t->res && hipGraphicsUnregisterResource(t->res) != hipSuccess)
        rc = set_error(GSR_E_DISPLAY, "hipGraphicsUnregisterResource failed for GL buffer %u", t->gl_buffer);
    delete t;
    return rc;
}

extern "C" int gsr_render_display(gsr_context* ctx, gsr_display_target* t, const void* d_scene, int layout,
                                  int64_t n, const gsr_camera* cam, int W, int H, int num_tile_x, int num_tile_y,
                                  int width_stride, int height_stride, float k, void* stream) {
    if (!ctx || !t) return set_error(GSR_E_ARG, "gsr_render_display: null context or target");
    if (W <= 0 || H <= 0) return set_error(GSR_E_ARG, "gsr_render_display: image size %dx%d", W, H);
    const hipStream_t s = static_cast<hipStream_t>(stream);
    float* img = nullptr;
    size_t bytes = 0;
    if (int rc = map_target(t, s, &img, &bytes)) return rc;
    const size_t need = 3 * sizeof(float) * (size_t)W * (size_t)H;
    int rc;
    if (bytes < need) {
        rc = set_error(GSR_E_ARG, "display target holds %zu bytes, a %dx%d image needs %zu", bytes, W, H, need);
    } else {
        rc = gsr_render(ctx, d_scene, layout, n, cam, W, H, num_tile_x, num_tile_y, width_stride, height_stride, k,
                        img, stream);
    }
    const int rc_unmap = unmap_target(t, s);
    return rc != GSR_OK ? rc : rc_unmap;
}

// ------------------------------------------------------------------ drop-in

namespace {
gsr_display_target* g_gl_target = nullptr;   // cached registration of the viewer's SSBO
unsigned int g_gl_buffer = 0;
int g_gl_w = 0, g_gl_h = 0;
}  // namespace

extern "C" void preprocessCUDAGaussiansGL(gsr_gaussian* d_gaussians, unsigned int gl_buffer, int num_gaussians,
                                          gsr_camera cam, int num_tile_y, int num_tile_x, int width_stride,
                                          int height_stride, int tile_W, int tile_H, float k) {
    std::lock_guard<std::mutex> lk(gsr::dropin_mutex());
    auto fail = [](const char* what) {
        std::fprintf(stderr, "preprocessCUDAGaussiansGL: %s: %s\n", what, gsr::last_error());
    };
    if (tile_W <= 0 || tile_H <= 0) {
        set_error(GSR_E_ARG, "bad image size %dx%d", tile_W, tile_H);
        fail("argument");
        return;
    }
    // a resize re-specifies the SSBO's storage (canvas.cpp:210-212): re-register
    if (!g_gl_target || g_gl_buffer != gl_buffer || g_gl_w != tile_W || g_gl_h != tile_H) {
        (void)gsr_display_free(g_gl_target);
        g_gl_target = nullptr;
        if (gsr_display_register_gl(gl_buffer, &g_gl_target) != GSR_OK) {
            fail("register");
            return;
        }
        g_gl_buffer = gl_buffer;
        g_gl_w = tile_W;
        g_gl_h = tile_H;
    }
    float* img = nullptr;
    size_t bytes = 0;
    if (map_target(g_gl_target, nullptr, &img, &bytes) != GSR_OK) {
        fail("map");
        return;
    }
    const char* what = "render";
    if (bytes < 3 * sizeof(float) * (size_t)tile_W * (size_t)tile_H) {
        set_error(GSR_E_ARG, "GL buffer %u holds %zu bytes, smaller than a %dx%d image", gl_buffer, bytes, tile_W,
                  tile_H);
        what = "size";
    } else if (gsr::dropin_render_device(d_gaussians, num_gaussians, cam, num_tile_y, num_tile_x, width_stride,
                                         height_stride, tile_W, tile_H, k, img, &what) == GSR_OK) {
        what = nullptr;
    }
    if (unmap_target(g_gl_target, nullptr) != GSR_OK && !what) what = "unmap";
    if (what) fail(what);
}
