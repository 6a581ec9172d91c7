/* gsr_gl.h — display interop: the render writes the
 * viewer's display buffer directly instead of going device -> host -> GL.
 *
 * The reference viewer renders into a host vector (canvas.cpp:337-342:
 * preprocessCUDAGaussians(..., d_out_pixels.data(), ...)) and then uploads it
 * into its colour SSBO every frame (canvas.cpp:350-351: glBufferSubData of
 * W*H*3 floats).  That SSBO is exactly our image: planar float32 [3][H][W]
 * (`float data[]`, std430, binding 0; read as data[c*W*H + y*W + x] by the
 * fragment shader, canvas.hpp:83-106; allocated canvas.cpp:118-121, 210-212).
 * Registering it with HIP lets gsr_render write it in place: no 24.9 MB D2H and
 * H2D per 1080p frame.
 *
 * GL is looked up at run time (dlopen of libGL.so.1 / libEGL.so.1), so libgsr
 * has no link dependency on GL; every GL entry point needs the viewer's GL
 * context current on the calling thread and returns GSR_E_DISPLAY otherwise.
 * A display target can also wrap plain device memory (a Vulkan / external
 * memory buffer already imported with hipExternalMemoryGetMappedBuffer, or any
 * device buffer), which takes the same render path without GL.
 */
#ifndef GSR_GL_H
#define GSR_GL_H

#include <stddef.h>
#include <stdint.h>

#include "gsr.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gsr_display_target gsr_display_target;

/* Register a GL buffer object (the viewer's colour SSBO, canvas.cpp:118) for
 * writing by the render (hipGraphicsGLRegisterBuffer, write-discard).  Call
 * again after the buffer's storage is re-specified (window resize,
 * canvas.cpp:210-212): a registration refers to the storage it saw. */
int gsr_display_register_gl(unsigned int gl_buffer, gsr_display_target** out);

/* Wrap device memory of `bytes` bytes as a display target (no GL). */
int gsr_display_wrap_device(void* d_ptr, size_t bytes, gsr_display_target** out);

/* Unregister / release a target (NULL is a no-op). */
int gsr_display_free(gsr_display_target* target);

/* 1 if a GL context (GLX or EGL) is current on this thread, else 0. */
int gsr_display_gl_current(void);

/* gsr_render into the target: map it on `stream`, check it holds 3*W*H floats,
 * render, unmap on `stream` (GL's next use of the buffer is ordered after the
 * frame's kernels).  Same arguments and return codes as gsr_render. */
int gsr_render_display(gsr_context* ctx, gsr_display_target* target, const void* d_scene, int layout,
                       int64_t n, const gsr_camera* cam, int W, int H, int num_tile_x, int num_tile_y,
                       int width_stride, int height_stride, float k, void* stream);

/* Canvas::render (canvas.cpp:337-342) without the host round trip: the
 * preprocessCUDAGaussians argument list with the colour SSBO's GL name in place
 * of the host `out_pixels` pointer (render.cu:871).  Synchronous like the
 * reference call; the registration is cached per (buffer, W, H).  The viewer
 * then draws without its glBufferSubData (canvas.cpp:351).  Errors go to stderr
 * and gsr_last_error(), as for preprocessCUDAGaussians. */
void preprocessCUDAGaussiansGL(gsr_gaussian* d_gaussians, unsigned int gl_buffer, int num_gaussians,
                               gsr_camera cam, int num_tile_y, int num_tile_x, int width_stride,
                               int height_stride, int tile_W, int tile_H, float k);

#ifdef __cplusplus
}
#endif

#endif /* GSR_GL_H */
