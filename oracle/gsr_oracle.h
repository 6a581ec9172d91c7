/*
 * gsr_oracle.h — CPU ORACLE (TEST INFRASTRUCTURE ONLY).
 *
 * A plain-C restatement of the reference renderer's semantics
 * (/root/reference/src/core/cuda/render.cu, math.cu, misc.cu and
 * utils/gaussians.cpp), used ONLY by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker / CPU baseline.  The product
 * (libgsr.so) never links, loads or calls anything in this directory.
 *
 * Parity pinning: the PLY loader, the camera matrices and the covariance
 * matrix chain are pinned against the reference's own host C++ compiled from
 * /root/reference by oracle/Makefile into oracle/_ref/ (tests/golden/ holds
 * the fixtures it produced, tests/golden/make_golden.py the script).  The
 * CUDA-only parts (cull, SH colour, 2D extent, binning, sort, blend) follow
 * render.cu as text; see DESIGN.md "Oracle".
 */
#ifndef GSR_ORACLE_H
#define GSR_ORACLE_H

#include <stdint.h>
#include "../include/gsr_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Per-Gaussian result of the cull + prepare stages (render.cu:472-786). */
typedef struct orc_splat {
    int32_t status;        /* 0 culled (render.cu:543,553-556), 1 dropped by prepare
                              (det / off-screen reject, render.cu:690,737), 2 visible */
    float color[3];        /* render.cu:502-534 */
    float ndc[3];          /* render.cu:545-552 */
    float view[3];         /* X, Y, Z (render.cu:539-542) */
    float inv_covar[4];    /* render.cu:694-701 */
    int32_t aabb[4];       /* xmin, ymin, xmax, ymax pixels (render.cu:748-759) */
    int32_t px_x, px_y;    /* render.cu:753-754 */
    uint32_t depth_key;    /* u32(-Z * 1e6f) (render.cu:850), saturating */
    float opacity;
} orc_splat;

/* misc.cu:13-134 restated: returns 0 ok, <0 error.  soa may be NULL to get n. */
int orc_ply_read(const char* path, float* soa, int64_t capacity, int64_t* n_out);
/* narrays 38 (3D) or 49 (4D arrays: trbf_center, exp(trbf_scale), motion_0..8). */
int orc_ply_read_ex(const char* path, float* soa, int narrays, int64_t capacity, int64_t* n_out);
/* SH-3 ("Inria-correct") mode for orc_preprocess / orc_render: soa then has
 * GSR_SCENE_SH3_NARRAYS arrays (process-wide switch; tests reset it). */
void orc_set_sh3(int on);
/* Blend contraction variant (gsr_oracle.c blend_step_var): md2 0..4, rgb 0..1, exp 0..2;
 * (1, 1, 0) = the shipped choice the kernels share. */
void orc_set_blend_variant(int md2, int rgb, int expm);
/* Config 5: the 38 arrays of a 4D scene at time t, no temporal cull. */
void orc_temporal(const float* soa49, int64_t n, float t, float* out38);

/* render.cu:620-621 fx, fy. */
void orc_intrinsics(const gsr_camera* cam, float* fx, float* fy);

/* Cull + prepare for every Gaussian of a SoA scene (38 arrays of n floats). */
int orc_preprocess(const float* soa, int64_t n, const gsr_camera* cam, int W, int H, float k,
                   orc_splat* out);

/* Full frame, splat-major: visible splats in (depth_key, index) order, each
 * composited over the pixels of its inclusive AABB (render.cu:323-341).
 * out: 3*W*H floats planar, row 0 = bottom.  threads <= 0: use all cores. */
int orc_render(const float* soa, int64_t n, const gsr_camera* cam, int W, int H,
               int num_tile_x, int num_tile_y, int width_stride, int height_stride,
               float k, float* out, int threads);

/* Same frame, reference-literal: the reference's own tiling (ws x hs tiles),
 * (tile << 32 | depth) keys sorted stably with index tie-break, per-tile
 * per-pixel loops (render.cu:266-367, 811-857).  Used to prove tile
 * invariance of the splat-major path.  Single-threaded. */
int orc_render_tiled(const float* soa, int64_t n, const gsr_camera* cam, int W, int H,
                     int num_tile_x, int num_tile_y, int width_stride, int height_stride,
                     float k, float* out);

/* Sub-steps exposed so tests can pin them against the reference's own host
 * math (math.cpp, compiled into oracle/_ref): tmp = V*[x,y,z,1], ndc = P*tmp
 * / w (render.cu:535-552) and the 2D covariance chain J*Rc*R*S*S*R^T*Rc^T*J^T
 * before the pixel scaling (render.cu:655-682). */
void orc_project(const float V[16], const float P[16], const float xyz[3], float tmp[4], float ndc[4]);
void orc_covariance_chain(const float quat[4], const float scale[3], const float XYZ[3], float fx,
                          float fy, const float r_cam[9], const float r_cam_T[9], float sigma2d[4]);

/* Deterministic math exported for the detmath tests (gsr_detmath.h). */
float orc_expf(float x);
float orc_blend_expf(float x);
void orc_blend_exp_sweep(float x_lo, float x_hi, int64_t* viol, double* max_ulp);
float orc_sinf(float x);
float orc_cosf(float x);
float orc_atan2f(float y, float x);

#ifdef __cplusplus
}
#endif

#endif
