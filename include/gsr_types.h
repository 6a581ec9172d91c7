/*
 * gsr_types.h — ABI types shared with the reference viewer.
 *
 * Every struct here is layout-identical to the reference type it replaces so
 * that the existing C++ viewer (src/core/render/canvas.cpp) can hand its own
 * objects across the boundary unchanged:
 *
 *   gsr_camera    == Camera              (src/core/scene/camera.hpp:2-41,  484 B, by value)
 *   gsr_gaussian  == Gaussian            (src/core/utils/gaussians.hpp:16-30, 240 B)
 *   gsr_lwg       == lightWeightGaussian (src/core/utils/gaussians.hpp:32-35, 16 B)
 *
 * The static asserts below pin the offsets measured from the reference
 * headers with g++.
 */
#ifndef GSR_TYPES_H
#define GSR_TYPES_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Camera (scene/camera.hpp:2-41).  The renderer reads position, fovY,
 * aspectRatio, nearClip, V_matrix, P_matrix, r_cam and r_cam_T
 * (render.cu:484-490, 614-618); the caller must have run
 * updateCameraMatrices() (camera.cpp:36-57) or gsr_camera_update(). */
typedef struct gsr_camera {
    float position[3];
    float lookAt[3];
    float w_up[3];
    float fovY;          /* degrees */
    float aspectRatio;
    float nearClip;
    float farClip;
    float forward_vec[3];
    float right_vec[3];
    float up_vec[3];
    float P_matrix[16];  /* row-major */
    float V_matrix[16];  /* row-major */
    float M_matrix[16];
    float f_axis[3];
    float r_axis[3];
    float u_axis[3];
    float r_cam[9];
    float r_cam_T[9];
    float plane_normals[24];
} gsr_camera;

/* Gaussian (utils/gaussians.hpp:16-30): the reference's AoS record.  It is
 * accepted as INPUT by preprocessCUDAGaussians when the caller hands over a
 * plain Gaussian[] array (e.g. produced by the reference's own loader).  Our
 * loader returns an opaque SoA scene block instead (gsr_scene_header). */
typedef struct gsr_gaussian {
    float x, y, z;
    float normals[3];
    float sh[27];
    float color[3];
    float opacity;
    float scale[3];
    float rot[4];          /* w, x, y, z (render.cu:153-164 normalises) */
    int32_t aabb[4];
    int32_t px_x, px_y;
    uint64_t radix_id;
    float X, Y, Z;
    float inv_covar[4];
} gsr_gaussian;

/* lightWeightGaussian (utils/gaussians.hpp:32-35): sort pair of the
 * reference's standalone sort entry oneSweep3DGaussianSort (render.cu:194). */
typedef struct gsr_lwg {
    uint64_t radix_id;     /* (tile << 32) | u32(-Z * 1e6) */
    uint32_t gaussian_id;
} gsr_lwg;

/*
 * Device scene block returned by loadGaussianCudaFromPly / gsr_scene_upload.
 * ONE hipMalloc: this 256-byte header followed by GSR_SCENE_NARRAYS float
 * arrays of `stride` elements each (structure of arrays, 256-B aligned), so
 * that the viewer's single cudaFree/hipFree of the returned pointer
 * (canvas.cpp:14-24, 286-291) releases everything.
 *
 * Array order (index into the array table):
 *   0..2   x, y, z                      (raw PLY positions)
 *   3      opacity  = 1/(1+expf(-v))     (gaussians.cpp:12-15, 25)
 *   4..6   scale_i  = (float)exp((double)v) (gaussians.cpp:26)
 *   7..10  rot_0..3 (w, x, y, z), raw    (gaussians.cpp:27)
 *   11..37 sh[0..26]: f_dc_0..2 then f_rest_0..23 (gaussians.cpp:23-24,
 *          misc.cu:74-77; f_rest_24..44 are dropped as in the reference)
 * 4D scene blocks (GSR_SCENE4D_NARRAYS, config 5 — Spacetime-Gaussian style,
 * DESIGN.md) append:
 *   38     trbf_center (temporal centre, raw)
 *   39     trbf_scale = (float)exp((double)v) (temporal scale)
 *   40..48 motion_0..8: linear xyz, quadratic xyz, cubic xyz (raw)
 * SH-3 blocks (GSR_SCENE_SH3_NARRAYS, opt-in "Inria-correct" mode)
 * replace 11..37 with 11..58 = sh[3k + c] for the 16 coefficients k of
 * degree <= 3: k = 0 from f_dc_c, k >= 1 from f_rest_{15c + k - 1} (the
 * channel-major layout of 3DGS training output).
 */
#define GSR_SCENE_MAGIC0 0x7fc0a5e1u   /* NaN bit patterns: never a sane AoS x,y,z */
#define GSR_SCENE_MAGIC1 0x7fc05352u
#define GSR_SCENE_MAGIC2 0x7fc03347u
#define GSR_SCENE_MAGIC3 0x7fc00001u
#define GSR_SCENE_NARRAYS 38
#define GSR_SCENE4D_NARRAYS 49
#define GSR_SCENE_SH3_NARRAYS 59      /* 3D block with full degree-3 SH (opt-in, GSR_PLY_SH3) */
#define GSR_SCENE_HEADER_BYTES 256

typedef struct gsr_scene_header {
    uint32_t magic[4];
    uint64_t count;        /* number of Gaussians */
    uint64_t stride;       /* elements per array (count rounded up to 64) */
    uint64_t narrays;      /* GSR_SCENE_NARRAYS or GSR_SCENE4D_NARRAYS */
    uint64_t reserved[27];
} gsr_scene_header;

/* Index of each attribute array inside a scene block. */
enum {
    GSR_A_X = 0, GSR_A_Y = 1, GSR_A_Z = 2,
    GSR_A_OPACITY = 3,
    GSR_A_SCALE0 = 4,
    GSR_A_ROT0 = 7,
    GSR_A_SH0 = 11,
    GSR_A_TCENTER = 38,
    GSR_A_TSCALE = 39,
    GSR_A_MOTION0 = 40
};

#ifdef __cplusplus
}  /* extern "C" */
static_assert(sizeof(gsr_camera) == 484, "Camera must stay 484 bytes (camera.hpp)");
static_assert(offsetof(gsr_camera, P_matrix) == 88, "Camera.P_matrix offset");
static_assert(offsetof(gsr_camera, V_matrix) == 152, "Camera.V_matrix offset");
static_assert(offsetof(gsr_camera, r_cam) == 316, "Camera.r_cam offset");
static_assert(sizeof(gsr_gaussian) == 240, "Gaussian must stay 240 bytes (gaussians.hpp)");
static_assert(offsetof(gsr_gaussian, sh) == 24, "Gaussian.sh offset");
static_assert(offsetof(gsr_gaussian, color) == 132, "Gaussian.color offset");
static_assert(offsetof(gsr_gaussian, opacity) == 144, "Gaussian.opacity offset");
static_assert(offsetof(gsr_gaussian, scale) == 148, "Gaussian.scale offset");
static_assert(offsetof(gsr_gaussian, rot) == 160, "Gaussian.rot offset");
static_assert(offsetof(gsr_gaussian, aabb) == 176, "Gaussian.aabb offset");
static_assert(offsetof(gsr_gaussian, radix_id) == 200, "Gaussian.radix_id offset");
static_assert(offsetof(gsr_gaussian, X) == 208, "Gaussian.X offset");
static_assert(offsetof(gsr_gaussian, inv_covar) == 220, "Gaussian.inv_covar offset");
static_assert(sizeof(gsr_lwg) == 16, "lightWeightGaussian must stay 16 bytes");
static_assert(sizeof(gsr_scene_header) == GSR_SCENE_HEADER_BYTES, "scene header size");
#endif

#endif /* GSR_TYPES_H */
