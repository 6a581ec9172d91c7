// viewer_link.cpp — TEST INFRASTRUCTURE (link-level drop-in proof).
//
// A translation unit written the way the reference viewer is: it includes the
// reference's OWN headers, unmodified, from /root/reference (render.cuh:27-37
// declares preprocessCUDAGaussians; camera.hpp:2-41 and gaussians.hpp:16-58 the
// types), declares the loader exactly as misc.cuh:4 does (that header also pulls in
// cuda_runtime.h, absent here), and links against libgsr.so — no gsr.h, no casts.
// Compiled by oracle/Makefile into oracle/_ref/viewer_link (only when the
// reference tree exists; the binary travels, the reference sources never do).
//
//   viewer_link --layout                      static layout checks passed; exit 0
//   viewer_link SCENE.ply W H OUT.f32 [AZIMUTH_DEG]
//       Canvas::loadGaussians + Canvas::render in miniature (canvas.cpp:11, 285-296,
//       337-342): load, Camera at (0,0,4) fovY 50 aspect W/H, orbit, 50x50
//       TilingInformation, one synchronous preprocessCUDAGaussians into a host image.
#include "render.cuh"

#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

Gaussian* loadGaussianCudaFromPly(const std::string& filename, int* out_numGaussians);  // misc.cuh:4

#include "gsr_types.h"   // our ABI types: the layouts must coincide field by field

#define SAME_FIELD(R, G, f) static_assert(offsetof(R, f) == offsetof(G, f), #R "::" #f)
SAME_FIELD(Camera, gsr_camera, position);
SAME_FIELD(Camera, gsr_camera, lookAt);
SAME_FIELD(Camera, gsr_camera, w_up);
SAME_FIELD(Camera, gsr_camera, fovY);
SAME_FIELD(Camera, gsr_camera, aspectRatio);
SAME_FIELD(Camera, gsr_camera, nearClip);
SAME_FIELD(Camera, gsr_camera, farClip);
SAME_FIELD(Camera, gsr_camera, forward_vec);
SAME_FIELD(Camera, gsr_camera, right_vec);
SAME_FIELD(Camera, gsr_camera, up_vec);
SAME_FIELD(Camera, gsr_camera, P_matrix);
SAME_FIELD(Camera, gsr_camera, V_matrix);
SAME_FIELD(Camera, gsr_camera, M_matrix);
SAME_FIELD(Camera, gsr_camera, f_axis);
SAME_FIELD(Camera, gsr_camera, r_axis);
SAME_FIELD(Camera, gsr_camera, u_axis);
SAME_FIELD(Camera, gsr_camera, r_cam);
SAME_FIELD(Camera, gsr_camera, r_cam_T);
SAME_FIELD(Camera, gsr_camera, plane_normals);
static_assert(sizeof(Camera) == sizeof(gsr_camera) && sizeof(Camera) == 484, "Camera size");
static_assert(alignof(Camera) == alignof(gsr_camera), "Camera alignment (by-value passing)");

SAME_FIELD(Gaussian, gsr_gaussian, x);
SAME_FIELD(Gaussian, gsr_gaussian, y);
SAME_FIELD(Gaussian, gsr_gaussian, z);
SAME_FIELD(Gaussian, gsr_gaussian, normals);
SAME_FIELD(Gaussian, gsr_gaussian, sh);
SAME_FIELD(Gaussian, gsr_gaussian, color);
SAME_FIELD(Gaussian, gsr_gaussian, opacity);
SAME_FIELD(Gaussian, gsr_gaussian, scale);
SAME_FIELD(Gaussian, gsr_gaussian, rot);
SAME_FIELD(Gaussian, gsr_gaussian, aabb);
SAME_FIELD(Gaussian, gsr_gaussian, px_x);
SAME_FIELD(Gaussian, gsr_gaussian, px_y);
SAME_FIELD(Gaussian, gsr_gaussian, radix_id);
SAME_FIELD(Gaussian, gsr_gaussian, X);
SAME_FIELD(Gaussian, gsr_gaussian, Y);
SAME_FIELD(Gaussian, gsr_gaussian, Z);
SAME_FIELD(Gaussian, gsr_gaussian, inv_covar);
static_assert(sizeof(Gaussian) == sizeof(gsr_gaussian) && sizeof(Gaussian) == 240, "Gaussian size");

SAME_FIELD(lightWeightGaussian, gsr_lwg, radix_id);
SAME_FIELD(lightWeightGaussian, gsr_lwg, gaussian_id);
static_assert(sizeof(lightWeightGaussian) == sizeof(gsr_lwg), "lightWeightGaussian size");

// the viewer frees the loader's block with cudaFree; the HIP twin here
extern "C" int hipFree(void*);

int main(int argc, char** argv) {
    if (argc == 2 && std::strcmp(argv[1], "--layout") == 0) {
        std::printf("layout ok: Camera %zu B, Gaussian %zu B\n", sizeof(Camera), sizeof(Gaussian));
        return 0;
    }
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s SCENE.ply W H OUT.f32 [AZIMUTH_DEG] | --layout\n", argv[0]);
        return 2;
    }
    const int W = std::atoi(argv[2]), H = std::atoi(argv[3]);
    const float azimuth = argc > 5 ? (float)std::atof(argv[5]) : 0.0f;
    int n = 0;
    Gaussian* d = loadGaussianCudaFromPly(std::string(argv[1]), &n);
    if (!d) {
        std::fprintf(stderr, "loadGaussianCudaFromPly failed\n");
        return 1;
    }
    Camera cam;
    const float pos[3] = {0.0f, 0.0f, 4.0f};
    cam.setPosition(pos);
    cam.setFovY(50.0f);
    cam.setAspectRatio((float)W / (float)H);
    cam.setClippingPlanes(0.1f, 100.0f);
    cam.updateCameraMatrices();
    cam.updateFrustumPlanes();
    if (azimuth != 0.0f) cam.orbit(azimuth, 0.0f);
    TilingInformation tiles(50, 50, H, W);   // Canvas ctor: TilingInformation(tile_y, tile_x, H, W)
    std::vector<float> img((size_t)3 * W * H, 0.0f);
    preprocessCUDAGaussians(d, img.data(), n, cam, tiles.num_tile_y, tiles.num_tile_x, tiles.width_stride,
                            tiles.height_stride, W, H, 3.0f);
    hipFree(d);
    FILE* f = std::fopen(argv[4], "wb");
    if (!f || std::fwrite(img.data(), sizeof(float), img.size(), f) != img.size()) return 1;
    std::fclose(f);
    std::printf("rendered %d Gaussians at %dx%d\n", n, W, H);
    return 0;
}
