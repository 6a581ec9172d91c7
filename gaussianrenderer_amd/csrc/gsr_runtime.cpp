// gsr_runtime.cpp — host runtime behind the C ABI of include/gsr.h.
//
// Owns the persistent per-context workspace (sized by high-water mark, never
// allocated per frame — the reference does ~10 cudaMalloc/cudaFree per frame,
// render.cu:891-902, 1144-1156), orchestrates the stage kernels on one HIP
// stream, and implements the drop-in entry points of the reference viewer
// (preprocessCUDAGaussians, loadGaussianCudaFromPly) plus the host helpers
// that mirror camera.cpp / gaussians.cpp.
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <random>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include <hip/hip_runtime.h>

#include "gsr.h"
#include "gsr_internal.h"
#include "gsr_detmath.h"

using gsr::Frame;
using gsr::Stats;

// ------------------------------------------------------------------ errors

static thread_local std::string g_err;

namespace gsr {
int set_error(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}
}  // namespace gsr

#define set_err gsr::set_error

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return set_err(GSR_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                           __FILE__, __LINE__);                                              \
    } while (0)

extern "C" const char* gsr_last_error(void) { return g_err.c_str(); }
extern "C" const char* gsr_version(void) { return "gsr 0.1 (gfx950)"; }

extern "C" int gsr_device_available(void) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return 0;
    return c > 0 ? 1 : 0;
}

// ------------------------------------------------------------------ camera (camera.cpp, math.cpp)

namespace {

void m_normalize(float v[3]) {   // math.cpp:7-20
    float nrm = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (nrm > 1e-8f) {
        v[0] /= nrm;
        v[1] /= nrm;
        v[2] /= nrm;
    } else {
        v[0] = 0.0f;
        v[1] = 0.0f;
        v[2] = 0.0f;
    }
}
float m_norm(const float v[3]) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
void m_cross(const float a[3], const float b[3], float o[3]) {   // math.cpp:45-49
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
void m_sub(const float a[3], const float b[3], float o[3]) {
    o[0] = a[0] - b[0];
    o[1] = a[1] - b[1];
    o[2] = a[2] - b[2];
}
void m_view(const float x[3], const float y[3], const float z[3], const float e[3], float o[16]) {  // math.cpp:65-90
    o[0] = x[0]; o[1] = x[1]; o[2] = x[2]; o[3] = -(x[0] * e[0] + x[1] * e[1] + x[2] * e[2]);
    o[4] = y[0]; o[5] = y[1]; o[6] = y[2]; o[7] = -(y[0] * e[0] + y[1] * e[1] + y[2] * e[2]);
    o[8] = z[0]; o[9] = z[1]; o[10] = z[2]; o[11] = -(z[0] * e[0] + z[1] * e[1] + z[2] * e[2]);
    o[12] = 0.0f; o[13] = 0.0f; o[14] = 0.0f; o[15] = 1.0f;
}
void m_persp(float fovY, float aspect, float nr, float fr, float o[16]) {   // math.cpp:91-97
    float f = 1.0f / std::tan(fovY * 0.5f * (M_PI / 180.0f));
    o[0] = f / aspect; o[1] = 0.0f; o[2] = 0.0f; o[3] = 0.0f;
    o[4] = 0.0f; o[5] = f; o[6] = 0.0f; o[7] = 0.0f;
    o[8] = 0.0f; o[9] = 0.0f; o[10] = (fr + nr) / (nr - fr); o[11] = (2 * fr * nr) / (nr - fr);
    o[12] = 0.0f; o[13] = 0.0f; o[14] = -1.0f; o[15] = 0.0f;
}
void m_mm4(const float A[16], const float B[16], float o[16]) {   // math.cpp:99-108
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            o[i * 4 + j] = 0.0f;
            for (int k = 0; k < 4; ++k) o[i * 4 + j] += A[i * 4 + k] * B[k * 4 + j];
        }
}

}  // namespace

extern "C" void gsr_camera_default(gsr_camera* c) {   // camera.cpp:8-13
    std::memset(c, 0, sizeof *c);
    c->fovY = 45.0f;
    c->aspectRatio = 1.0f;
    c->nearClip = 0.1f;
    c->farClip = 100.0f;
    c->position[2] = 5.0f;
    c->up_vec[1] = 1.0f;
    c->w_up[1] = 1.0f;
}

extern "C" void gsr_camera_update(gsr_camera* c) {   // camera.cpp:36-57
    m_sub(c->lookAt, c->position, c->f_axis);
    m_normalize(c->f_axis);
    m_cross(c->f_axis, c->w_up, c->r_axis);
    m_normalize(c->r_axis);
    m_cross(c->r_axis, c->f_axis, c->u_axis);
    for (int i = 0; i < 3; i++) c->f_axis[i] = -c->f_axis[i];
    for (int i = 0; i < 3; i++) {
        c->r_cam[i] = c->r_axis[i];
        c->r_cam[3 + i] = c->u_axis[i];
        c->r_cam[6 + i] = c->f_axis[i];
    }
    const float* A = c->r_cam;
    float* T = c->r_cam_T;
    T[0] = A[0]; T[1] = A[3]; T[2] = A[6];
    T[3] = A[1]; T[4] = A[4]; T[5] = A[7];
    T[6] = A[2]; T[7] = A[5]; T[8] = A[8];
    m_view(c->r_axis, c->u_axis, c->f_axis, c->position, c->V_matrix);
    m_persp(c->fovY, c->aspectRatio, c->nearClip, c->farClip, c->P_matrix);
    m_mm4(c->P_matrix, c->V_matrix, c->M_matrix);
}

extern "C" void gsr_camera_update_frustum(gsr_camera* c) {   // camera.cpp:59-121
    float* pl = c->plane_normals;
    const float* f = c->f_axis;
    const float* p = c->position;
    for (int i = 0; i < 3; i++) pl[i] = f[i];
    pl[3] = (f[0] * p[0] + f[1] * p[1] + f[2] * p[2] - c->nearClip);
    for (int i = 0; i < 3; i++) pl[4 + i] = -f[i];
    pl[7] = -(f[0] * p[0] + f[1] * p[1] + f[2] * p[2] - c->farClip);
    float t_y = std::tan(c->fovY * 0.5f * (M_PI / 180.0f));
    float t_x = t_y * c->aspectRatio;
    const float sgn[4] = {-1.0f, 1.0f, -1.0f, 1.0f};
    for (int q = 0; q < 4; q++) {
        const float* ax = (q < 2) ? c->r_axis : c->u_axis;
        const float tt = (q < 2) ? t_x : t_y;
        float nrm[3];
        for (int i = 0; i < 3; i++) nrm[i] = (sgn[q] < 0) ? (f[i] * tt - ax[i]) : (f[i] * tt + ax[i]);
        m_normalize(nrm);
        for (int i = 0; i < 3; i++) pl[8 + 4 * q + i] = nrm[i];
        pl[11 + 4 * q] = 0.0f;
    }
}

extern "C" void gsr_camera_zoom(gsr_camera* c, float delta) {   // camera.cpp:123-128
    for (int i = 0; i < 3; i++) c->position[i] += c->f_axis[i] * delta;
    gsr_camera_update(c);
}

extern "C" void gsr_camera_orbit(gsr_camera* c, float azimuth, float elevation) {   // camera.cpp:130-158
    azimuth = azimuth * M_PI / 180.0f;
    elevation = elevation * M_PI / 180.0f;
    float rv[3];
    m_sub(c->position, c->lookAt, rv);
    float radius = m_norm(rv);
    float theta = std::atan2(rv[2], rv[0]);
    float phi = std::acos(rv[1] / radius);
    theta += azimuth;
    phi += elevation;
    const float epsilon = 0.01f;
    if (phi < epsilon) phi = epsilon;
    if (phi > M_PI - epsilon) phi = M_PI - epsilon;
    rv[0] = radius * std::sin(phi) * std::cos(theta);
    rv[1] = radius * std::cos(phi);
    rv[2] = radius * std::sin(phi) * std::sin(theta);
    for (int i = 0; i < 3; i++) c->position[i] = c->lookAt[i] + rv[i];
    gsr_camera_update(c);
}

extern "C" void gsr_camera_intrinsics(const gsr_camera* cam, float* fx, float* fy) {
    // render.cu:620-621: fy = 1/tanf(fovY*0.5f*(CUDART_PI_F/180.0f)); tanf taken
    // correctly rounded (float(tan(double))) so the oracle computes the same.
    const float PI_F = 3.141592654f;
    const float arg = cam->fovY * 0.5f * (PI_F / 180.0f);
    const float t = (float)std::tan((double)arg);
    *fy = 1.0f / t;
    *fx = *fy / cam->aspectRatio;
}

// ------------------------------------------------------------------ device scene blocks

static int64_t scene_stride(int64_t n) { return (n + 63) / 64 * 64; }

extern "C" void* gsr_scene_upload_ex(const float* host_soa, int narrays, int64_t n) {
    if (n < 0 || n > INT32_MAX || (n > 0 && !host_soa) ||
        (narrays != GSR_SCENE_NARRAYS && narrays != GSR_SCENE4D_NARRAYS && narrays != GSR_SCENE_SH3_NARRAYS)) {
        set_err(GSR_E_ARG, "gsr_scene_upload: bad argument");
        return nullptr;
    }
    const int64_t stride = scene_stride(n);
    const size_t bytes = GSR_SCENE_HEADER_BYTES + sizeof(float) * (size_t)narrays * (size_t)stride;
    void* d = nullptr;
    hipError_t e = hipMalloc(&d, bytes);
    if (e != hipSuccess) {
        set_err(GSR_E_HIP, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
        return nullptr;
    }
    gsr_scene_header h{};
    h.magic[0] = GSR_SCENE_MAGIC0;
    h.magic[1] = GSR_SCENE_MAGIC1;
    h.magic[2] = GSR_SCENE_MAGIC2;
    h.magic[3] = GSR_SCENE_MAGIC3;
    h.count = (uint64_t)n;
    h.stride = (uint64_t)stride;
    h.narrays = (uint64_t)narrays;
    e = hipMemcpy(d, &h, sizeof h, hipMemcpyHostToDevice);
    float* arr = reinterpret_cast<float*>(static_cast<char*>(d) + GSR_SCENE_HEADER_BYTES);
    if (e == hipSuccess && n > 0)
        e = hipMemcpy2D(arr, sizeof(float) * (size_t)stride, host_soa, sizeof(float) * (size_t)n,
                        sizeof(float) * (size_t)n, (size_t)narrays, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        set_err(GSR_E_HIP, "scene upload failed: %s", hipGetErrorString(e));
        (void)hipFree(d);
        return nullptr;
    }
    return d;
}

extern "C" int64_t gsr_scene_bytes(int narrays, int64_t n) {
    if (n < 0 || n > INT32_MAX ||
        (narrays != GSR_SCENE_NARRAYS && narrays != GSR_SCENE4D_NARRAYS && narrays != GSR_SCENE_SH3_NARRAYS))
        return set_err(GSR_E_ARG, "gsr_scene_bytes: bad argument");
    return (int64_t)GSR_SCENE_HEADER_BYTES + (int64_t)sizeof(float) * narrays * scene_stride(n);
}

extern "C" int gsr_scene_copy(void* d_dst, const void* d_scene, int narrays, int64_t n, void* stream) {
    const int64_t bytes = gsr_scene_bytes(narrays, n);
    if (bytes < 0) return (int)bytes;
    if (!d_dst || !d_scene) return set_err(GSR_E_ARG, "gsr_scene_copy: null pointer");
    gsr_scene_header h{};
    HIP_TRY(hipMemcpy(&h, d_scene, sizeof h, hipMemcpyDeviceToHost));
    if (h.count != (uint64_t)n || h.narrays != (uint64_t)narrays)
        return set_err(GSR_E_ARG, "gsr_scene_copy: block holds %llu Gaussians x %llu arrays, not %lld x %d",
                       (unsigned long long)h.count, (unsigned long long)h.narrays, (long long)n, narrays);
    HIP_TRY(hipMemcpyAsync(d_dst, d_scene, (size_t)bytes, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)));
    return GSR_OK;
}

extern "C" void* gsr_scene_upload(const float* host_soa, int64_t n) {
    return gsr_scene_upload_ex(host_soa, GSR_SCENE_NARRAYS, n);
}

extern "C" void gsr_scene_free(void* d) {
    if (d) (void)hipFree(d);
}

extern "C" int gsr_scene_download(const void* d, float* host_soa, int64_t n) {
    if (!d || !host_soa || n < 0) return set_err(GSR_E_ARG, "gsr_scene_download: bad argument");
    gsr_scene_header h{};
    HIP_TRY(hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost));
    const int narrays = (h.narrays == GSR_SCENE4D_NARRAYS || h.narrays == GSR_SCENE_SH3_NARRAYS)
                            ? (int)h.narrays : GSR_SCENE_NARRAYS;
    const int64_t stride = scene_stride(n);
    const float* arr = reinterpret_cast<const float*>(static_cast<const char*>(d) + GSR_SCENE_HEADER_BYTES);
    if (n == 0) return GSR_OK;
    HIP_TRY(hipMemcpy2D(host_soa, sizeof(float) * (size_t)n, arr, sizeof(float) * (size_t)stride,
                        sizeof(float) * (size_t)n, (size_t)narrays, hipMemcpyDeviceToHost));
    return GSR_OK;
}

extern "C" gsr_gaussian* gsr_load_ply_device_ex(const char* filename, int* out_n, int flags, int* out_narrays) {
    int64_t n = -1;
    int is4d = 0;
    int rc = gsr_ply_read_host_ex(filename, nullptr,
                                  (flags & GSR_PLY_SH3) ? GSR_SCENE_SH3_NARRAYS : GSR_SCENE_NARRAYS, 0, &n, flags,
                                  &is4d);
    if (n >= 0 && out_n) *out_n = (int)n;   // misc.cu:38 sets the count before reading data
    if (rc) {
        std::fprintf(stderr, "%s\n", g_err.c_str());
        return nullptr;
    }
    int narrays = (is4d && out_narrays) ? GSR_SCENE4D_NARRAYS : GSR_SCENE_NARRAYS;
    if (flags & GSR_PLY_SH3) narrays = GSR_SCENE_SH3_NARRAYS;   // 3D only (4D properties ignored)
    std::vector<float> soa((size_t)narrays * (size_t)n);
    rc = gsr_ply_read_host_ex(filename, soa.data(), narrays, n, &n, flags, nullptr);
    if (rc) {
        std::fprintf(stderr, "%s\n", g_err.c_str());
        return nullptr;
    }
    void* d = gsr_scene_upload_ex(soa.data(), narrays, n);
    if (!d) std::fprintf(stderr, "CUDA memory allocation failed: %s\n", g_err.c_str());
    if (out_narrays) *out_narrays = narrays;
    return static_cast<gsr_gaussian*>(d);
}

extern "C" gsr_gaussian* gsr_load_ply_device(const char* filename, int* out_n) {
    return gsr_load_ply_device_ex(filename, out_n, 0, nullptr);
}

gsr_gaussian* loadGaussianCudaFromPly(const std::string& filename, int* out_numGaussians) {
    return gsr_load_ply_device(filename.c_str(), out_numGaussians);
}

// ------------------------------------------------------------------ context

struct FrameEvents {
    int mode;
    hipEvent_t ev[GSR_NUM_STAGES + 1];
};

struct gsr_context {
    std::mutex mu;
    // capacities (elements)
    int64_t n_cap = 0, p_cap = 0, t_cap = 0, soa_cap = 0;
    uint4* rec = nullptr;
    uint64_t* items[2] = {nullptr, nullptr};
    // pair buffers: p_cap u64 each, used as {keys: p_cap x 4 B, values: p_cap x 4 B}
    uint64_t* pairs[2] = {nullptr, nullptr};
    uint64_t* rect = nullptr;        // per-Gaussian tile rectangle (preprocess output)
    bool rect_packed = false;        // this frame's rects are packed (binning path, set by gsr_preprocess)
    uint64_t* srect = nullptr;       // binning path: two u32 rect-payload buffers the depth sort carries
                                     // (pack_rect), one of them depth-ordered at its end
    uint16_t* spans = nullptr;       // binning path: per-Gaussian tile row spans (tile_row_spans)
    bool spans_frame = false;        // this frame's preprocess wrote them (the row pass reads them)
    uint32_t* hist = nullptr;
    uint32_t* totals = nullptr;
    unsigned long long* wg = nullptr;
    Stats* stats = nullptr;          // device: [0] frame, [1] sticky
    Stats* hstats = nullptr;         // host-mapped copy of the sticky stats
    Stats* hstats_dev = nullptr;
    uint2* ranges = nullptr;
    float* soa_tmp = nullptr;
    unsigned long long* consumed = nullptr;   // diagnostics: blend counters (or stamps)
    int64_t consumed_cap = 0;
    bool diagnostics = false;
    int blend_variant = 0;
    float time = 0.0f;               // frame time for 4D scene blocks
    int tile_items = 16;             // tile sort: items per thread (8 | 16)
    int depth_items = 0;             // depth sort: items per thread (0 = by size | 8 | 16)
    int tile_groups = 1024;          // tile sort: workgroup cap (measured best: 2 tiles of items per group)
    int tile_split_even = 1;         // tile sort: digits split evenly over the passes
    int depth_skip = 1;              // depth sort: skip trailing identity passes (device-side plan)
    int depth_budget = 4;            // binning path: depth passes launched (adapts to the plan's needs)
    int depth_budget_streak = 0;     // consecutive checked frames that needed fewer passes than the budget
    int depth_budget_seen = 0;       // most passes any of those frames needed
    int passes_launched = 4;         // passes the last depth sort launched
    uint32_t* dstats = nullptr;      // depth-sort pass plan: 4 final words + 4 per upsweep workgroup
    uint32_t* nlive = nullptr;       // visible count of the live partition (device word)
    int depth_compact = 2;           // live partition before the depth sort: 0 off, 1 on, 2 4D scenes only
    bool compact_frame = false;      // this frame's preprocess items went to items[1] for the partition
    bool last_compact = false;       // the last sorted frame sorted only its visible prefix
    int depth_groups = 0;            // depth sort: workgroup cap (0 = default)
    int tile_binning = 1;            // row + column binning instead of emit + tile sort (grids <= 256 x 256)
    int bin_row_items = 4;           // binning: items per thread of a row-pass tile (4 | 8 | 16)
    int bin_col_items = 8;           // binning: items per thread of a column-pass tile (4 | 8 | 16)
    int tile_spans = 2;              // binning: drop the tiles of a splat's first four tile rows that
                                     // it provably cannot composite on (GSR_TUNE_TILE_SPANS): 0 off,
                                     // 1 on, 2 on up to kSpansAutoMax Gaussians
    int bin_col_groups = 0;          // binning: column-pass workgroups (chunks are strided over them);
                                     // 0 = by scene size (n / 1024 clamped to 1024..4096)
    uint64_t* binmeta = nullptr;     // binning: row pair totals (u64 x 256) then row item totals (u32 x 256)
    uint32_t* cbins = nullptr;       // binning: column counts per chunk (256 x chunks)
    int64_t cbins_cap = 0;
    bool last_binned = false;        // the last sorted frame took the binning path
    int blend_exp = 1;               // blend: 1 = fast exp, exact decisions (default); 0 = gsr_blend_expf (bit-exact)
                                     // tests and guarded T tests (re-blends what it cannot vouch for)
    int depth_split = 2;             // GSR_TUNE_DEPTH_SPLIT: 0 off, 1 on, 2 on above kLargeScene Gaussians
    int split_pm = 250;              // split point: phase A bins the nearest split_pm / 1000 of the depth order
    uint32_t split_epoch = 0;        // bumped at every restart of the controller (retry, knob): phase B
                                     // publishes it with the split point, so evidence from before the
                                     // restart is never taken for the restarted split point's
    int split_floor = 0;             // 5/4 of the last split point that left blocks unsaturated
    int split_clean = 0;             // checked split frames in a row that left none
    int split_off_frames = 0;        // frames since the split point reached 1000 (split off); after
                                     // split_retry of them, on a new camera, the split is tried again
    int split_retry = 0;             // frames before the next retry (kSplitRetry, doubling after each
                                     // retry that found no saturating view, back after a clean one)
    float split_off_view[32] = {};   // V and P of the frame the split was turned off on
    float prev_view[32] = {};        // V and P of the previous frame (a still camera: the same twice)
    bool split_frame = false;        // the sorted frame is split (phase A lists binned by sort_locked)
    bool split_rebin = false;        // phase B's lists replaced phase A's: a repeated blend bins phase A again
    bool split_seen = false;         // a split frame was blended since the last controller update
    bool split_spec = false;         // speculate: queue no phase B (the split point cannot shrink further
                                     // and 8 checked frames in a row needed none); a frame that then
                                     // leaves a block unsaturated is reported as GSR_E_OVERFLOW
    bool frame_spec = false;         // the sorted frame is blended without phase B
    float split_view[32] = {};       // V and P of this context's last split frame: a frame speculates
                                     // only with the same camera (its threshold then fits it)
    uint32_t split_na = 0;           // phase A's depth-order prefix (count mode) / the split point
    bool split_key = false;          // the preprocess left its items in items[1] for a threshold partition
    bool frame_key = false;          // the sorted frame is split in key mode (near part sorted, far part
                                     // sorted by phase B)
    bool split_key_ready = false;    // *kcut holds a threshold from an earlier split frame of this context
    bool last_split_key = false;     // the last sorted frame left its far part unsorted (phase B may not run)
    uint32_t* kcut = nullptr;        // depth split: the next frame's depth threshold (device word)
    uint32_t* kcut_frame = nullptr;  // depth split: this frame's threshold (the near sort copies it)
    uint64_t* src_items = nullptr;   // depth split, key mode: the preprocess order (both sorts' pass 0 read it)
    uint32_t* sat = nullptr;         // depth split, phase B: summed-area table of the unsaturated tiles
    uint32_t* nfar = nullptr;        // depth split, phase B: far items whose rect touches one (device word)
    int64_t src_cap = 0;
    uint64_t* pre_out = nullptr;     // where the preprocess wrote its items
    bool records_partial = false;    // the preprocess wrote only the near Gaussians' records
    const float* pre_arrays = nullptr;   // the preprocessed scene arrays (the far record pass re-reads them)
    const void* pre_scene = nullptr;     // the scene pointer gsr_preprocess was given
    int64_t pre_stride = 0;
    int pre_layout = 0;
    uint32_t* dstats_far = nullptr;  // depth split: the far sort's pass plan
    int far_launched = 4;            // passes the far sort launched
    float* tbuf = nullptr;           // depth split: saved transmittance, 64 floats per 8x8 block
    uint8_t* bflag = nullptr;        // depth split: per block, left unsaturated by phase A
    uint32_t* gate = nullptr;        // depth split: count of such blocks (device word)
    int64_t split_cap = 0;           // blocks tbuf / bflag hold
    int blend_band_tiles = 4;        // blend: tiles per spatial band, bands dealt round-robin to the
                                     // XCDs (0: one contiguous band per XCD)
    int completion_events = 1;       // 0: no completion event / overflow query (stream capture)
    int rank_atomic = -1;            // GSR_TUNE_RANK_ATOMIC: 1 = ranks from returning LDS atomics when the
                                     // device self-check passed, 0 = ballot matching; -1 = not yet set
                                     // (the environment's GSR_RANK_ATOMIC=0 selects 0, else 1)
    bool rank_ok = false;            // the device passed the rank-order self-check (ensure_static)
    bool overflow_seen = false;      // an overflow was reported since the last gsr_sync (which reports it again)
    // bucket depth sort (GSR_TUNE_DEPTH_BUCKETS, gsr_kernels.hip "bucket depth sort")
    int fuse_rows = 1;               // GSR_TUNE_BUCKET_ROWS: the bucket sort's local kernel counts the row pass
    int col_chunk = 0;               // GSR_TUNE_COL_CHUNK: 0 = by scene size (col_chunk_for), 1024, 2048
    int bucket_sort = 1;             // 0 = LSD passes; 1 = bucket sort after the context's first frame
                                     // (big buckets above 2M, bkt_big); 2 = test hook: as 1 with a local
                                     // capacity of 64 items (most buckets take the global path); 3 = the
                                     // small-bucket kind at any size (A/B)
    uint32_t* bkt_split = nullptr;   // 2 x kMaxBuckets splitters (double-buffered: read one, write the other)
    uint4* bkt_rec = nullptr;        // the scatter's 16-B records (n_cap of them, with the items)
    int bkt_par = 0;                 // the half the next bucket-sorted frame reads
    int bkt_B = 0;                   // buckets the splitters were made for (0: none yet)
    const void* bkt_scene = nullptr; // the scene they were made from (another scene reseeds them)
    unsigned int bkt_work_seen = 0;  // hstats->bkt_over_work when the last frame was prepared
    bool bds_frame = false;          // this frame's preprocess items went to items[1] for the bucket sort
    bool last_bds = false;           // the last sorted frame was bucket-sorted (order in items[0], no pass plan)
    bool bkt_rows_fused = false;     // its local sorts wrote the row pass's counts (bucket = row chunk): the
                                     // next binning skips its count kernel (once: the row scan consumes them)
    int fail_frame = 0;              // GSR_TUNE_FAIL_FRAME: gsr_render_path fails this frame (> 0) once
    uint32_t* fstatus = nullptr;     // the current frame's validity word (gsr_render_path_status; device,
                                     // nullable): GSR_FRAME_* bits, written by its column scans / blend
    // frame state
    Frame fr{};
    int64_t n = 0;
    bool have_pre = false, have_sort = false;
    int pair_buf = 0;
    int ntiles = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done_ev = nullptr;
    bool pending = false;
    // timing
    int timing = 0;
    int timing_stride = 1;           // record the timing events on every k-th frame only
    int64_t timing_count = 0;        // frames seen since timing was enabled
    bool timing_now = false;         // this frame records events
    std::vector<hipEvent_t> ev_pool;
    std::vector<FrameEvents> ev_frames;
    FrameEvents cur{};
    // drop-in helpers
    float* out_tmp = nullptr;
    int64_t out_cap = 0;
    // frames in flight (gsr_render_path): lane 0 is this context on the caller's
    // stream; lane l >= 1 is a private child context (own workspace) on its own
    // non-blocking stream.  Children are only touched under this context's mutex.
    int inflight = 3;
    std::vector<gsr_context*> lanes;          // lanes[l - 1] = child of lane l
    std::vector<hipStream_t> lane_streams;    // lane_streams[l - 1]
    hipEvent_t fork_ev = nullptr;
    std::vector<hipEvent_t> join_evs;         // one per child lane
    std::vector<hipEvent_t> alias_evs;        // ring of `inflight` events: output reuse across lanes
};

namespace {

// Scenes above this many Gaussians: tile row spans off (their by-index code gather
// leaves the L2), the depth split on (GSR_TUNE_TILE_SPANS / GSR_TUNE_DEPTH_SPLIT = 2).
constexpr int64_t kLargeScene = 3 << 19;
constexpr int kSplitMinPm = 20;       // smallest split point (per mille)
constexpr int kSplitRetry = 256;      // frames with the split turned off before it is tried again
constexpr int kSplitRetryMax = 1 << 14;

// The depth split applies to this context's frames of n Gaussians (binning path;
// gsr_render / gsr_render_path decide it per frame, the stage API never).  Its two blend
// phases always run the exact blend, whatever GSR_TUNE_BLEND_EXP says for other frames.
bool split_enabled(const gsr_context* c, int64_t n) {
    return n > 0 && c->blend_variant != 3 && c->split_pm < 1000 &&
           (c->depth_split == 1 || (c->depth_split == 2 && n > kLargeScene));
}

// Buckets of the bucket depth sort for n items: about 1,024 items per bucket (local sorts
// of ~930 live items at config 2 against a 2,048-item capacity), 256..kMaxBuckets.
int bkt_count(int64_t n) {
    int b = 256;
    while (b < gsr::kMaxBuckets && (int64_t)b * 1024 < n) b *= 2;
    return b;
}

// Two kinds of bucket sort.  Up to 2M Gaussians ~n / 1,024 buckets (up to 4,096) of <= 2,048
// items sorted by 256-thread workgroups (config 2 one frame at a time +7.7 %, config 5 +9.7 %).
// Above, that kind's scatter measured slower than the LSD passes at 5M (config 3 orbit: 181
// against 141 us, profiles/r06d_kt_c3_orbit_bucket_it56.txt); there 512 big buckets of ~n / 512
// items (gsr_internal.h launch_bucket_sort_big), each sorted by one 1,024-thread workgroup in
// LDS: 124 us, config 3 orbit +2.1 % in flight, +1.7 % one frame at a time
// (profiles/r06k_big_buckets_c3_orbit.txt).  Knob 28: 1 (default) both kinds by size; 2 the
// test hook (64-item capacity, either kind); 3 the small-bucket kind at any size (A/B).
constexpr int64_t kBucketSortMaxN = (int64_t)2048 * 1024;
bool bkt_applies(const gsr_context* c, int64_t n) { return n > 0 && c->bucket_sort != 0; }
bool bkt_big(const gsr_context* c, int64_t n) { return c->bucket_sort != 3 && n > kBucketSortMaxN; }
// A/B: GSR_BIG_BUCKETS=1024 sorts 1,024 big buckets with 512-thread workgroups
int big_bucket_count() {
    static const int b = [] { const char* e = std::getenv("GSR_BIG_BUCKETS"); return e && std::atoi(e) == 1024 ? 1024 : gsr::kBigBuckets; }();
    return b;
}
int bkt_count(const gsr_context* c, int64_t n) { return bkt_big(c, n) ? big_bucket_count() : bkt_count(n); }

// Row items per column-pass chunk (GSR_TUNE_COL_CHUNK 0): 1,024 up to the same 2M
// Gaussians (config 2: column scatter 26.0 -> 21.6 us, chain -2 us), 2,048 above (config 3:
// the doubled chunk count costs the count and scan +10 us), profiles/r05_ab_col_chunk.txt.
int col_chunk_for(const gsr_context* c) {
    return c->col_chunk ? c->col_chunk : (c->n <= kBucketSortMaxN ? 1024 : 2048);
}

int groups_for(int64_t n, int64_t per) {
    int64_t g = (n + per - 1) / per;
    return (int)std::max<int64_t>(1, std::min<int64_t>(g, gsr::kMaxSortGroups));
}

template <typename T>
int realloc_dev(T** p, size_t count) {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    if (count == 0) count = 1;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * count));
    return GSR_OK;
}

// ---- rank-order self-check, once per process and device (gsr_kernels.hip
// k_rank_order_check).  The sort and binning kernels rank with returning LDS atomics
// only on a gfx950 device that returned every same-address lane in lane order.
struct RankCheck {
    int state = -1;                  // -1 not run, 0 failed / not gfx950, 1 passed
    unsigned long long ops = 0, bad = 0;
};
std::mutex g_rank_mu;
std::unordered_map<int, RankCheck> g_rank;

int rank_check_device(RankCheck* out) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_rank_mu);
    RankCheck& rc = g_rank[dev];
    if (rc.state < 0) {
        hipDeviceProp_t prop{};
        HIP_TRY(hipGetDeviceProperties(&prop, dev));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            rc.state = 0;
        } else {
            HIP_TRY(gsr::rank_order_check(&rc.ops, &rc.bad));
            rc.state = rc.ops > 0 && rc.bad == 0 ? 1 : 0;
        }
    }
    if (out) *out = rc;
    return GSR_OK;
}

int default_rank_atomic() {
    const char* e = std::getenv("GSR_RANK_ATOMIC");
    return e && e[0] == '0' ? 0 : 1;
}

int ensure_static(gsr_context* c) {
    if (c->rank_atomic < 0) c->rank_atomic = default_rank_atomic();
    if (c->hist) return GSR_OK;
    {
        RankCheck rk;
        if (int rc = rank_check_device(&rk)) return rc;
        c->rank_ok = rk.state == 1;
    }
    if (int rc = realloc_dev(&c->hist, 256 * (size_t)gsr::kMaxSortGroups)) return rc;
    // LSD digit totals / bucket totals + bucket starts
    if (int rc = realloc_dev(&c->totals, 2 * (size_t)gsr::kMaxBuckets + 2)) return rc;
    if (int rc = realloc_dev(&c->bkt_split, 2 * (size_t)gsr::kMaxBuckets)) return rc;
    if (int rc = realloc_dev(&c->wg, (size_t)gsr::kMaxSortGroups)) return rc;
    if (int rc = realloc_dev(&c->stats, 2)) return rc;
    if (int rc = realloc_dev(&c->dstats, 4 + 4 * (size_t)gsr::kMaxSortGroups)) return rc;
    if (int rc = realloc_dev(&c->nlive, 1)) return rc;
    if (int rc = realloc_dev(&c->binmeta, 256 + 128)) return rc;
    if (int rc = realloc_dev(&c->gate, 1)) return rc;
    if (int rc = realloc_dev(&c->kcut, 1)) return rc;
    if (int rc = realloc_dev(&c->kcut_frame, 1)) return rc;
    if (int rc = realloc_dev(&c->nfar, 1)) return rc;
    if (int rc = realloc_dev(&c->sat, 257 * 257)) return rc;   // grids <= 256 x 256 tiles
    if (int rc = realloc_dev(&c->dstats_far, 4 + 4 * (size_t)gsr::kMaxSortGroups)) return rc;
    HIP_TRY(hipMemset(c->kcut, 0xff, sizeof(uint32_t)));
    HIP_TRY(hipMemset(c->stats, 0, 2 * sizeof(Stats)));
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->hstats), sizeof(Stats), hipHostMallocMapped));
    std::memset(c->hstats, 0, sizeof(Stats));
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->hstats_dev), c->hstats, 0));
    HIP_TRY(hipEventCreateWithFlags(&c->done_ev, hipEventDisableTiming));
    return GSR_OK;
}

int ensure_n(gsr_context* c, int64_t n) {
    if (n <= c->n_cap) return GSR_OK;
    const int64_t cap = std::max<int64_t>(n, 1024);
    HIP_TRY(hipDeviceSynchronize());
    if (int rc = realloc_dev(&c->rec, 4 * (size_t)cap)) return rc;
    if (int rc = realloc_dev(&c->items[0], (size_t)cap)) return rc;
    if (int rc = realloc_dev(&c->items[1], (size_t)cap)) return rc;
    if (int rc = realloc_dev(&c->rect, (size_t)cap)) return rc;
    if (int rc = realloc_dev(&c->srect, (size_t)cap)) return rc;
    if (int rc = realloc_dev(&c->spans, (size_t)cap)) return rc;
    // the bucket sort's 16-B records (allocated with the items, so gsr_reserve covers them
    // and a captured frame never allocates)
    if (int rc = realloc_dev(&c->bkt_rec, (size_t)cap)) return rc;
    c->n_cap = cap;
    if (c->p_cap < 4 * cap) {
        const int64_t pc = std::min<int64_t>(std::max<int64_t>(4 * cap, 1 << 20), 0xffffffffLL);
        if (int rc = realloc_dev(&c->pairs[0], (size_t)pc)) return rc;
        if (int rc = realloc_dev(&c->pairs[1], (size_t)pc)) return rc;
        c->p_cap = pc;
    }
    return GSR_OK;
}

int ensure_pairs(gsr_context* c, int64_t p) {
    if (p <= c->p_cap) return GSR_OK;
    const int64_t pc = std::min<int64_t>(p, 0xffffffffLL);
    HIP_TRY(hipDeviceSynchronize());
    if (int rc = realloc_dev(&c->pairs[0], (size_t)pc)) return rc;
    if (int rc = realloc_dev(&c->pairs[1], (size_t)pc)) return rc;
    c->p_cap = pc;
    return GSR_OK;
}

int ensure_tiles(gsr_context* c, int64_t t) {
    if (t <= c->t_cap) return GSR_OK;
    HIP_TRY(hipDeviceSynchronize());
    if (int rc = realloc_dev(&c->ranges, (size_t)t)) return rc;
    c->t_cap = t;
    return GSR_OK;
}

// Depth split, key mode: the preprocess order of n items.
int ensure_src(gsr_context* c, int64_t n) {
    if (n <= c->src_cap) return GSR_OK;
    HIP_TRY(hipDeviceSynchronize());
    if (int rc = realloc_dev(&c->src_items, (size_t)std::max<int64_t>(n, 1024))) return rc;
    c->src_cap = std::max<int64_t>(n, 1024);
    return GSR_OK;
}

// Depth split buffers for the current tile grid (4 blocks per tile).
int ensure_split(gsr_context* c) {
    const int64_t blocks = 4 * (int64_t)c->ntiles;
    if (blocks <= c->split_cap) return GSR_OK;
    HIP_TRY(hipDeviceSynchronize());
    if (int rc = realloc_dev(&c->tbuf, 64 * (size_t)blocks)) return rc;
    if (int rc = realloc_dev(&c->bflag, (size_t)blocks)) return rc;
    c->split_cap = blocks;
    return GSR_OK;
}

int ensure_soa(gsr_context* c, int64_t n) {
    const int64_t need = (int64_t)GSR_SCENE_NARRAYS * scene_stride(n);
    if (need <= c->soa_cap) return GSR_OK;
    HIP_TRY(hipDeviceSynchronize());
    if (int rc = realloc_dev(&c->soa_tmp, (size_t)need)) return rc;
    c->soa_cap = need;
    return GSR_OK;
}

hipEvent_t get_event(gsr_context* c) {
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// Record the boundary event that opens stage `stage` (stage == GSR_NUM_STAGES closes the frame).
void mark(gsr_context* c, int stage) {
    if (!c->timing || !c->timing_now) return;
    const bool want = (c->timing == 2) || stage == GSR_STAGE_BLEND || stage == GSR_STAGE_RESUME ||
                      stage == GSR_NUM_STAGES;
    if (!want) return;
    hipEvent_t e = get_event(c);
    if (!e) return;
    c->cur.ev[stage] = e;
    (void)hipEventRecord(e, c->stream);
}

// The split point and the controller's epoch as phase B publishes them (Stats::split_pm).
uint32_t split_tag(const gsr_context* c) { return (uint32_t)c->split_pm | ((c->split_epoch & 0xffffu) << 16); }

// Depth split point after a frame that needed phase B: up by half, floor at 5/4 of the
// old point, no speculation.
void split_grow(gsr_context* c) {
    c->split_floor = std::min(1000, c->split_pm * 5 / 4 + 1);
    c->split_pm = std::min(1000, c->split_pm * 3 / 2 + 1);
    c->split_clean = 0;
    c->split_spec = false;
}

void hv_clear_spec(gsr_context* c) {
    reinterpret_cast<volatile Stats*>(c->hstats)->spec_miss = 0;
}

// Read the sticky stats of finished work; grow the pair buffer after an overflow.
// An overflow (pairs over capacity, a depth sort short of passes, or a speculative
// depth-split frame that needed phase B) is reported once here and remembered in
// overflow_seen until gsr_sync, so a blocking sync also reports what a non-blocking
// check inside a render call already consumed.  The depth split's controller runs here
// too (the counts phase B published for the finished frames).
int check_overflow(gsr_context* c, bool blocking) {
    if (!c->pending) {
        // with completion events off (stream capture) no event marks finished work: a
        // blocking check (gsr_sync) drains the device and reads the sticky words anyway,
        // so an overflow or a speculative miss is still reported there
        if (!blocking || c->completion_events || !c->hstats) return GSR_OK;
        HIP_TRY(hipDeviceSynchronize());
    } else if (blocking) {
        HIP_TRY(hipEventSynchronize(c->done_ev));
    } else if (hipEventQuery(c->done_ev) != hipSuccess) {
        return GSR_OK;
    }
    c->pending = false;
    const volatile Stats* hv = c->hstats;
    Stats s{};
    s.pairs_total = hv->pairs_total;
    s.pairs_eff = hv->pairs_eff;
    s.overflow = hv->overflow;
    s.depth_passes = hv->depth_passes;
    if (!s.overflow && hv->spec_miss) {
        // a speculative frame (no phase B queued) left a block unsaturated: drain, then
        // report it like an overflow (the caller re-renders) and stop speculating
        HIP_TRY(hipDeviceSynchronize());
        hv_clear_spec(c);
        split_grow(c);
        c->overflow_seen = true;
        return set_err(GSR_E_OVERFLOW, "depth split: a frame rendered without phase B left blocks unsaturated; "
                                       "re-render");
    }
    if (!s.overflow && c->split_seen) {
        // depth split point: up by half when phase A left blocks unsaturated (phase B
        // ran), down by an eighth after 8 checked frames in a row that needed no phase B,
        // never below 5/4 of the last point that needed it; when it cannot shrink any
        // further, the next frames speculate (no phase B queued)
        c->split_seen = false;
        const int64_t u = hv->split_unsat;
        if (hv->split_pm != split_tag(c)) {
            // the newest phase B ran at an earlier split point (frames in flight): no
            // evidence about the current one yet
        } else if (u == 0) {
            c->split_retry = kSplitRetry;   // a saturating view: the next turn-off retries soon
            if (++c->split_clean >= 8) {
                c->split_clean = 0;
                const int next = std::max(std::max(kSplitMinPm, c->split_floor), c->split_pm * 7 / 8);
                if (next >= c->split_pm) c->split_spec = true;
                c->split_pm = next;
            }
        } else {
            const int pm_old = c->split_pm;
            split_grow(c);   // phase A left blocks unsaturated
            // at or above the starting point, 2 % of the blocks or more left unsaturated
            // means tiles that see past the scene, which no split point saturates (phase B
            // would run on every frame, at a cost above the unsplit frame's): off at once
            // rather than in four growth steps (automatic mode; a forced split keeps growing)
            if (c->depth_split == 2 && pm_old >= 250 && u * 50 >= 4 * (int64_t)c->ntiles) c->split_pm = 1000;
            if (c->split_pm >= 1000) {
                // the split turned itself off: the next frames list the whole order's pairs.
                // Size the pair buffer for them now (the split frames' pairs scaled to the
                // whole order) rather than overflow and re-render a chunk
                const int64_t want = (int64_t)(s.pairs_total * 1000 / (unsigned)pm_old) * 5 / 4 + 4096;
                if (int rc = ensure_pairs(c, want)) return rc;
            }
        }
    }
    if (!s.overflow) {
        // lower the pass budget once 4 checked frames in a row needed fewer passes
        if (s.depth_passes >= 1 && (int)s.depth_passes < c->depth_budget) {
            c->depth_budget_seen = std::max(c->depth_budget_seen, (int)s.depth_passes);
            if (++c->depth_budget_streak >= 4) {
                c->depth_budget = c->depth_budget_seen;
                c->depth_budget_streak = 0;
                c->depth_budget_seen = 0;
            }
        } else {
            c->depth_budget_streak = 0;
            c->depth_budget_seen = 0;
        }
        return GSR_OK;
    }
    // frames queued after the event may still be running: drain them, then read the
    // sticky stats again, so that a pair overflow of one of them (bit 0) is seen and
    // the grown capacity covers its total too (ensure_pairs syncs again; cheap)
    HIP_TRY(hipDeviceSynchronize());
    s.overflow |= hv->overflow;
    if (hv->pairs_total > s.pairs_total) s.pairs_total = hv->pairs_total;
    c->overflow_seen = true;
    // a speculative miss in the same frames: stop speculating before the words are
    // cleared, or the re-render of this camera speculates (and misses) again
    if (hv->spec_miss) split_grow(c);
    if (s.overflow & 2u) {   // back to four launched passes
        c->depth_budget = 4;
        c->depth_budget_streak = 0;
        c->depth_budget_seen = 0;
    }
    if (s.overflow & 1u) {
        const int64_t want = (int64_t)(s.pairs_total + s.pairs_total / 4 + 4096);
        if (int rc = ensure_pairs(c, want)) return rc;
    }
    HIP_TRY(hipMemset(c->stats + 1, 0, sizeof(Stats)));
    std::memset(c->hstats, 0, sizeof(Stats));
    if (s.overflow & 1u)
        return set_err(GSR_E_OVERFLOW, "pair buffer overflowed (%llu pairs); grown to %lld; re-render",
                       (unsigned long long)s.pairs_total, (long long)c->p_cap);
    return set_err(GSR_E_OVERFLOW, "depth sort needed %u passes, %d were launched; re-render",
                   (unsigned)s.depth_passes, c->passes_launched);
}

int fill_frame(gsr_context* c, const gsr_camera* cam, int W, int H, int nx, int ny, int ws, int hs, float k) {
    if (!cam) return set_err(GSR_E_ARG, "null camera");
    if (W <= 0 || H <= 0 || W > 32768 || H > 32768)
        return set_err(GSR_E_ARG, "image size %dx%d out of range [1, 32768]", W, H);
    if (nx <= 0 || ny <= 0 || ws <= 0 || hs <= 0)
        return set_err(GSR_E_ARG, "bad tiling nx=%d ny=%d ws=%d hs=%d", nx, ny, ws, hs);
    Frame& f = c->fr;
    std::memcpy(f.V, cam->V_matrix, sizeof f.V);
    std::memcpy(f.P, cam->P_matrix, sizeof f.P);
    std::memcpy(f.Rc, cam->r_cam, sizeof f.Rc);
    std::memcpy(f.RcT, cam->r_cam_T, sizeof f.RcT);
    std::memcpy(f.campos, cam->position, sizeof f.campos);
    f.znear = cam->nearClip;
    gsr_camera_intrinsics(cam, &f.fx, &f.fy);
    f.k = k;
    f.W = W;
    f.H = H;
    f.cover_w = (int)std::min<int64_t>((int64_t)nx * ws, W);
    f.cover_h = (int)std::min<int64_t>((int64_t)ny * hs, H);
    f.tiles_x = (W + GSR_TILE_PX - 1) / GSR_TILE_PX;
    f.tiles_y = (H + GSR_TILE_PX - 1) / GSR_TILE_PX;
    return GSR_OK;
}

int ceil_log2(int64_t v) {
    int k = 0;
    while ((int64_t(1) << k) < v) k++;
    return k;
}

}  // namespace

extern "C" gsr_context* gsr_create(void) {
    gsr_context* c = new gsr_context();
    const char* e = std::getenv("GSR_BLEND_EXP");
    if (e && e[0] == '0') c->blend_exp = 0;   // the exact blend (bit-identical to the oracle)
    if (e && e[0] == '1') c->blend_exp = 1;
    return c;
}

extern "C" void gsr_destroy(gsr_context* c) {
    if (!c) return;
    (void)hipDeviceSynchronize();
    for (auto* l : c->lanes) gsr_destroy(l);
    for (auto s : c->lane_streams) (void)hipStreamDestroy(s);
    for (auto e : c->join_evs) (void)hipEventDestroy(e);
    for (auto e : c->alias_evs) (void)hipEventDestroy(e);
    if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
    for (auto* p : {(void*)c->rec, (void*)c->items[0], (void*)c->items[1], (void*)c->rect, (void*)c->pairs[0],
                    (void*)c->pairs[1], (void*)c->hist, (void*)c->totals, (void*)c->wg, (void*)c->stats, (void*)c->dstats,
                    (void*)c->ranges, (void*)c->soa_tmp, (void*)c->out_tmp, (void*)c->consumed, (void*)c->binmeta,
                    (void*)c->cbins, (void*)c->srect, (void*)c->spans, (void*)c->nlive, (void*)c->tbuf,
                    (void*)c->bflag, (void*)c->gate, (void*)c->kcut, (void*)c->dstats_far, (void*)c->kcut_frame,
                    (void*)c->src_items, (void*)c->sat, (void*)c->nfar, (void*)c->bkt_rec})
        if (p) (void)hipFree(p);
    if (c->hstats) (void)hipHostFree(c->hstats);
    if (c->done_ev) (void)hipEventDestroy(c->done_ev);
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    for (auto& f : c->ev_frames)
        for (auto e : f.ev)
            if (e) (void)hipEventDestroy(e);
    delete c;
}

extern "C" int gsr_reserve(gsr_context* c, int64_t n, int64_t pairs) {
    if (!c || n < 0 || pairs < 0) return set_err(GSR_E_ARG, "gsr_reserve: bad argument");
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = ensure_static(c)) return rc;
    if (int rc = ensure_n(c, n)) return rc;
    return ensure_pairs(c, pairs);
}

static int preprocess_locked(gsr_context* c, const void* scene, int layout, int64_t n, const gsr_camera* cam,
                             int W, int H, int nx, int ny, int ws, int hs, float k, void* stream) {
    if (n < 0 || n > INT32_MAX) return set_err(GSR_E_ARG, "Gaussian count %lld out of range", (long long)n);
    if (n > 0 && !scene) return set_err(GSR_E_ARG, "null scene");
    if (layout != GSR_LAYOUT_SCENE_BLOCK && layout != GSR_LAYOUT_AOS && layout != GSR_LAYOUT_SCENE_BLOCK_4D &&
        layout != GSR_LAYOUT_SCENE_BLOCK_SH3)
        return set_err(GSR_E_ARG, "unknown scene layout %d", layout);
    if (int rc = fill_frame(c, cam, W, H, nx, ny, ws, hs, k)) return rc;
    if (int rc = ensure_static(c)) return rc;
    int rc_over = check_overflow(c, false);
    if (rc_over != GSR_OK && rc_over != GSR_E_OVERFLOW) return rc_over;
    if (int rc = ensure_n(c, n)) return rc;
    c->ntiles = c->fr.tiles_x * c->fr.tiles_y;
    if (int rc = ensure_tiles(c, c->ntiles)) return rc;
    c->stream = static_cast<hipStream_t>(stream);
    c->n = n;
    if (c->timing) {
        c->cur = FrameEvents{};
        c->cur.mode = c->timing;
        c->timing_now = (c->timing_count++ % c->timing_stride) == 0;
    }
    mark(c, GSR_STAGE_PREPROCESS);
    const float* arrays = nullptr;
    int64_t stride = scene_stride(n);
    if (layout == GSR_LAYOUT_AOS) {
        if (int rc = ensure_soa(c, n)) return rc;
        HIP_TRY(gsr::launch_aos_to_soa(static_cast<const gsr_gaussian*>(scene), n, c->soa_tmp, stride, c->stream));
        arrays = c->soa_tmp;
    } else {
        arrays = reinterpret_cast<const float*>(static_cast<const char*>(scene) + GSR_SCENE_HEADER_BYTES);
    }
    // depth split: the controller turned it off (split point 1000) because phase A kept
    // leaving blocks unsaturated; a camera that moved elsewhere can bring back views whose
    // tiles all saturate, so after split_retry frames, once the camera differs from the
    // one it was turned off on (a fixed camera, or a 4D scene's fixed camera over time,
    // never retries) and has stopped there (the same camera two frames running: a camera
    // that keeps moving, e.g. an orbit, never retries — its threshold would always come
    // from another view, and the controller's evidence lags the frames queued ahead of
    // it), it is tried again from the starting point; each retry doubles the next wait,
    // up to kSplitRetryMax, until a retry finds a view whose tiles all saturate
    const bool still = std::memcmp(c->prev_view, c->fr.V, sizeof c->fr.V) == 0 &&
                       std::memcmp(c->prev_view + 16, c->fr.P, sizeof c->fr.P) == 0;
    std::memcpy(c->prev_view, c->fr.V, sizeof c->fr.V);
    std::memcpy(c->prev_view + 16, c->fr.P, sizeof c->fr.P);
    if (c->split_pm >= 1000 && (c->depth_split == 1 || (c->depth_split == 2 && n > kLargeScene))) {
        if (c->split_off_frames == 0) {
            std::memcpy(c->split_off_view, c->fr.V, sizeof c->fr.V);
            std::memcpy(c->split_off_view + 16, c->fr.P, sizeof c->fr.P);
        }
        if (c->split_retry == 0) c->split_retry = kSplitRetry;
        c->split_off_frames = std::min(c->split_off_frames + 1, 1 << 30);
        const bool moved = std::memcmp(c->split_off_view, c->fr.V, sizeof c->fr.V) != 0 ||
                           std::memcmp(c->split_off_view + 16, c->fr.P, sizeof c->fr.P) != 0;
        if (c->split_off_frames >= c->split_retry && moved && still) {
            c->split_retry = std::min(2 * c->split_retry, kSplitRetryMax);
            c->split_off_frames = 0;
            c->split_pm = 250;
            c->split_epoch++;
            c->split_floor = 0;
            c->split_clean = 0;
            c->split_key_ready = false;
        }
    } else {
        c->split_off_frames = 0;
    }
    // depth split with a depth threshold (a threshold exists from an earlier split
    // frame): the items go to src_items, which both sorts' pass 0 read
    c->split_key = split_enabled(c, n) && c->split_key_ready && c->tile_binning && c->fr.tiles_x <= 256 &&
                   c->fr.tiles_y <= 256;
    // live partition (global depth sort on the binning path): the items go to
    // items[1] and the partition writes the visible-first order into items[0]
    // bucket depth sort (splitters exist for this scene size): the items go to items[1], the
    // sort writes the order into items[0]; it keeps culled items apart itself, so it
    // replaces the live partition
    // the splitters are this scene's and did not just fail: a frame whose global path sorted
    // more than n / 8 item-passes (a camera cut, a zoom: most of the scene in a few buckets
    // over capacity, with wide key spans) makes the next one reseed them from the LSD passes
    // (a camera jump could put most of a 2M scene into one bucket, sorted by one
    // workgroup, a frame of tens of ms).  Buckets of tied keys cost the global path nothing
    // (no passes) and do not count: reseeding could not split them.  bkt_over_work is
    // host-mapped and lags by the frames in flight; the test hook 2 (capacity 64) keeps them.
    {
        const unsigned int work = c->hstats ? ((const volatile Stats*)c->hstats)->bkt_over_work : 0u;
        const bool spike = c->bucket_sort != 2 && (int64_t)(work - c->bkt_work_seen) > n / 8;
        c->bkt_work_seen = work;
        if (c->bkt_B && (spike || c->bkt_scene != scene)) c->bkt_B = 0;
    }
    c->bds_frame = bkt_applies(c, n) && !c->split_key && c->bucket_sort && c->bkt_B == bkt_count(c, n) && c->tile_binning &&
                   c->fr.tiles_x <= 256 && c->fr.tiles_y <= 256;
    c->compact_frame = n > 0 && !c->split_key && !c->bds_frame &&
                       (c->depth_compact == 1 || (c->depth_compact == 2 && layout == GSR_LAYOUT_SCENE_BLOCK_4D)) &&
                       c->tile_binning && c->fr.tiles_x <= 256 && c->fr.tiles_y <= 256;
    // the binning path takes the tile rects packed to 4 B (pack_rect), the pair path 8 B;
    // the sort follows the path chosen here (rect_packed)
    c->rect_packed = c->tile_binning && c->fr.tiles_x <= 256 && c->fr.tiles_y <= 256;
    // tile row spans: the row pass gathers each source's 2-B code by index; up to 1.5M
    // Gaussians the codes (<= 3 MB) stay in an XCD's 4-MB L2 and the gather is cheap:
    // config 2 (1M) +0.8 % one frame at a time, +1.2 % in flight; config 5 (2M) -1 % in
    // flight, config 3 (5M) -3 / -6 % (profiles/r02_ab_tile_spans.txt)
    c->spans_frame = c->rect_packed && (c->tile_spans == 1 || (c->tile_spans == 2 && n <= kLargeScene));
    // key mode: records only for the Gaussians nearer than the threshold (the far ones
    // are written by a second pass if phase B or a one-phase sort needs them)
    // (speculative frames only: a frame that queues phase B needs every record there)
    c->records_partial = c->split_key && c->split_spec && !c->spans_frame;
    c->pre_arrays = arrays;
    c->pre_scene = scene;
    c->pre_stride = stride;
    c->pre_layout = layout;
    const gsr::RecSplit rsp{c->records_partial ? 1 : 0, c->kcut, c->kcut_frame, nullptr};
    if (c->split_key) {
        if (int rc = ensure_src(c, n)) return rc;
    }
    c->pre_out = c->split_key ? c->src_items : c->items[c->compact_frame || c->bds_frame ? 1 : 0];
    HIP_TRY(gsr::launch_preprocess(arrays, stride, n, c->fr, c->rec, c->pre_out,
                                   c->rect,
                                   c->rect_packed, layout == GSR_LAYOUT_SCENE_BLOCK_4D,
                                   layout == GSR_LAYOUT_SCENE_BLOCK_SH3, c->time, c->stream,
                                   c->spans_frame ? c->spans : nullptr, &rsp));
    c->have_pre = true;
    c->have_sort = false;
    return rc_over;
}

static void* pair_keys(gsr_context* c, int b) { return c->pairs[b]; }
static uint32_t* pair_vals(gsr_context* c, int b) {
    return reinterpret_cast<uint32_t*>(c->pairs[b]) + c->p_cap;
}

// Column-pass chunk counts for the current capacity and grid.
static int ensure_cbins(gsr_context* c) {
    const int64_t need = 256 * (int64_t)gsr::bin_col_chunks_max((uint32_t)c->p_cap, c->fr.tiles_y);
    if (need > c->cbins_cap) {
        HIP_TRY(hipDeviceSynchronize());
        if (int rc = realloc_dev(&c->cbins, (size_t)need)) return rc;
        c->cbins_cap = need;
    }
    return GSR_OK;
}

// Ranks from returning LDS atomics: asked for (GSR_TUNE_RANK_ATOMIC) and verified on the device.
static bool rank_atomic_on(const gsr_context* c) { return c->rank_atomic > 0 && c->rank_ok; }

// Rect payload buffer b (0 or 1) of the binning's depth sort: the two u32 halves of srect.
static uint32_t* pay_buf(gsr_context* c, int b) {
    return reinterpret_cast<uint32_t*>(c->srect) + (b ? c->n_cap : 0);
}

// Global stable depth sort of the preprocess items (key << 32 | index), 4 x 8-bit
// passes with the device-side pass plan; with rects (binning) the passes carry them and
// leaves them in depth order (pay_buf(c, passes run & 1)).  Result in items[passes run & 1].
static int depth_sort_locked(gsr_context* c, bool with_rects, bool plain = false) {
    const uint32_t n = (uint32_t)c->n;
    c->bkt_rows_fused = false;
    // bucket depth sort: the first sort of a frame whose preprocess prepared for it (a
    // repeated sort of the frame takes the LSD passes over the sorted items[0])
    if (with_rects && !c->split_key && c->bds_frame && !c->have_sort && c->pre_out != c->items[0]) {
        const int B = c->bkt_B;
        if (bkt_big(c, c->n)) {
            // 512 buckets of ~n / 512 items, four 2,048-item tiles per scatter workgroup; the row
            // pass counts for itself (its 2,048-source chunks are cheaper than bucket chunks)
            static const int g_env = [] { const char* e = std::getenv("GSR_BB_GROUPS"); return e ? std::atoi(e) : 0; }();
            const int G = std::min(g_env > 0 ? g_env : groups_for(c->n, 4 * gsr::kMaxBucketCap), gsr::kBigBucketGroups);
            uint32_t* s_in = c->bkt_split + (size_t)c->bkt_par * gsr::kMaxBuckets;
            uint32_t* s_out = c->bkt_split + (size_t)(c->bkt_par ^ 1) * gsr::kMaxBuckets;
            HIP_TRY(gsr::launch_bucket_sort_big(c->pre_out, c->items[0], c->items[1], n, B, G, s_in, s_out, c->hist,
                                                c->totals, reinterpret_cast<const uint32_t*>(c->rect), pay_buf(c, 0),
                                                pay_buf(c, 1), rank_atomic_on(c), c->bucket_sort == 2 ? 64u : 16384u,
                                                c->hstats_dev ? &c->hstats_dev->bkt_over : nullptr, c->stream,
                                                c->bkt_rec));
            c->bkt_rows_fused = false;
            c->bkt_par ^= 1;
            c->last_bds = true;
            c->last_compact = false;
            c->last_split_key = false;
            c->compact_frame = false;
            c->bds_frame = false;
            c->passes_launched = 4;
            return GSR_OK;
        }
        const int G = std::min(groups_for(c->n, gsr::kMaxBucketCap), gsr::kMaxBucketGroups);
        // a plain frame (one binning over the whole order): the local sorts also count the
        // row pass's items and pairs per bucket, which becomes the row pass's chunk
        const bool fuse = plain && c->fuse_rows && (int64_t)512 * B <= 256 * (int64_t)gsr::kMaxSortGroups;
        uint32_t* s_in = c->bkt_split + (size_t)c->bkt_par * gsr::kMaxBuckets;
        uint32_t* s_out = c->bkt_split + (size_t)(c->bkt_par ^ 1) * gsr::kMaxBuckets;
        HIP_TRY(gsr::launch_bucket_sort(c->pre_out, c->items[0], c->items[1], n, B, G, s_in, s_out, c->hist,
                                        c->totals, reinterpret_cast<const uint32_t*>(c->rect), pay_buf(c, 0),
                                        pay_buf(c, 1), rank_atomic_on(c), c->bucket_sort == 2 ? 64u : gsr::kMaxBucketCap,
                                        c->hstats_dev ? &c->hstats_dev->bkt_over : nullptr, c->stream,
                                        fuse ? c->fr.tiles_y : 0, c->bkt_rec));
        c->bkt_rows_fused = fuse;
        c->bkt_par ^= 1;
        c->last_bds = true;
        c->last_compact = false;
        c->last_split_key = false;
        c->compact_frame = false;
        c->bds_frame = false;
        c->passes_launched = 4;   // no pass plan on this frame: the column scan's depth check is off
        return GSR_OK;
    }
    c->last_bds = false;
    // smaller tiles for the 1M-item depth sort: ~500 workgroups instead of ~250 (-2.6 %
    // frame time one at a time; in flight 8 and 16 measure within 1.5 % of each other,
    // either way round: profiles/r02_ab_depth_items.txt)
    // depth split, key mode: pass 0 reads the whole preprocess order (src_items) and keeps
    // the keys below the threshold; the passes sort only that near part (its count goes to
    // nlive; about 2 x the split point's items), the far part is sorted inside phase B
    const bool key = with_rects && c->split_key;
    const int64_t n_sorted =
        key ? std::min<int64_t>(c->n, std::max<int64_t>(2 * ((int64_t)c->n * c->split_pm / 1000), 65536)) : c->n;
    const int di = c->depth_items ? c->depth_items : (n_sorted < (int64_t(4) << 20) ? 8 : 16);
    int gd = groups_for(key ? c->n : n_sorted, 256 * di);   // pass 0 reads all n
    int gd_near = groups_for(n_sorted, 256 * di);
    if (c->depth_groups) {
        gd = std::min(gd, c->depth_groups);
        gd_near = std::min(gd_near, c->depth_groups);
    }
    const bool part = with_rects && c->compact_frame;
    // visible items first (index order) into items[0]; the passes sort only those
    if (part)
        HIP_TRY(gsr::launch_partition(c->pre_out, n, std::min(groups_for(c->n, 4096), gsr::kMaxSortGroups), c->hist,
                                      c->nlive, c->items[0], reinterpret_cast<const uint32_t*>(c->rect),
                                      pay_buf(c, 0), pay_buf(c, 1), c->stream));
    // a repeated sort of a key-mode frame starts again from the preprocess order
    const bool resort_src = !key && !part && c->have_sort && c->last_split_key;
    if (resort_src)
        HIP_TRY(hipMemcpyAsync(c->items[0], c->src_items, (size_t)n * 8, hipMemcpyDeviceToDevice, c->stream));
    c->last_compact = part;
    c->last_split_key = key;
    if (key) c->split_key = false;
    // pass 0's rect payloads: from the partition (-1), read at the item's position when
    // the input is the preprocess order (1: item j has index j), else gathered (0)
    const int rect_mode = part ? -1 : (key || resort_src || !c->have_sort ? 1 : 0);
    // items[1] is the sort's scratch from here on; a repeated sort of this frame sorts
    // the whole partitioned items[0] (same order: visible and culled keys never tie)
    if (part) c->compact_frame = false;
    // Trailing passes the device plan skips still cost a launch each (upsweep, scan and
    // downsweep returning at once: ~12 us of the frame's dependent chain).  On the
    // binning path the host launches only as many passes as recent frames needed
    // (depth_budget, check_overflow); a frame that needs more is flagged by the
    // column scan and re-rendered with all four, like a pair-buffer overflow.
    const int launch = with_rects && c->depth_skip ? std::max(1, std::min(4, c->depth_budget)) : 4;
    c->passes_launched = launch;
    const gsr::SortFilter near{1, c->kcut, c->nlive, c->kcut_frame};
    for (int p = 0; p < launch; p++) {
        const bool f0 = key && p == 0;
        HIP_TRY(gsr::launch_radix_pass(f0 ? c->src_items : c->items[p & 1], c->items[(p + 1) & 1],
                                       (part || (key && p > 0)) ? c->nlive : nullptr, n, 32 + 8 * p, 8,
                                       key && p > 0 ? gd_near : gd, di,
                                       c->hist, c->totals, nullptr, c->stream, c->depth_skip ? c->dstats : nullptr,
                                       p, with_rects ? reinterpret_cast<const uint32_t*>(c->rect) : nullptr, rect_mode,
                                       with_rects ? pay_buf(c, 0) : nullptr,
                                       with_rects ? pay_buf(c, 1) : nullptr, rank_atomic_on(c), nullptr, nullptr,
                                       f0 ? &near : nullptr));
    }
    // the bucket sort's first splitters: quantiles of this whole sorted order (the next
    // frame of this scene size is bucket-sorted)
    if (with_rects && !key && c->bucket_sort && bkt_applies(c, c->n) && c->bkt_B != bkt_count(c, c->n)) {
        const int B = bkt_count(c, c->n);
        HIP_TRY(gsr::launch_bkt_splitters(c->items[0], c->items[1], c->depth_skip ? c->dstats : nullptr, n,
                                          part ? c->nlive : nullptr, B,
                                          c->bkt_split + (size_t)c->bkt_par * gsr::kMaxBuckets, c->stream));
        c->bkt_B = B;
        c->bkt_scene = c->pre_scene;
    }
    return GSR_OK;
}

// Depth split, key mode, phase B: the far part [nlive, n) sorted on its own (its own
// pass plan), every kernel returning at once when phase A saturated every block.
static int far_sort_locked(gsr_context* c) {
    const uint32_t n = (uint32_t)c->n;
    const int di = c->depth_items ? c->depth_items : (c->n < (int64_t(4) << 20) ? 8 : 16);
    int gd = groups_for(c->n, 256 * di);
    if (c->depth_groups) gd = std::min(gd, c->depth_groups);
    // the pass budget follows the near sorts (phase A's column scan reports them, and
    // their key range can be far narrower); the far keys get at least three passes
    // (keys below 2^24, depths under 16.7), so a phase B is rarely short of passes
    const int launch = c->depth_skip ? std::max(3, std::min(4, c->depth_budget)) : 4;
    c->far_launched = launch;
    // the summed-area table of the tiles phase A left unsaturated; pass 0 reads the whole
    // preprocess order and keeps the items with keys at or above the frame's threshold
    // whose rect touches such a tile, writing them from position nlive (count in nfar);
    // the later passes sort [nlive, nlive + nfar)
    HIP_TRY(gsr::launch_split_sat(c->bflag, c->fr.tiles_x, c->fr.tiles_y, c->sat, c->gate, c->stream));
    const gsr::SortFilter far{2, c->kcut_frame, c->nfar, nullptr, c->sat, c->fr.tiles_x + 1, nullptr};
    const gsr::SortFilter rest{0, nullptr, nullptr, nullptr, nullptr, 0, c->nfar};
    for (int p = 0; p < launch; p++)
        HIP_TRY(gsr::launch_radix_pass(p == 0 ? c->src_items : c->items[p & 1], c->items[(p + 1) & 1], nullptr, n,
                                       32 + 8 * p, 8, gd, di, c->hist, c->totals, nullptr, c->stream,
                                       c->depth_skip ? c->dstats_far : nullptr, p,
                                       reinterpret_cast<const uint32_t*>(c->rect), p == 0 ? 1 : 0, pay_buf(c, 0),
                                       pay_buf(c, 1), rank_atomic_on(c), c->nlive, c->gate, p == 0 ? &far : &rest));
    return GSR_OK;
}

// The far Gaussians' records, when the preprocess wrote only the near ones (key mode):
// gated = phase B (returns at once when phase A saturated every block), else always.
static int far_records_locked(gsr_context* c, bool gated) {
    if (!c->records_partial) return GSR_OK;
    const gsr::RecSplit rsp{2, nullptr, c->kcut_frame, gated ? c->gate : nullptr};
    HIP_TRY(gsr::launch_preprocess(c->pre_arrays, c->pre_stride, c->n, c->fr, c->rec, c->items[0], c->rect,
                                   c->rect_packed, c->pre_layout == GSR_LAYOUT_SCENE_BLOCK_4D,
                                   c->pre_layout == GSR_LAYOUT_SCENE_BLOCK_SH3, c->time, c->stream, nullptr, &rsp));
    if (!gated) c->records_partial = false;
    return GSR_OK;
}

// Row pass, then column pass (gsr_kernels.hip "tile binning") over the depth-order
// positions [base, base + count): tile lists in pair_vals(c, 1), ranges.  gate_mode:
// 0 plain; 1 = depth split phase A (clears the gate); 2 = phase B (every kernel returns
// at once when the gate is 0).
// rs (nullable): the depth split's device-side ranges and threshold update; far: the
// positions were sorted by far_sort_locked (its pass plan and pass count apply).
static int bin_locked(gsr_context* c, uint32_t base, uint32_t count, int gate_mode, bool marks,
                      const gsr::RowSplit* rs = nullptr, bool far = false) {
    const uint32_t cap = (uint32_t)c->p_cap;
    if (int rc = ensure_cbins(c)) return rc;
    auto* row_pairs = reinterpret_cast<unsigned long long*>(c->binmeta);
    auto* row_items = reinterpret_cast<uint32_t*>(c->binmeta + 256);
    // key mode, phase A: about 2 x the split point's items (the count is on the device)
    const int64_t est = rs && rs->cut_mode == 1 ? std::min<int64_t>(count, std::max<int64_t>(2 * (int64_t)rs->na, 65536))
                                                : (int64_t)count;
    // Sources per row-pass chunk (rounded up to a multiple of 1,024, the chunks capped at
    // 4,096): 1,024, and 3,072 for a whole-order pass above 2M Gaussians (config 3 orbit, big
    // buckets: the row pass 72.8 -> 65.8 us, the count and scan pay per chunk and the scatter
    // takes 3,072 sources as well as ~1,200; 4,096: 68.7, profiles/r06o_kt_row_chunk_c3.txt).
    // GSR_ROW_CHUNK forces one size (A/B).
    static const int64_t row_chunk_env = [] {
        const char* e = std::getenv("GSR_ROW_CHUNK");
        return e ? std::max<int64_t>(1024, std::atoll(e)) : (int64_t)0;
    }();
    const int64_t row_chunk = row_chunk_env ? row_chunk_env : (!rs && est > kBucketSortMaxN ? 3072 : 1024);
    const int gb = std::min(groups_for(est, row_chunk), gsr::kMaxSortGroups / 2);
    // (a bucket-sorted frame has no pass plan: its order is in items[0], its rects in pay_buf 0)
    uint32_t* dst = c->depth_skip && !(c->last_bds && !far) ? (far ? c->dstats_far : c->dstats) : nullptr;
    // after a bucket-sorted plain frame the buckets are the row chunks and their counts exist
    const bool fused = c->bkt_rows_fused && gate_mode == 0 && base == 0 && !rs && !far && count == (uint32_t)c->n;
    c->bkt_rows_fused = false;
    const uint32_t* cstart = fused ? c->totals + c->bkt_B : nullptr;
    HIP_TRY(gsr::launch_bin_rows(c->items[0], c->items[1], dst, count, pay_buf(c, 0),
                                 pay_buf(c, 1), fused ? c->bkt_B : gb,
                                 c->hist, row_items, row_pairs, cap, c->fr.tiles_y, c->pairs[0], c->bin_row_items,
                                 c->stream, c->spans_frame ? c->spans : nullptr, rank_atomic_on(c), base,
                                 gate_mode ? c->gate : nullptr, gate_mode, rs && rs->cut_mode ? c->nlive : nullptr,
                                 rs, cstart));
    if (marks) mark(c, GSR_STAGE_TILE_SORT);
    // column-pass workgroups: ~one 2048-item chunk each (config 3: 2048-4096 groups 12 us
    // faster than 1024; config 2: 1024 best, profiles/r02_ab_col_groups.txt)
    const int gcol = c->bin_col_groups ? c->bin_col_groups
                                       : (int)std::min<int64_t>(4096, std::max<int64_t>(1024, c->n / 1024));
    HIP_TRY(gsr::launch_bin_cols(c->pairs[0], row_items, row_pairs, c->cbins, gcol, cap,
                                 c->fr.tiles_x, c->fr.tiles_y, pair_vals(c, 1), c->ranges, c->stats,
                                 c->hstats_dev, c->bin_col_items, c->stream,
                                 dst, far ? c->far_launched : c->passes_launched, rank_atomic_on(c),
                                 gate_mode == 2 ? c->gate : nullptr, c->fstatus, col_chunk_for(c)));
    c->pair_buf = 1;
    return GSR_OK;
}

// allow_split: the caller blends right after (gsr_render, gsr_render_path), so the
// depth split may apply (the stage API gsr_sort / gsr_blend keeps one phase).
static int sort_locked(gsr_context* c, bool allow_split) {
    if (!c->have_pre) return set_err(GSR_E_ARG, "gsr_sort before gsr_preprocess");
    const uint32_t n = (uint32_t)c->n;
    const bool bin = c->rect_packed;   // the path gsr_preprocess chose (its rect format)
    c->last_binned = bin;
    // depth split for this frame (gsr_render / gsr_render_path on the binning path):
    // count mode sorts the whole order and phase A bins its nearest na positions; key
    // mode (a threshold from an earlier split frame exists) partitions by the threshold
    // and sorts only the near part, which phase A bins
    const uint32_t na = (uint32_t)std::max<int64_t>(1, ((int64_t)n * c->split_pm + 999) / 1000);
    const bool split = bin && allow_split && split_enabled(c, c->n) && na < n;
    if (c->split_key && !split) {   // preprocessed for key mode: sort every visible item instead
        c->split_key = false;
        c->compact_frame = true;
    }
    if ((c->compact_frame || c->bds_frame) && !bin) {   // knobs changed since gsr_preprocess
        HIP_TRY(hipMemcpyAsync(c->items[0], c->pre_out, (size_t)n * 8, hipMemcpyDeviceToDevice, c->stream));
        c->compact_frame = false;
        c->bds_frame = false;
    }
    const bool key = split && c->split_key;
    if (!key) {   // a frame preprocessed for key mode that is not split that way: all records
        if (int rc = far_records_locked(c, false)) return rc;
    }
    // ---- stable depth sort of (key << 32 | index), 4 x 8 bits; for the binning
    // path the passes carry the rects, depth-ordered at the end (pay_buf) ----
    mark(c, GSR_STAGE_DEPTH_SORT);
    if (int rc = depth_sort_locked(c, bin, bin && !split)) return rc;
    // result in items[passes run & 1] (device-side plan; emission picks it)
    if (bin) {
        // depth split: phase A bins the near part (blend_locked blends it, then sorts
        // and bins the rest where needed)
        c->split_frame = split;
        c->split_rebin = false;
        c->frame_key = key;
        // speculate only when the camera is the one the threshold came from (a moving camera
        // would leave blocks unsaturated and cost a re-render)
        const bool same_view = std::memcmp(c->split_view, c->fr.V, sizeof c->fr.V) == 0 &&
                               std::memcmp(c->split_view + 16, c->fr.P, sizeof c->fr.P) == 0;
        // (and only with completion events on: a captured graph would bake "no phase B"
        // into every replay)
        c->frame_spec = split && key && c->split_spec && same_view && c->completion_events;
        if (split) {
            std::memcpy(c->split_view, c->fr.V, sizeof c->fr.V);
            std::memcpy(c->split_view + 16, c->fr.P, sizeof c->fr.P);
        }
        mark(c, GSR_STAGE_EMIT);
        if (split) {
            if (int rc = ensure_split(c)) return rc;
            c->split_na = na;
            const gsr::RowSplit rs{key ? 1 : 0, na, nullptr};
            if (int rc = bin_locked(c, 0, key ? n : na, 1, true, &rs)) return rc;
        } else {
            if (int rc = bin_locked(c, 0, n, 0, true)) return rc;
        }
        mark(c, GSR_STAGE_RANGES);
        c->have_sort = true;
        return GSR_OK;
    }
    // ---- pair emission in depth order (srect staged in the free items buffer) ----
    mark(c, GSR_STAGE_EMIT);
    const int ge = groups_for(c->n, 1024);
    const bool key16 = c->ntiles <= 65536;
    HIP_TRY(gsr::launch_emit(c->items[0], c->items[1], c->depth_skip ? c->dstats : nullptr, n, c->rect, ge, c->wg,
                             c->stats, c->hstats_dev, (uint32_t)c->p_cap, c->fr.tiles_x, c->fr.tiles_y,
                             pair_keys(c, 0), key16, pair_vals(c, 0), c->ranges, c->stream, c->fstatus));
    // ---- stable key-value tile sort ----
    mark(c, GSR_STAGE_TILE_SORT);
    const int tbits = std::max(1, ceil_log2(c->ntiles));
    int gp = groups_for(c->p_cap, 256 * c->tile_items);
    if (c->tile_groups) gp = std::min(gp, c->tile_groups);
    int cur = 0;
    // digits split evenly over the passes (13 bits: 7 + 6, not 8 + 5): longer
    // digit runs per sorted tile of items, so the scattered stores coalesce better
    const int tpasses = (tbits + 7) / 8;
    const int tdig = c->tile_split_even ? (tbits + tpasses - 1) / tpasses : 8;
    for (int sh = 0; sh < tbits; sh += tdig) {
        const int bits = std::min(tdig, tbits - sh);
        const bool last = sh + tdig >= tbits;    // final pass: values only + tile ranges
        HIP_TRY(gsr::launch_kv_pass(pair_keys(c, cur), pair_vals(c, cur), last ? nullptr : pair_keys(c, cur ^ 1),
                                    pair_vals(c, cur ^ 1), key16, &c->stats[0].pairs_eff, sh, bits, gp,
                                    c->tile_items, c->hist, c->totals, last ? c->ranges : nullptr, c->stream));
        cur ^= 1;
    }
    c->pair_buf = cur;
    mark(c, GSR_STAGE_RANGES);
    c->have_sort = true;
    return GSR_OK;
}

static int blend_locked(gsr_context* c, float* d_out) {
    if (!c->have_sort) return set_err(GSR_E_ARG, "gsr_blend before gsr_sort");
    if (!d_out) return set_err(GSR_E_ARG, "null output");
    mark(c, GSR_STAGE_BLEND);
    if (c->diagnostics) {
        // counters (16) and the per-pixel take map, or, for the timestamp schedule,
        // 2 stamps per wave
        const int64_t need = c->blend_variant == 3 ? 12 * (int64_t)c->ntiles + 64   // >= 2 x the padded grid
                                                   : 16 + (int64_t)c->fr.W * c->fr.H;
        if (c->consumed_cap < need) {
            if (int rc = realloc_dev(&c->consumed, (size_t)need)) return rc;
            c->consumed_cap = need;
        }
        HIP_TRY(hipMemsetAsync(c->consumed, 0, (size_t)need * sizeof(unsigned long long), c->stream));
    }
    if (c->split_frame) {
        // depth split: blend phase A (saving the blocks it leaves unsaturated), bin the
        // rest of the depth order, resume those blocks; phase B's kernels return at once
        // on the device when phase A saturated every block
        const uint32_t n = (uint32_t)c->n;
        const bool key = c->frame_key;
        if (key && c->blend_variant == 3)
            return set_err(GSR_E_ARG, "gsr_blend: blend knobs changed after a depth-split frame; render it again");
        const gsr::RowSplit ra{key ? 1 : 0, c->split_na, nullptr};
        if (c->split_rebin && c->blend_variant != 3) {
            if (int rc = bin_locked(c, 0, key ? n : c->split_na, 1, false, &ra)) return rc;
        }
        if (c->blend_variant != 3) {
            // phase A; its workgroup 0 also sets the next frame's threshold from the near
            // depth order (key mode: the near part; count mode: the whole order)
            const bool spec = c->frame_spec;
            const gsr::SplitCut cut{c->items[0], c->items[1], c->depth_skip && !c->last_bds ? c->dstats : nullptr,
                                    key ? c->nlive : nullptr, n, c->split_na, c->split_rebin ? nullptr : c->kcut};
            gsr::BlendSplit a{1, c->tbuf, c->bflag, c->gate, nullptr, spec ? c->hstats_dev : nullptr, cut, 0u,
                              spec ? c->fstatus : nullptr};
            HIP_TRY(gsr::launch_blend(pair_vals(c, c->pair_buf), c->ranges, c->rec, c->fr, d_out,
                                      c->diagnostics ? c->consumed : nullptr, false, c->blend_band_tiles, 0,
                                      c->stream, &a));
            c->split_key_ready = true;
            mark(c, GSR_STAGE_RESUME);
            if (!spec) {
                // phase B: (key mode) sort the far part, then bin the rest of the order
                const gsr::RowSplit rb{key ? 2 : 0, c->split_na, key ? c->nfar : nullptr};
                if (key && !c->split_rebin) {
                    if (int rc = far_sort_locked(c)) return rc;
                    if (int rc = far_records_locked(c, true)) return rc;
                }
                if (int rc = bin_locked(c, key ? 0 : c->split_na, key ? n : n - c->split_na, 2, false, &rb, key))
                    return rc;
                // (cut: only the near count and the split point, for the published tag)
                const gsr::SplitCut bcut{nullptr, nullptr, nullptr, key ? c->nlive : nullptr, n, c->split_na, nullptr};
                gsr::BlendSplit b{2, c->tbuf, c->bflag, c->gate, c->hstats_dev, nullptr, bcut, split_tag(c),
                                  nullptr};
                HIP_TRY(gsr::launch_blend(pair_vals(c, c->pair_buf), c->ranges, c->rec, c->fr, d_out,
                                          c->diagnostics ? c->consumed : nullptr, false, c->blend_band_tiles, 0,
                                          c->stream, &b));
                c->split_seen = true;
            }
            c->split_rebin = true;
        } else {
            // knobs changed since the sort: bin the whole depth order again, one phase
            if (int rc = bin_locked(c, 0, (uint32_t)c->n, 0, false)) return rc;
            c->split_frame = false;
            HIP_TRY(gsr::launch_blend(pair_vals(c, c->pair_buf), c->ranges, c->rec, c->fr, d_out,
                                      c->diagnostics ? c->consumed : nullptr, c->blend_variant == 3,
                                      c->blend_band_tiles, c->blend_exp, c->stream));
        }
    } else {
        HIP_TRY(gsr::launch_blend(pair_vals(c, c->pair_buf), c->ranges, c->rec, c->fr, d_out,
                                  c->diagnostics ? c->consumed : nullptr, c->blend_variant == 3,
                                  c->blend_band_tiles, c->blend_exp, c->stream));
    }
    mark(c, GSR_NUM_STAGES);
    if (c->timing && c->timing_now) c->ev_frames.push_back(c->cur);
    c->cur = FrameEvents{};
    // At most one completion event in flight: while the last one is unread, later
    // frames skip the record (~3 us each). The overflow stats are sticky, so reading
    // them when that older frame completes still sees every overflow so far, and
    // gsr_sync drains the stream before it reads them.
    if (!c->pending && c->completion_events) {
        HIP_TRY(hipEventRecord(c->done_ev, c->stream));
        c->pending = true;
    }
    return GSR_OK;
}

extern "C" int gsr_preprocess(gsr_context* c, const void* scene, int layout, int64_t n, const gsr_camera* cam,
                              int W, int H, int nx, int ny, int ws, int hs, float k, void* stream) {
    if (!c) return set_err(GSR_E_ARG, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    return preprocess_locked(c, scene, layout, n, cam, W, H, nx, ny, ws, hs, k, stream);
}

extern "C" int gsr_sort(gsr_context* c, void* stream) {
    if (!c) return set_err(GSR_E_ARG, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    c->stream = static_cast<hipStream_t>(stream);
    return sort_locked(c, false);
}

extern "C" int gsr_blend(gsr_context* c, float* d_out, void* stream) {
    if (!c) return set_err(GSR_E_ARG, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    c->stream = static_cast<hipStream_t>(stream);
    return blend_locked(c, d_out);
}

extern "C" int gsr_render(gsr_context* c, const void* scene, int layout, int64_t n, const gsr_camera* cam, int W,
                          int H, int nx, int ny, int ws, int hs, float k, float* d_out, void* stream) {
    if (!c) return set_err(GSR_E_ARG, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    int rc = preprocess_locked(c, scene, layout, n, cam, W, H, nx, ny, ws, hs, k, stream);
    if (rc != GSR_OK && rc != GSR_E_OVERFLOW) return rc;
    if (int r2 = sort_locked(c, true)) return r2;
    if (int r3 = blend_locked(c, d_out)) return r3;
    return rc;
}

// ------------------------------------------------------------------ frames in flight

namespace {

// Everything that selects kernels or schedules (all settings are bit-identical);
// diagnostics and timing stay on lane 0 only.
void copy_settings(gsr_context* d, const gsr_context* s) {
    d->tile_items = s->tile_items;
    d->depth_items = s->depth_items;
    d->bucket_sort = s->bucket_sort;
    d->fuse_rows = s->fuse_rows;
    d->col_chunk = s->col_chunk;
    d->tile_groups = s->tile_groups;
    d->tile_split_even = s->tile_split_even;
    d->depth_skip = s->depth_skip;
    d->depth_groups = s->depth_groups;
    d->tile_binning = s->tile_binning;
    d->bin_row_items = s->bin_row_items;
    d->bin_col_items = s->bin_col_items;
    d->tile_spans = s->tile_spans;
    d->bin_col_groups = s->bin_col_groups;
    d->blend_band_tiles = s->blend_band_tiles;
    d->blend_exp = s->blend_exp;
    d->depth_split = s->depth_split;   // the split point adapts per lane (set at creation and by the knob)
    d->completion_events = s->completion_events;
    d->depth_compact = s->depth_compact;
    d->rank_atomic = s->rank_atomic;
}

// Lanes 1..F-1: child contexts, streams and events, created once and kept.
int ensure_lanes(gsr_context* c, int F) {
    if (!c->fork_ev) HIP_TRY(hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming));
    while ((int)c->lanes.size() < F - 1) {
        gsr_context* l = new gsr_context();
        l->inflight = 1;
        l->split_pm = c->split_pm;
        l->split_floor = c->split_floor;
        hipStream_t s = nullptr;
        hipEvent_t e = nullptr;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            if (s) (void)hipStreamDestroy(s);
            gsr_destroy(l);
            return set_err(GSR_E_HIP, "frames in flight: stream/event creation failed");
        }
        c->lanes.push_back(l);
        c->lane_streams.push_back(s);
        c->join_evs.push_back(e);
    }
    while ((int)c->alias_evs.size() < F) {
        hipEvent_t e = nullptr;
        HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->alias_evs.push_back(e);
    }
    for (int l = 0; l < F - 1; l++) copy_settings(c->lanes[l], c);
    return GSR_OK;
}

int render_one_locked(gsr_context* c, const void* scene, int layout, int64_t n, const gsr_camera* cam, int W,
                      int H, int nx, int ny, int ws, int hs, float k, float* d_out, hipStream_t s) {
    int rc = preprocess_locked(c, scene, layout, n, cam, W, H, nx, ny, ws, hs, k, s);
    if (rc != GSR_OK && rc != GSR_E_OVERFLOW) return rc;
    if (int r2 = sort_locked(c, true)) return r2;
    if (int r3 = blend_locked(c, d_out)) return r3;
    return rc;
}

}  // namespace

extern "C" int gsr_set_frames_in_flight(gsr_context* c, int frames) {
    if (!c || frames < 1 || frames > GSR_MAX_FRAMES_IN_FLIGHT)
        return set_err(GSR_E_ARG, "gsr_set_frames_in_flight: frames must be 1..%d", GSR_MAX_FRAMES_IN_FLIGHT);
    std::lock_guard<std::mutex> lk(c->mu);
    c->inflight = frames;
    return GSR_OK;
}

extern "C" int gsr_frames_in_flight(gsr_context* c) {
    if (!c) return set_err(GSR_E_ARG, "null context");
    return c->inflight;
}

extern "C" int gsr_render_path(gsr_context* c, const void* scene, int layout, int64_t n, const gsr_camera* cams,
                               const float* times, int nframes, int W, int H, int nx, int ny, int ws, int hs,
                               float k, float* const* d_outs, void* stream) {
    return gsr_render_path_ex(c, scene, layout, n, cams, times, nframes, W, H, nx, ny, ws, hs, k, d_outs, stream,
                              nullptr, nullptr, 0);
}

extern "C" int gsr_render_path_ex(gsr_context* c, const void* scene, int layout, int64_t n, const gsr_camera* cams,
                                  const float* times, int nframes, int W, int H, int nx, int ny, int ws, int hs,
                                  float k, float* const* d_outs, void* stream, void* const* frame_events,
                                  void* const* wait_events, int flags) {
    return gsr_render_path_status(c, scene, layout, n, cams, times, nframes, W, H, nx, ny, ws, hs, k, d_outs, stream,
                                  frame_events, wait_events, flags, nullptr);
}

extern "C" int gsr_render_path_status(gsr_context* c, const void* scene, int layout, int64_t n,
                                      const gsr_camera* cams, const float* times, int nframes, int W, int H, int nx,
                                      int ny, int ws, int hs, float k, float* const* d_outs, void* stream,
                                      void* const* frame_events, void* const* wait_events, int flags,
                                      uint32_t* const* d_status) {
    if (!c) return set_err(GSR_E_ARG, "null context");
    if (flags & ~(GSR_PATH_NO_JOIN | GSR_PATH_NO_FORK))
        return set_err(GSR_E_ARG, "gsr_render_path_ex: unknown flags 0x%x", flags);
    if (nframes < 0 || (nframes > 0 && (!cams || !d_outs)))
        return set_err(GSR_E_ARG, "gsr_render_path: bad frame arrays");
    for (int i = 0; i < nframes; i++)
        if (!d_outs[i]) return set_err(GSR_E_ARG, "gsr_render_path: null output for frame %d", i);
    std::lock_guard<std::mutex> lk(c->mu);
    if (nframes == 0) return GSR_OK;
    const hipStream_t S = static_cast<hipStream_t>(stream);
    const int F = std::max(1, std::min(c->inflight, nframes));
    if (int rc = ensure_lanes(c, F)) return rc;
    if (int rc = ensure_static(c)) return rc;
    // children start at the parent's pair high-water mark (each still grows on its own overflow)
    for (int l = 0; l < F - 1; l++) {
        gsr_context* ch = c->lanes[l];
        if (int rc = ensure_static(ch)) return rc;
        if (ch->p_cap < c->p_cap && c->p_cap > 0) {
            if (int rc = ensure_n(ch, std::max<int64_t>(n, 1))) return rc;
            if (int rc = ensure_pairs(ch, c->p_cap)) return rc;
        }
    }
    // fork: every lane starts after the work already queued on the caller's stream
    if (F > 1 && !(flags & GSR_PATH_NO_FORK)) {
        HIP_TRY(hipEventRecord(c->fork_ev, S));
        for (int l = 0; l < F - 1; l++) HIP_TRY(hipStreamWaitEvent(c->lane_streams[l], c->fork_ev, 0));
    }
    // Output reuse: a frame writing a buffer that an earlier frame of this call wrote on
    // ANOTHER lane must wait for that writer, however far back it ran (lanes are not
    // ordered with each other).  prev[i] = the last earlier frame writing d_outs[i];
    // a writer whose buffer is reused on another lane records its lane's event after
    // it, and the reuser waits on that event's latest record (at or after the writer
    // on the same stream, so the wait covers it).
    std::vector<int> prev(nframes, -1);
    std::vector<char> record(nframes, 0);
    {
        std::unordered_map<const float*, int> last;
        last.reserve(2 * (size_t)nframes);
        for (int i = 0; i < nframes; i++) {
            auto it = last.find(d_outs[i]);
            if (it != last.end()) {
                prev[i] = it->second;
                if (it->second % F != i % F) record[it->second] = 1;
            }
            last[d_outs[i]] = i;
        }
    }
    int result = GSR_OK;
    int err = GSR_OK;   // the first error; the frames queued before it are still joined below
    const float t_saved = c->time;
    auto hip_fail = [&](hipError_t e, const char* what) {
        return set_err(GSR_E_HIP, "gsr_render_path: %s: %s", what, hipGetErrorString(e));
    };
    for (int i = 0; i < nframes && err == GSR_OK; i++) {
        const int lane = i % F;
        gsr_context* lc = lane == 0 ? c : c->lanes[lane - 1];
        const hipStream_t ls = lane == 0 ? S : c->lane_streams[lane - 1];
        if (prev[i] >= 0 && prev[i] % F != lane) {
            if (hipError_t e = hipStreamWaitEvent(ls, c->alias_evs[prev[i] % F], 0)) {
                err = hip_fail(e, "output reuse wait");
                break;
            }
        }
        if (wait_events && wait_events[i]) {
            if (hipError_t e = hipStreamWaitEvent(ls, static_cast<hipEvent_t>(wait_events[i]), 0)) {
                err = hip_fail(e, "wait event");
                break;
            }
        }
        if (times) lc->time = times[i];
        else lc->time = t_saved;
        // the frame's validity word is the lane's only while its frame is queued: the guard
        // clears it on every exit, so a later gsr_render on this context (or an erroring
        // frame's early return) never writes through a pointer the caller may have freed
        struct StatusScope {
            gsr_context* lc;
            ~StatusScope() { lc->fstatus = nullptr; }
        } status_scope{lc};
        lc->fstatus = d_status ? d_status[i] : nullptr;
        int rc;
        if (c->fail_frame > 0 && i == c->fail_frame) {   // GSR_TUNE_FAIL_FRAME (test hook, once)
            c->fail_frame = 0;
            rc = set_err(GSR_E_ARG, "gsr_render_path: frame %d failed (GSR_TUNE_FAIL_FRAME test hook)", i);
        } else {
            rc = render_one_locked(lc, scene, layout, n, &cams[i], W, H, nx, ny, ws, hs, k, d_outs[i], ls);
        }
        if (rc == GSR_E_OVERFLOW) {
            result = GSR_E_OVERFLOW;
        } else if (rc != GSR_OK) {
            err = rc;
            break;
        }
        if (record[i]) {
            if (hipError_t e = hipEventRecord(c->alias_evs[lane], ls)) err = hip_fail(e, "output reuse event");
        }
        if (err == GSR_OK && frame_events && frame_events[i]) {
            if (hipError_t e = hipEventRecord(static_cast<hipEvent_t>(frame_events[i]), ls))
                err = hip_fail(e, "frame event");
        }
    }
    // on every exit after the fork, errors included (render.cu:914-923 reports a failed
    // step and the caller's frame loop goes on): the time knob is restored, the caller's
    // stream is the context's again, and work queued on it afterwards sees every frame the
    // lanes took (a caller that frees or reuses an output after an error must not race a
    // lane still writing it).  A join failure after an earlier error keeps the first message.
    c->time = t_saved;
    c->stream = S;
    for (int l = 0; l < F - 1 && l + 1 < nframes && !(flags & GSR_PATH_NO_JOIN); l++) {
        hipError_t e = hipEventRecord(c->join_evs[l], c->lane_streams[l]);
        if (e == hipSuccess) e = hipStreamWaitEvent(S, c->join_evs[l], 0);
        if (e != hipSuccess && err == GSR_OK) err = hip_fail(e, "join");
    }
    return err != GSR_OK ? err : result;
}

extern "C" int gsr_sync(gsr_context* c) {
    if (!c) return set_err(GSR_E_ARG, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    int result = GSR_OK;
    for (size_t l = 0; l < c->lanes.size(); l++) {
        gsr_context* lc = c->lanes[l];
        HIP_TRY(hipStreamSynchronize(c->lane_streams[l]));
        const int rc = check_overflow(lc, true);
        if (rc != GSR_OK && rc != GSR_E_OVERFLOW) return rc;
        if (lc->overflow_seen) result = GSR_E_OVERFLOW;
        lc->overflow_seen = false;
    }
    if (c->stream || c->pending) HIP_TRY(hipStreamSynchronize(c->stream));
    const int rc = check_overflow(c, true);
    if (rc != GSR_OK && rc != GSR_E_OVERFLOW) return rc;
    if (c->overflow_seen) result = GSR_E_OVERFLOW;
    c->overflow_seen = false;
    if (result == GSR_E_OVERFLOW && rc == GSR_OK)
        set_err(GSR_E_OVERFLOW, "a frame since the last gsr_sync was incomplete (reported earlier); re-render");
    return result;
}

// ------------------------------------------------------------------ readback

extern "C" int64_t gsr_pair_count(gsr_context* c) {
    if (!c || !c->stats) return -1;
    std::lock_guard<std::mutex> lk(c->mu);
    Stats s{};
    if (hipStreamSynchronize(c->stream) != hipSuccess) return -1;
    if (hipMemcpy(&s, c->stats, sizeof s, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return (int64_t)s.pairs_total;
}

extern "C" int64_t gsr_row_item_count(gsr_context* c) {
    if (!c || !c->binmeta) return -1;
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->have_sort || !c->last_binned) return -1;
    uint32_t rows[256];
    if (hipStreamSynchronize(c->stream) != hipSuccess) return -1;
    if (hipMemcpy(rows, c->binmeta + 256, sizeof rows, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    int64_t total = 0;
    for (uint32_t v : rows) total += v;
    return total;
}

static int depth_passes_locked(gsr_context* c, int* passes);
static int sorted_items_locked(gsr_context* c, uint64_t* host, int64_t n);

// The device record's fourth word is the blend's cull word (gsr_kernels.hip
// cull_word); the readback layout's fourth word {tile x range, tile y range,
// tile count, depth key} is rebuilt from the preprocess tile rects (index order)
// and the frame's depth items: (key << 32 | index) in index order right after
// preprocess or in a per-tile-order frame, depth-sorted after a global sort.
extern "C" int gsr_read_splats(gsr_context* c, void* host, int64_t n) {
    if (!c || !host || n < 0 || n > c->n) return set_err(GSR_E_ARG, "gsr_read_splats: bad argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (!n) return GSR_OK;
    if (!c->have_pre) return set_err(GSR_E_ARG, "gsr_read_splats: no preprocessed frame");
    if (c->records_partial) {   // key-mode split frame: the far Gaussians' records first
        if (int rc = far_records_locked(c, false)) return rc;
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    HIP_TRY(hipMemcpy(host, c->rec, (size_t)n * GSR_SPLAT_RECORD_BYTES, hipMemcpyDeviceToHost));
    std::vector<uint64_t> rect((size_t)n), items((size_t)c->n);
    if (c->rect_packed) {   // 4-B rects (gsr_kernels.hip pack_rect): tx0 | tx1 << 8 | ty0 << 16 | ty1 << 24
        std::vector<uint32_t> p((size_t)n);
        HIP_TRY(hipMemcpy(p.data(), c->rect, (size_t)n * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < (size_t)n; i++)
            rect[i] = (uint64_t)(p[i] & 0xffu) | ((uint64_t)((p[i] >> 8) & 0xffu) << 16) |
                      ((uint64_t)((p[i] >> 16) & 0xffu) << 32) | ((uint64_t)(p[i] >> 24) << 48);
    } else {
        HIP_TRY(hipMemcpy(rect.data(), c->rect, (size_t)n * 8, hipMemcpyDeviceToHost));
    }
    if (c->have_sort && c->last_split_key) {
        // a key-mode split frame: its preprocess order holds every item's key
        HIP_TRY(hipMemcpy(items.data(), c->src_items, (size_t)c->n * 8, hipMemcpyDeviceToHost));
    } else if (c->have_sort) {
        if (int rc = sorted_items_locked(c, items.data(), c->n)) return rc;
    } else {   // preprocess order (items[1] for the live partition, src_items for a key-mode split)
        HIP_TRY(hipMemcpy(items.data(), c->pre_out ? c->pre_out : c->items[0], (size_t)c->n * 8,
                          hipMemcpyDeviceToHost));
    }
    auto* w = static_cast<uint32_t*>(host);
    for (uint64_t it : items) {
        const uint32_t i = (uint32_t)it;
        if (i < (uint64_t)n) w[(size_t)i * 16 + 15] = (uint32_t)(it >> 32);
    }
    for (int64_t i = 0; i < n; i++) {
        const uint64_t r = rect[(size_t)i];
        const int tx0 = (int)(r & 0xffffu), tx1 = (int)((r >> 16) & 0xffffu);
        const int ty0 = (int)((r >> 32) & 0xffffu), ty1 = (int)(r >> 48);
        uint32_t* q = w + (size_t)i * 16;
        // the device keeps the centre pixel as the float the blend uses; the
        // readback layout's int32 (exact for |px| <= 2^24, saturating like gsr_f2i_sat)
        for (int k = 8; k < 10; k++) {
            float f;
            std::memcpy(&f, q + k, 4);
            const int32_t v = f >= 2147483648.0f ? INT32_MAX : (f < -2147483648.0f ? INT32_MIN : (int32_t)f);
            std::memcpy(q + k, &v, 4);
        }
        q[12] = (uint32_t)r;
        q[13] = (uint32_t)(r >> 32);
        q[14] = (uint32_t)((tx1 - tx0 + 1) * (ty1 - ty0 + 1));
    }
    return GSR_OK;
}

static int depth_passes_locked(gsr_context* c, int* passes) {
    *passes = 4;
    if (c->last_bds) {   // bucket-sorted: no LSD passes, the order is in items[0]
        *passes = 0;
        return GSR_OK;
    }
    if (!c->depth_skip) return GSR_OK;
    uint32_t st[4];   // same plan as the kernels (gsr_kernels.hip depth_pass_skipped)
    HIP_TRY(hipMemcpy(st, c->dstats, sizeof st, hipMemcpyDeviceToHost));
    int p = 1;
    for (; p < 4; ++p) {
        const bool skip = st[3] == 0u || ((~st[0] >> (8 * p)) == (st[1] >> (8 * p)) && !((st[2] >> p) & 1u));
        if (skip) break;
    }
    *passes = p;
    return GSR_OK;
}

// First n items of the last globally sorted frame's depth order (stream drained).
static int sorted_items_locked(gsr_context* c, uint64_t* host, int64_t n) {
    if (c->last_split_key)
        return set_err(GSR_E_ARG, "depth order unavailable: the last frame was depth-split by a threshold (its far "
                                  "part is sorted only when phase B runs); set GSR_TUNE_DEPTH_SPLIT to 0");
    int p = 4;
    if (int rc = depth_passes_locked(c, &p)) return rc;
    int64_t head = n;
    if (c->last_compact) {   // sorted visible prefix in items[p & 1], culled tail (index order) in items[0]
        uint32_t live = 0;
        HIP_TRY(hipMemcpy(&live, c->nlive, sizeof live, hipMemcpyDeviceToHost));
        head = std::min<int64_t>(n, live);
        if (n > head)
            HIP_TRY(hipMemcpy(host + head, c->items[0] + head, (size_t)(n - head) * 8, hipMemcpyDeviceToHost));
    }
    if (head) HIP_TRY(hipMemcpy(host, c->items[p & 1], (size_t)head * 8, hipMemcpyDeviceToHost));
    return GSR_OK;
}

extern "C" int gsr_depth_passes(gsr_context* c) {
    if (!c || !c->have_sort) return set_err(GSR_E_ARG, "gsr_depth_passes: no sorted frame");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipStreamSynchronize(c->stream));
    int p = 4;
    if (int rc = depth_passes_locked(c, &p)) return rc;
    return p;
}

extern "C" int gsr_bucket_sizes(gsr_context* c, uint32_t* sizes, int cap) {
    if (!c || cap < 0 || (cap > 0 && !sizes)) return set_err(GSR_E_ARG, "gsr_bucket_sizes: bad argument");
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->have_sort || !c->last_bds || !c->bkt_B || !c->totals) return 0;
    HIP_TRY(hipStreamSynchronize(c->stream));
    // k_bkt_scan's bucket totals (totals[0 .. B)), which a bucket-sorted frame's later
    // kernels only read
    const int m = std::min(cap, c->bkt_B);
    if (m) HIP_TRY(hipMemcpy(sizes, c->totals, (size_t)m * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return c->bkt_B;
}

extern "C" int gsr_read_depth_order(gsr_context* c, uint64_t* host, int64_t n) {
    if (!c || !host || n < 0 || n > c->n || !c->have_sort) return set_err(GSR_E_ARG, "gsr_read_depth_order: bad argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipStreamSynchronize(c->stream));
    return sorted_items_locked(c, host, n);
}

extern "C" int64_t gsr_read_pairs(gsr_context* c, uint64_t* host, int64_t cap) {
    if (!c || !host || cap < 0 || !c->have_sort) return set_err(GSR_E_ARG, "gsr_read_pairs: bad argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipStreamSynchronize(c->stream));
    Stats s{};
    HIP_TRY(hipMemcpy(&s, c->stats, sizeof s, hipMemcpyDeviceToHost));
    const int64_t m = std::min<int64_t>(cap, s.pairs_eff);
    if (!m) return 0;
    // the sorted pairs live as values + tile ranges; rebuild (tile << 32 | index) tile by
    // tile.  Ranges ascend with the tile; with tile row spans the binning leaves unused
    // slots between rows (pairs_total counts every tile of every rect), so the listed
    // pairs are packed here and their count returned.
    std::vector<uint32_t> vals((size_t)m);
    std::vector<uint2> rg((size_t)c->ntiles);
    HIP_TRY(hipMemcpy(vals.data(), pair_vals(c, c->pair_buf), (size_t)m * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(rg.data(), c->ranges, sizeof(uint2) * rg.size(), hipMemcpyDeviceToHost));
    int64_t k = 0;
    for (int t = 0; t < c->ntiles; t++) {
        if (!rg[t].y) continue;
        for (int64_t j = ~rg[t].x; j < (int64_t)rg[t].y && j < m; j++)
            host[k++] = ((uint64_t)(uint32_t)t << 32) | vals[(size_t)j];
    }
    return k;
}

extern "C" int gsr_tile_grid(gsr_context* c, int* tx, int* ty) {
    if (!c || !tx || !ty) return set_err(GSR_E_ARG, "gsr_tile_grid: bad argument");
    *tx = c->fr.tiles_x;
    *ty = c->fr.tiles_y;
    return GSR_OK;
}

extern "C" int gsr_read_tile_ranges(gsr_context* c, uint32_t* host, int64_t nt) {
    if (!c || !host || nt < 0 || nt > c->ntiles || !c->have_sort) return set_err(GSR_E_ARG, "gsr_read_tile_ranges: bad argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (nt) HIP_TRY(hipMemcpy(host, c->ranges, (size_t)nt * 8, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < nt; i++) {         // device form {~start, end}, zero = empty
        const uint32_t x = host[2 * i], y = host[2 * i + 1];
        host[2 * i] = y ? ~x : 0u;
        host[2 * i + 1] = y;
    }
    return GSR_OK;
}

// ------------------------------------------------------------------ timing

extern "C" int gsr_set_timing(gsr_context* c, int mode) {
    return gsr_set_timing_stride(c, mode, 1);
}

extern "C" int gsr_set_timing_stride(gsr_context* c, int mode, int stride) {
    if (!c || mode < 0 || mode > 2 || stride < 1) return set_err(GSR_E_ARG, "gsr_set_timing: bad argument");
    std::lock_guard<std::mutex> lk(c->mu);
    c->timing = mode;
    c->timing_stride = stride;
    c->timing_count = 0;
    return GSR_OK;
}

extern "C" int gsr_stage_times(gsr_context* c, double* ms, int64_t* frames) {
    if (!c || !ms) return set_err(GSR_E_ARG, "gsr_stage_times: bad argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int s = 0; s < GSR_NUM_STAGES; s++) ms[s] = 0.0;
    for (auto& f : c->ev_frames) {
        // stages may be recorded out of index order (per-tile depth order runs its
        // depth stage after the binning passes): each stage lasts until the next
        // recorded boundary in TIME order
        hipEvent_t e0 = nullptr;
        for (int s = 0; s <= GSR_NUM_STAGES && !e0; s++) e0 = f.ev[s];
        float at[GSR_NUM_STAGES + 1];
        for (int s = 0; s <= GSR_NUM_STAGES; s++) {
            at[s] = -1.0f;
            if (f.ev[s] && e0 && hipEventElapsedTime(&at[s], e0, f.ev[s]) != hipSuccess) at[s] = -1.0f;
        }
        for (int s = 0; s < GSR_NUM_STAGES; s++) {
            if (!f.ev[s] || at[s] < 0.0f) continue;
            float next = -1.0f;
            for (int q = 0; q <= GSR_NUM_STAGES; q++)
                if (q != s && f.ev[q] && at[q] >= 0.0f && (at[q] > at[s] || (at[q] == at[s] && q > s)) &&
                    (next < 0.0f || at[q] < next))
                    next = at[q];
            if (next >= 0.0f) ms[s] += next - at[s];
        }
        for (auto e : f.ev)
            if (e) c->ev_pool.push_back(e);
    }
    if (frames) *frames = (int64_t)c->ev_frames.size();
    c->ev_frames.clear();
    return GSR_OK;
}

extern "C" int gsr_set_diagnostics(gsr_context* c, int on) {
    if (!c) return set_err(GSR_E_ARG, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    c->diagnostics = on != 0;
    return GSR_OK;
}

extern "C" int gsr_set_time(gsr_context* c, float t) {
    if (!c) return set_err(GSR_E_ARG, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    c->time = t;
    return GSR_OK;
}

extern "C" int gsr_get_tuning(gsr_context* c, int knob, int* value) {
    if (!c || !value) return set_err(GSR_E_ARG, "gsr_get_tuning: null argument");
    std::lock_guard<std::mutex> lk(c->mu);
    switch (knob) {
    case GSR_TUNE_BLEND_SCHEDULE: *value = c->blend_variant; break;
    case GSR_TUNE_TILE_SORT_ITEMS: *value = c->tile_items; break;
    case GSR_TUNE_DEPTH_SORT_ITEMS: *value = c->depth_items; break;
    case GSR_TUNE_TILE_SORT_GROUPS: *value = c->tile_groups; break;
    case GSR_TUNE_DEPTH_SORT_GROUPS: *value = c->depth_groups; break;
    case GSR_TUNE_TILE_SORT_SPLIT: *value = c->tile_split_even ? 1 : 0; break;
    case GSR_TUNE_DEPTH_SORT_SKIP: *value = c->depth_skip ? 1 : 0; break;
    case GSR_TUNE_TILE_BINNING: *value = c->tile_binning; break;
    case GSR_TUNE_BIN_ROW_ITEMS: *value = c->bin_row_items; break;
    case GSR_TUNE_BIN_COL_ITEMS: *value = c->bin_col_items; break;
    case GSR_TUNE_BIN_COL_GROUPS: *value = c->bin_col_groups; break;
    case GSR_TUNE_COMPLETION_EVENTS: *value = c->completion_events ? 1 : 0; break;
    case GSR_TUNE_BLEND_BAND_TILES: *value = c->blend_band_tiles; break;
    case GSR_TUNE_DEPTH_COMPACT: *value = c->depth_compact; break;
    case GSR_TUNE_TILE_SPANS: *value = c->tile_spans; break;
    case GSR_TUNE_BLEND_EXP: *value = c->blend_exp; break;
    case GSR_TUNE_DEPTH_SPLIT: *value = c->depth_split; break;
    case GSR_TUNE_DEPTH_SPLIT_PERMILLE: *value = c->split_pm; break;
    case GSR_TUNE_DEPTH_SPLIT_UNSAT: *value = c->hstats ? (int)((const volatile Stats*)c->hstats)->split_unsat : 0; break;
    case GSR_TUNE_DEPTH_SPLIT_STATE: *value = !c->split_frame ? 0 : !c->frame_key ? 1 : c->frame_spec ? 3 : 2; break;
    case GSR_TUNE_DEPTH_BUCKETS: *value = c->bucket_sort; break;
    case GSR_TUNE_BUCKET_ROWS: *value = c->fuse_rows; break;
    case GSR_TUNE_COL_CHUNK: *value = c->col_chunk; break;
    case GSR_TUNE_FAIL_FRAME: *value = c->fail_frame; break;
    case GSR_TUNE_DEPTH_BUCKETS_OVER:
    case GSR_TUNE_DEPTH_BUCKETS_WORK: {
        auto get = [&](const gsr_context* x) -> int64_t {
            if (!x->hstats) return 0;
            const volatile Stats* h = (const volatile Stats*)x->hstats;
            return knob == GSR_TUNE_DEPTH_BUCKETS_OVER ? (int64_t)h->bkt_over : (int64_t)h->bkt_over_work;
        };
        int64_t v = get(c);
        for (auto* l : c->lanes) v += get(l);
        *value = (int)std::min<int64_t>(v, INT32_MAX);
        break;
    }
    case GSR_TUNE_RANK_ATOMIC: *value = c->rank_atomic < 0 ? default_rank_atomic() : c->rank_atomic; break;
    case GSR_TUNE_RANK_ATOMIC_ACTIVE: {
        RankCheck rk;
        if (int rc = rank_check_device(&rk)) return rc;
        const int asked = c->rank_atomic < 0 ? default_rank_atomic() : c->rank_atomic;
        *value = asked > 0 && rk.state == 1 ? 1 : 0;
        break;
    }
    default: return set_err(GSR_E_ARG, "gsr_get_tuning: unknown knob");
    }
    return GSR_OK;
}

extern "C" int gsr_set_tuning(gsr_context* c, int knob, int value) {
    if (!c) return set_err(GSR_E_ARG, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    switch (knob) {
    case GSR_TUNE_BLEND_SCHEDULE:
        if (value != 0 && value != 3)
            return set_err(GSR_E_ARG, "gsr_set_tuning: blend schedule must be 0 (default) or 3 (timeline stamps)");
        c->blend_variant = value;
        return GSR_OK;
    case GSR_TUNE_TILE_SORT_ITEMS:
        if (value != 8 && value != 16) return set_err(GSR_E_ARG, "gsr_set_tuning: tile-sort items must be 8 or 16");
        c->tile_items = value;
        return GSR_OK;
    case GSR_TUNE_DEPTH_SORT_ITEMS:
        if (value != 0 && value != 4 && value != 8 && value != 16)
            return set_err(GSR_E_ARG, "gsr_set_tuning: depth-sort items must be 0, 4, 8 or 16");
        c->depth_items = value;
        return GSR_OK;
    case GSR_TUNE_TILE_BINNING:
        c->tile_binning = value != 0;
        return GSR_OK;
    case GSR_TUNE_BIN_ROW_ITEMS:
    case GSR_TUNE_BIN_COL_ITEMS:
        if (value != 4 && value != 8 && value != 16)
            return set_err(GSR_E_ARG, "gsr_set_tuning: binning items per thread must be 4, 8 or 16");
        (knob == GSR_TUNE_BIN_ROW_ITEMS ? c->bin_row_items : c->bin_col_items) = value;
        return GSR_OK;
    case GSR_TUNE_BLEND_BAND_TILES:
        if (value < 0 || value > 65536) return set_err(GSR_E_ARG, "gsr_set_tuning: blend band tiles must be 0..65536");
        c->blend_band_tiles = value;
        return GSR_OK;
    case GSR_TUNE_COMPLETION_EVENTS:
        c->completion_events = value != 0;
        return GSR_OK;
    case GSR_TUNE_BIN_COL_GROUPS:
        if (value < 0 || value > 65536) return set_err(GSR_E_ARG, "gsr_set_tuning: bad column-pass group count");
        c->bin_col_groups = value;
        return GSR_OK;
    case GSR_TUNE_DEPTH_COMPACT:
        if (value < 0 || value > 2) return set_err(GSR_E_ARG, "gsr_set_tuning: depth compaction must be 0, 1 or 2");
        c->depth_compact = value;
        return GSR_OK;
    case GSR_TUNE_DEPTH_SORT_SKIP:
        c->depth_skip = value != 0;
        return GSR_OK;
    case GSR_TUNE_TILE_SPANS:
        if (value < 0 || value > 2) return set_err(GSR_E_ARG, "gsr_set_tuning: tile spans must be 0, 1 or 2");
        c->tile_spans = value;
        return GSR_OK;
    case GSR_TUNE_TILE_SORT_SPLIT:
        c->tile_split_even = value != 0;
        return GSR_OK;
    case GSR_TUNE_BLEND_EXP:
        if (value < 0 || value > 2) return set_err(GSR_E_ARG, "gsr_set_tuning: blend exp must be 0, 1 or 2");
        c->blend_exp = value;
        return GSR_OK;
    case GSR_TUNE_DEPTH_SPLIT:
        if (value < 0 || value > 2) return set_err(GSR_E_ARG, "gsr_set_tuning: depth split must be 0, 1 or 2");
        c->depth_split = value;
        // the next split frame sorts the whole order (count mode), queues phase B
        c->split_key_ready = c->split_spec = false;
        for (auto* l : c->lanes) l->split_key_ready = l->split_spec = false;
        return GSR_OK;
    case GSR_TUNE_DEPTH_SPLIT_PERMILLE:
        if (value < 1 || value > 999) return set_err(GSR_E_ARG, "gsr_set_tuning: split point must be 1..999");
    {
        auto restart = [value](gsr_context* x) {   // a new starting point for every lane
            x->split_pm = value;
            x->split_epoch++;
            x->split_floor = 0;
            x->split_clean = 0;
            x->split_spec = false;
            x->split_key_ready = false;
        };
        restart(c);
        for (auto* l : c->lanes) restart(l);
        return GSR_OK;
    }
    case GSR_TUNE_RANK_ATOMIC:
        if (value != 0 && value != 1) return set_err(GSR_E_ARG, "gsr_set_tuning: rank path must be 0 or 1");
        c->rank_atomic = value;
        return GSR_OK;
    case GSR_TUNE_DEPTH_BUCKETS:
        if (value < 0 || value > 3) return set_err(GSR_E_ARG, "gsr_set_tuning: depth buckets must be 0..3");
        c->bucket_sort = value;
        return GSR_OK;
    case GSR_TUNE_COL_CHUNK:
        if (value != 0 && value != 1024 && value != 2048)
            return set_err(GSR_E_ARG, "gsr_set_tuning: column chunk must be 0, 1024 or 2048");
        c->col_chunk = value;
        return GSR_OK;
    case GSR_TUNE_BUCKET_ROWS:
        c->fuse_rows = value != 0;
        return GSR_OK;
    case GSR_TUNE_FAIL_FRAME:
        if (value < 0) return set_err(GSR_E_ARG, "gsr_set_tuning: fail frame must be >= 0");
        c->fail_frame = value;
        return GSR_OK;
    case GSR_TUNE_RANK_ATOMIC_ACTIVE:
    case GSR_TUNE_DEPTH_SPLIT_UNSAT:
    case GSR_TUNE_DEPTH_SPLIT_STATE:
    case GSR_TUNE_DEPTH_BUCKETS_OVER:
    case GSR_TUNE_DEPTH_BUCKETS_WORK:
        return set_err(GSR_E_ARG, "gsr_set_tuning: knob %d is read-only", knob);
    case GSR_TUNE_TILE_SORT_GROUPS:
    case GSR_TUNE_DEPTH_SORT_GROUPS:
        if (value < 0 || value > gsr::kMaxSortGroups) return set_err(GSR_E_ARG, "gsr_set_tuning: bad group cap");
        (knob == GSR_TUNE_TILE_SORT_GROUPS ? c->tile_groups : c->depth_groups) = value;
        return GSR_OK;
    default:
        return set_err(GSR_E_ARG, "gsr_set_tuning: unknown knob");
    }
}

extern "C" int gsr_rank_order_check(int64_t* lane_ops, int64_t* mismatches) {
    if (!lane_ops || !mismatches) return set_err(GSR_E_ARG, "gsr_rank_order_check: null argument");
    unsigned long long ops = 0, bad = 0;
    HIP_TRY(gsr::rank_order_check(&ops, &bad));
    *lane_ops = (int64_t)ops;
    *mismatches = (int64_t)bad;
    return GSR_OK;
}

extern "C" int gsr_set_blend_variant(gsr_context* c, int variant) {
    if (!c) return set_err(GSR_E_ARG, "null context");
    if (variant != 0 && variant != 3)
        return set_err(GSR_E_ARG, "gsr_set_blend_variant: variant must be 0 (default) or 3 (timeline stamps)");
    std::lock_guard<std::mutex> lk(c->mu);
    c->blend_variant = variant;
    return GSR_OK;
}

extern "C" int gsr_blend_stamps(gsr_context* c, uint64_t* out, int64_t n) {
    if (!c || !out || !c->consumed || n < 0 || n > c->consumed_cap)
        return set_err(GSR_E_ARG, "gsr_blend_stamps: bad argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (n) HIP_TRY(hipMemcpy(out, c->consumed, (size_t)n * 8, hipMemcpyDeviceToHost));
    return GSR_OK;
}

extern "C" int64_t gsr_blend_records_loaded(gsr_context* c) {
    int64_t v[8];
    if (gsr_blend_counters(c, v)) return -1;
    return v[0];
}

extern "C" int gsr_blend_counters_ex(gsr_context* c, int64_t* out, int n) {
    if (!c || !c->consumed || !out || n < 0 || n > 16 || c->blend_variant == 3)
        return set_err(GSR_E_ARG, "gsr_blend_counters_ex: diagnostics were off or bad count");
    std::lock_guard<std::mutex> lk(c->mu);
    unsigned long long v[16] = {};
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(v, c->consumed, sizeof v, hipMemcpyDeviceToHost));
    for (int i = 0; i < n; i++) out[i] = (int64_t)v[i];
    return GSR_OK;
}

extern "C" int gsr_blend_take_map(gsr_context* c, uint64_t* out, int64_t n) {
    if (!c || !c->consumed || !out || c->blend_variant == 3 || n != (int64_t)c->fr.W * c->fr.H ||
        c->consumed_cap < 16 + n)
        return set_err(GSR_E_ARG, "gsr_blend_take_map: diagnostics were off or bad size");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (n) HIP_TRY(hipMemcpy(out, c->consumed + 16, (size_t)n * 8, hipMemcpyDeviceToHost));
    return GSR_OK;
}

extern "C" int gsr_blend_counters(gsr_context* c, int64_t* out4) {
    if (!c || !c->consumed || !out4) return set_err(GSR_E_ARG, "gsr_blend_counters: diagnostics were off");
    std::lock_guard<std::mutex> lk(c->mu);
    unsigned long long v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(v, c->consumed, sizeof v, hipMemcpyDeviceToHost));
    for (int i = 0; i < 8; i++) out4[i] = (int64_t)v[i];
    return GSR_OK;
}

// ------------------------------------------------------------------ math probe

extern "C" int gsr_math_probe(const float* host_in, int n, float* host_out) {
    if (!host_in || !host_out || n <= 0) return set_err(GSR_E_ARG, "gsr_math_probe: bad argument");
    float *din = nullptr, *dout = nullptr;
    HIP_TRY(hipMalloc(&din, sizeof(float) * 2 * (size_t)n));
    HIP_TRY(hipMalloc(&dout, sizeof(float) * 9 * (size_t)n));
    HIP_TRY(hipMemcpy(din, host_in, sizeof(float) * 2 * (size_t)n, hipMemcpyHostToDevice));
    HIP_TRY(gsr::launch_math_probe(din, n, dout, nullptr));
    HIP_TRY(hipMemcpy(host_out, dout, sizeof(float) * 9 * (size_t)n, hipMemcpyDeviceToHost));
    (void)hipFree(din);
    (void)hipFree(dout);
    return GSR_OK;
}

extern "C" int gsr_exp_probe2(float x_lo, float x_hi, float x_big, int64_t* violations,
                              int64_t* packed_mismatches, float* err_all, float* err_big) {
    if (!violations || !packed_mismatches || !err_all || !err_big || !(x_lo < x_hi))
        return set_err(GSR_E_ARG, "gsr_exp_probe: bad argument");
    unsigned long long* dv = nullptr;
    uint32_t* de = nullptr;
    HIP_TRY(hipMalloc(&dv, 2 * sizeof(unsigned long long)));
    HIP_TRY(hipMalloc(&de, 2 * sizeof(uint32_t)));
    HIP_TRY(hipMemset(dv, 0, 2 * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(de, 0, 2 * sizeof(uint32_t)));
    HIP_TRY(gsr::launch_exp_probe(gsr_float_key(x_lo), gsr_float_key(x_hi), x_big, dv, de, nullptr));
    unsigned long long v[2] = {0, 0};
    uint32_t e[2] = {0, 0};
    HIP_TRY(hipMemcpy(v, dv, sizeof v, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(e, de, sizeof e, hipMemcpyDeviceToHost));
    (void)hipFree(dv);
    (void)hipFree(de);
    *violations = (int64_t)v[0];
    *packed_mismatches = (int64_t)v[1];
    *err_all = gsr_bits_to_float(e[0]);
    *err_big = gsr_bits_to_float(e[1]);
    return GSR_OK;
}

// The round-3 signature: one int64 behind `violations` (the packed-loop count is
// gsr_exp_probe2's).
extern "C" int gsr_exp_probe(float x_lo, float x_hi, float x_big, int64_t* violations, float* err_all,
                             float* err_big) {
    int64_t packed = 0;
    return gsr_exp_probe2(x_lo, x_hi, x_big, violations, &packed, err_all, err_big);
}

extern "C" int gsr_alpha_cut_probe(const float* host_op, int n, float* host_out) {
    if (!host_op || !host_out || n <= 0) return set_err(GSR_E_ARG, "gsr_alpha_cut_probe: bad argument");
    float *din = nullptr, *dout = nullptr;
    HIP_TRY(hipMalloc(&din, sizeof(float) * (size_t)n));
    HIP_TRY(hipMalloc(&dout, sizeof(float) * (size_t)n));
    HIP_TRY(hipMemcpy(din, host_op, sizeof(float) * (size_t)n, hipMemcpyHostToDevice));
    HIP_TRY(gsr::launch_xs_probe(din, n, dout, nullptr));
    HIP_TRY(hipMemcpy(host_out, dout, sizeof(float) * (size_t)n, hipMemcpyDeviceToHost));
    (void)hipFree(din);
    (void)hipFree(dout);
    return GSR_OK;
}

// ------------------------------------------------------------------ drop-in render

static std::mutex g_dropin_mu;
static gsr_context* g_dropin = nullptr;

// Whole drop-in frame into a DEVICE image (3*W*H floats) on the drop-in
// context, synchronous like the reference call: scene-layout detection from the
// block header, and up to two re-renders after a pair-buffer overflow.  Shared by
// preprocessCUDAGaussians (host image) and preprocessCUDAGaussiansGL (the
// viewer's SSBO, gsr_gl.cpp).  Returns a GSR_* code; `what` names the failing step.
int gsr::dropin_render_device(gsr_gaussian* d_gaussians, int num_gaussians, const gsr_camera& cam,
                              int num_tile_y, int num_tile_x, int width_stride, int height_stride, int W,
                              int H, float k, float* d_out, const char** what) {
    *what = "render";
    if (!g_dropin) g_dropin = gsr_create();
    gsr_context* c = g_dropin;
    // Layout detection: our scene block starts with a NaN-pattern magic.
    int layout = GSR_LAYOUT_AOS;
    if (num_gaussians > 0 && d_gaussians) {
        gsr_scene_header h{};
        *what = "scene";
        // One synchronous read (~16 us each on the viewer's frame): the whole header
        // when even an AoS buffer of num_gaussians records is at least that long (2+
        // records), else the magic first (16 B fit inside any 240-B AoS record) and the
        // rest of the header only once it is known to be our block.
        const bool whole = (int64_t)num_gaussians * (int64_t)sizeof(gsr_gaussian) >= (int64_t)sizeof h;
        HIP_TRY(hipMemcpy(whole ? static_cast<void*>(&h) : static_cast<void*>(&h.magic), d_gaussians,
                          whole ? sizeof h : sizeof h.magic, hipMemcpyDeviceToHost));
        if (h.magic[0] == GSR_SCENE_MAGIC0 && h.magic[1] == GSR_SCENE_MAGIC1 && h.magic[2] == GSR_SCENE_MAGIC2 &&
            h.magic[3] == GSR_SCENE_MAGIC3) {
            if (!whole) HIP_TRY(hipMemcpy(&h, d_gaussians, sizeof h, hipMemcpyDeviceToHost));
            // 4D blocks render at the drop-in context's time (gsr_set_time on it is not
            // reachable through this ABI, so t = 0: the sequence's first frame)
            layout = h.narrays == GSR_SCENE4D_NARRAYS    ? GSR_LAYOUT_SCENE_BLOCK_4D
                     : h.narrays == GSR_SCENE_SH3_NARRAYS ? GSR_LAYOUT_SCENE_BLOCK_SH3
                                                         : GSR_LAYOUT_SCENE_BLOCK;
            if ((int64_t)h.count != num_gaussians)
                return set_err(GSR_E_ARG, "num_gaussians %d != scene block count %llu", num_gaussians,
                               (unsigned long long)h.count);
        }
    }
    for (int attempt = 0; attempt < 3; attempt++) {
        *what = "render";
        int rc = gsr_render(c, d_gaussians, layout, num_gaussians, &cam, W, H, num_tile_x, num_tile_y,
                            width_stride, height_stride, k, d_out, nullptr);
        if (rc != GSR_OK && rc != GSR_E_OVERFLOW) return rc;
        *what = "sync";
        rc = gsr_sync(c);
        if (rc != GSR_E_OVERFLOW) return rc;
    }
    // each overflow grows the buffer to 1.25x the frame's pair count, so a repeat
    // means the scene or camera changed under us: report it, never a partial image
    return set_err(GSR_E_OVERFLOW, "pair buffer still overflowing after 3 renders");
}

extern "C" void preprocessCUDAGaussians(gsr_gaussian* d_gaussians, float* out_pixels, int num_gaussians,
                                        gsr_camera cam, int num_tile_y, int num_tile_x, int width_stride,
                                        int height_stride, int tile_W, int tile_H, float k) {
    std::lock_guard<std::mutex> lk(gsr::dropin_mutex());
    auto fail = [](const char* what) { std::fprintf(stderr, "preprocessCUDAGaussians: %s: %s\n", what, g_err.c_str()); };
    if (!out_pixels || tile_W <= 0 || tile_H <= 0) {
        set_err(GSR_E_ARG, "bad output buffer or size");
        fail("argument");
        return;
    }
    if (!g_dropin) g_dropin = gsr_create();
    gsr_context* c = g_dropin;
    const size_t npx = 3 * (size_t)tile_W * (size_t)tile_H;
    if ((int64_t)npx > c->out_cap) {
        if (realloc_dev(&c->out_tmp, npx)) { fail("alloc"); return; }
        c->out_cap = (int64_t)npx;
    }
    const char* what = "render";
    if (gsr::dropin_render_device(d_gaussians, num_gaussians, cam, num_tile_y, num_tile_x, width_stride,
                                  height_stride, tile_W, tile_H, k, c->out_tmp, &what) != GSR_OK) {
        fail(what);
        return;
    }
    if (hipMemcpy(out_pixels, c->out_tmp, npx * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) {
        set_err(GSR_E_HIP, "image readback failed");
        fail("readback");
    }
}

std::mutex& gsr::dropin_mutex() { return g_dropin_mu; }
const char* gsr::last_error() { return g_err.c_str(); }

// ------------------------------------------------------------------ reference sort ABI
//
// Both entry points take HOST arrays like the reference (they copy H2D, sort,
// copy D2H) and report the device time of the sort passes in *kernel_ms
// (cudaEvent bracket of render.cu:221-253 / onesweep.cu:217-240).

namespace {

struct SortBufs {
    uint64_t* a = nullptr;
    uint64_t* b = nullptr;
    uint64_t* c = nullptr;
    uint32_t* hist = nullptr;
    uint32_t* totals = nullptr;
    ~SortBufs() {
        for (void* p : {(void*)a, (void*)b, (void*)c, (void*)hist, (void*)totals})
            if (p) (void)hipFree(p);
    }
    int alloc(uint32_t n, bool third) {
        HIP_TRY(hipMalloc(&a, sizeof(uint64_t) * std::max<size_t>(n, 1)));
        HIP_TRY(hipMalloc(&b, sizeof(uint64_t) * std::max<size_t>(n, 1)));
        if (third) HIP_TRY(hipMalloc(&c, sizeof(uint64_t) * std::max<size_t>(n, 1)));
        HIP_TRY(hipMalloc(&hist, sizeof(uint32_t) * 256 * gsr::kMaxSortGroups));
        HIP_TRY(hipMalloc(&totals, sizeof(uint32_t) * 256));
        return GSR_OK;
    }
};

// Stable sort of n items on bits [32, 32 + nbits); returns the buffer holding the result.
int sort_high_bits(SortBufs& sb, uint64_t* a, uint64_t* b, uint32_t n, int nbits, uint64_t** result) {
    const int g = groups_for(n, gsr::kSortTile);
    uint64_t* src = a;
    uint64_t* dst = b;
    for (int sh = 0; sh < nbits; sh += 8) {
        HIP_TRY(gsr::launch_radix_pass(src, dst, nullptr, n, 32 + sh, std::min(8, nbits - sh), g, 16, sb.hist,
                                       sb.totals, nullptr, nullptr));
        std::swap(src, dst);
    }
    *result = src;
    return GSR_OK;
}

}  // namespace

extern "C" void oneSweepSort(int* input, int* output, int N, int maxVal, float* kernel_ms) {
    (void)maxVal;   // the reference sorts all 32 bits regardless (onesweep.cu:197-198)
    if (kernel_ms) *kernel_ms = 0.0f;
    if (N <= 0) return;
    if (!input || !output) {
        std::fprintf(stderr, "oneSweepSort: null buffer\n");
        return;
    }
    auto body = [&]() -> int {
        SortBufs sb;
        if (int rc = sb.alloc((uint32_t)N, false)) return rc;
        int* dkeys = nullptr;
        HIP_TRY(hipMalloc(&dkeys, sizeof(int) * (size_t)N));
        HIP_TRY(hipMemcpy(dkeys, input, sizeof(int) * (size_t)N, hipMemcpyHostToDevice));
        hipEvent_t e0, e1;
        HIP_TRY(hipEventCreate(&e0));
        HIP_TRY(hipEventCreate(&e1));
        HIP_TRY(hipEventRecord(e0, nullptr));
        HIP_TRY(gsr::launch_items_from_keys(dkeys, (uint32_t)N, sb.a, nullptr));
        uint64_t* res = nullptr;
        if (int rc = sort_high_bits(sb, sb.a, sb.b, (uint32_t)N, 32, &res)) return rc;
        HIP_TRY(gsr::launch_keys_from_items(res, (uint32_t)N, dkeys, nullptr));
        HIP_TRY(hipEventRecord(e1, nullptr));
        HIP_TRY(hipEventSynchronize(e1));
        float ms = 0.0f;
        HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
        if (kernel_ms) *kernel_ms = ms;
        HIP_TRY(hipMemcpy(output, dkeys, sizeof(int) * (size_t)N, hipMemcpyDeviceToHost));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipFree(dkeys);
        return GSR_OK;
    };
    if (body() != GSR_OK) std::fprintf(stderr, "oneSweepSort: %s\n", g_err.c_str());
}

extern "C" void oneSweep3DGaussianSort(gsr_lwg* d_in, int N, int num_bits, float* kernel_ms) {
    if (kernel_ms) *kernel_ms = 0.0f;
    if (N <= 0) return;
    if (!d_in || num_bits <= 0 || num_bits > 64) {
        std::fprintf(stderr, "oneSweep3DGaussianSort: bad argument\n");
        return;
    }
    // numPasses = (num_bits + 7) / 8 full 8-bit digits (render.cu:201): sort on
    // the low 8*numPasses bits of radix_id, stable, values travel with keys.
    const int nb = 8 * ((num_bits + 7) / 8);
    auto body = [&]() -> int {
        SortBufs sb;
        if (int rc = sb.alloc((uint32_t)N, true)) return rc;
        gsr_lwg *din = nullptr, *dout = nullptr;
        HIP_TRY(hipMalloc(&din, sizeof(gsr_lwg) * (size_t)N));
        HIP_TRY(hipMalloc(&dout, sizeof(gsr_lwg) * (size_t)N));
        HIP_TRY(hipMemcpy(din, d_in, sizeof(gsr_lwg) * (size_t)N, hipMemcpyHostToDevice));
        hipEvent_t e0, e1;
        HIP_TRY(hipEventCreate(&e0));
        HIP_TRY(hipEventCreate(&e1));
        HIP_TRY(hipEventRecord(e0, nullptr));
        // stage 1: low min(32, nb) bits
        const int b1 = std::min(32, nb);
        HIP_TRY(gsr::launch_items_from_lwg(din, nullptr, (uint32_t)N, 0, b1 == 32 ? 0xffffffffu : ((1u << b1) - 1u),
                                           sb.a, nullptr));
        uint64_t* r1 = nullptr;
        if (int rc = sort_high_bits(sb, sb.a, sb.b, (uint32_t)N, b1, &r1)) return rc;
        const uint64_t* s1 = nullptr;
        const uint64_t* s2 = r1;
        if (nb > 32) {
            // stage 2: bits [32, nb), stable over the stage-1 order (LSD composition)
            const int b2 = nb - 32;
            uint64_t* spare = (r1 == sb.a) ? sb.b : sb.a;
            HIP_TRY(gsr::launch_items_from_lwg(din, r1, (uint32_t)N, 32, b2 == 32 ? 0xffffffffu : ((1u << b2) - 1u),
                                               sb.c, nullptr));
            uint64_t* r2 = nullptr;
            if (int rc = sort_high_bits(sb, sb.c, spare, (uint32_t)N, b2, &r2)) return rc;
            s1 = r1;
            s2 = r2;
        }
        HIP_TRY(gsr::launch_gather_lwg(din, s1, s2, (uint32_t)N, dout, nullptr));
        HIP_TRY(hipEventRecord(e1, nullptr));
        HIP_TRY(hipEventSynchronize(e1));
        float ms = 0.0f;
        HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
        if (kernel_ms) *kernel_ms = ms;
        HIP_TRY(hipMemcpy(d_in, dout, sizeof(gsr_lwg) * (size_t)N, hipMemcpyDeviceToHost));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipFree(din);
        (void)hipFree(dout);
        return GSR_OK;
    };
    if (body() != GSR_OK) std::fprintf(stderr, "oneSweep3DGaussianSort: %s\n", g_err.c_str());
}
