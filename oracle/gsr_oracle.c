/*
 * gsr_oracle.c — CPU ORACLE (TEST INFRASTRUCTURE ONLY; see gsr_oracle.h).
 *
 * Restates, op for op and in the same order, the single-precision arithmetic
 * of the reference CUDA path so the HIP kernels can be checked bit-for-bit.
 * Build: gcc -O2 -ffp-contract=off (no implicit FMA, no fast-math; x86-64
 * SSE arithmetic is IEEE single with FLT_EVAL_METHOD == 0).
 *
 * Decisions where the reference is nondeterministic or undefined:
 *  - visible splats are ordered by (depth key, ORIGINAL index); the reference
 *    orders ties by shared-memory atomics (render.cu:559, 844);
 *  - float -> int casts saturate as the GPU's cvt does (gsr_f2i_sat/f2u_sat);
 *  - transcendental functions are the deterministic ones of gsr_detmath.h.
 */
#define _GNU_SOURCE
#include "gsr_oracle.h"
#include "../include/gsr_detmath.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

float orc_expf(float x) { return gsr_expf(x); }
float orc_blend_expf(float x) { return gsr_blend_expf(x); }

/* Exhaustive sweep of gsr_blend_expf over every float in [x_lo, x_hi] (OpenMP):
 * *viol = the number of x with f(x) > f(next float), *max_ulp = the largest error
 * against the double-precision exp in units of the float spacing at the result, over
 * the x of the sweep that lie in [-87, 88.7] (normal results, no overflow). */
void orc_blend_exp_sweep(float x_lo, float x_hi, int64_t* viol, double* max_ulp) {
    const uint32_t klo = gsr_float_key(x_lo), khi = gsr_float_key(x_hi);
    int64_t v = 0;
    double mu = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : v) reduction(max : mu)
    for (int64_t k = (int64_t)klo; k < (int64_t)khi; ++k) {
        const float x = gsr_key_float((uint32_t)k);
        const float e = gsr_blend_expf(x);
        if (e > gsr_blend_expf(gsr_key_float((uint32_t)k + 1u))) v++;
        if (x >= -87.0f && x <= 88.7f) {
            const double ref = exp((double)x);
            int ex;
            frexp(ref, &ex);
            const double u = fabs((double)e - ref) / ldexp(1.0, ex - 24);
            if (u > mu) mu = u;
        }
    }
    *viol = v;
    *max_ulp = mu;
}
float orc_sinf(float x) { return gsr_sinf(x); }
float orc_cosf(float x) { return gsr_cosf(x); }
float orc_atan2f(float y, float x) { return gsr_atan2f(y, x); }
float orc_alpha_take_min_x(float op) { return gsr_alpha_take_min_x(op); }
int orc_alpha_taken(float op, float x) { return gsr_alpha_taken(op, x); }

/* ------------------------------------------------------------ PLY loader */

/* std::getline: read up to '\n' (dropped); returns 0 at EOF with nothing read. */
static int read_line(FILE* f, char** buf, size_t* cap) {
    ssize_t len = getline(buf, cap, f);
    if (len < 0) return 0;
    if (len > 0 && (*buf)[len - 1] == '\n') (*buf)[len - 1] = 0;
    return 1;
}

static int starts_with(const char* s, const char* p) { return strncmp(s, p, strlen(p)) == 0; }

/* Slot kinds of gaussians.hpp:10 (SlotType). */
enum { S_X, S_Y, S_Z, S_NORMAL, S_DC, S_REST, S_OPACITY, S_SCALE, S_ROT, S_TCENTER, S_TSCALE, S_MOTION, S_SKIP };

/* misc.cu:13-134 + gaussians.cpp:17-30 (storeGaussianFromProperty). */
int orc_ply_read_ex(const char* path, float* soa, int narrays, int64_t capacity, int64_t* n_out) {
    FILE* f = fopen(path, "rb");
    if (!f) return -3;
    char* line = NULL;
    size_t cap = 0;
    char format[256] = {0};
    int have = 0;
    while (read_line(f, &line, &cap)) {                 /* misc.cu:25-30 */
        if (starts_with(line, "format ")) {
            snprintf(format, sizeof format, "%s", line + 7);
            have = 1;
            break;
        }
    }
    int found = 0;
    while (have && read_line(f, &line, &cap)) {         /* misc.cu:32-36 */
        if (starts_with(line, "element vertex ")) { found = 1; break; }
    }
    if (!found) { free(line); fclose(f); return -4; }
    char* end = NULL;
    long long nv = strtoll(line + 15, &end, 10);        /* std::stoi, misc.cu:37 */
    if (end == line + 15 || nv < 0) { free(line); fclose(f); return -4; }
    *n_out = nv;

    int kinds[1024];
    int idxs[1024];
    int nprops = 0;
    while (read_line(f, &line, &cap)) {                 /* misc.cu:58-90 */
        if (strcmp(line, "end_header") == 0) break;
        if (!starts_with(line, "property ")) continue;
        char type[256] = {0}, name[256] = {0};
        if (sscanf(line + 9, "%255s %255s", type, name) < 2) name[0] = 0;
        int kind = S_SKIP, idx = 0;
        if (!strcmp(name, "x")) kind = S_X;
        else if (!strcmp(name, "y")) kind = S_Y;
        else if (!strcmp(name, "z")) kind = S_Z;
        else if (!strcmp(name, "nxx")) { kind = S_NORMAL; idx = 0; }   /* sic, misc.cu:68 */
        else if (!strcmp(name, "ny")) { kind = S_NORMAL; idx = 1; }
        else if (!strcmp(name, "nz")) { kind = S_NORMAL; idx = 2; }
        else if (!strcmp(name, "f_dc_0")) { kind = S_DC; idx = 0; }
        else if (!strcmp(name, "f_dc_1")) { kind = S_DC; idx = 1; }
        else if (!strcmp(name, "f_dc_2")) { kind = S_DC; idx = 2; }
        else if (starts_with(name, "f_rest_")) {
            int r = atoi(name + 7);
            if (r >= 0 && r < (narrays == GSR_SCENE_SH3_NARRAYS ? 45 : 24)) { kind = S_REST; idx = r; }   /* misc.cu:76 */
        } else if (!strcmp(name, "opacity")) kind = S_OPACITY;
        else if (starts_with(name, "scale_")) { idx = atoi(name + 6); kind = (idx >= 0 && idx < 3) ? S_SCALE : S_SKIP; }
        else if (starts_with(name, "rot_")) { idx = atoi(name + 4); kind = (idx >= 0 && idx < 4) ? S_ROT : S_SKIP; }
        /* config 5 (own spec): Spacetime-Gaussian temporal properties */
        else if (!strcmp(name, "trbf_center")) kind = S_TCENTER;
        else if (!strcmp(name, "trbf_scale")) kind = S_TSCALE;
        else if (starts_with(name, "motion_")) { idx = atoi(name + 7); kind = (idx >= 0 && idx < 9) ? S_MOTION : S_SKIP; }
        if (nprops < 1024) { kinds[nprops] = kind; idxs[nprops] = idx; }
        nprops++;
    }
    free(line);
    if (strcmp(format, "binary_little_endian 1.0") != 0 || nprops > 1024 || nv > 2147483647LL) {
        fclose(f);
        return -4;
    }
    /* the data must hold the header's rows (the reference trusts the count; a test
     * oracle refuses what the product refuses, tests/test_ply_malformed.py) */
    const long here = ftell(f);
    if (here < 0 || fseek(f, 0, SEEK_END) != 0) { fclose(f); return -3; }
    const long avail = ftell(f) - here;
    if (fseek(f, here, SEEK_SET) != 0 || (long long)nprops * 4 * nv > (long long)avail) { fclose(f); return -3; }
    if (!soa || capacity < nv) { fclose(f); return 0; }

    const int64_t n = nv;
    memset(soa, 0, sizeof(float) * (size_t)narrays * (size_t)n);   /* Gaussian g{} */
    if (narrays == GSR_SCENE4D_NARRAYS)   /* 4D defaults: a static Gaussian (temporal scale 1) */
        for (int64_t i = 0; i < n; i++) soa[GSR_A_TSCALE * n + i] = 1.0f;
    float* row = (float*)malloc(sizeof(float) * (size_t)(nprops > 0 ? nprops : 1));
    int rc = 0;
    for (int64_t i = 0; i < n && rc == 0; i++) {
        if (nprops > 0 && fread(row, sizeof(float), (size_t)nprops, f) != (size_t)nprops) { rc = -3; break; }
        for (int p = 0; p < nprops; p++) {
            const float v = row[p];
            switch (kinds[p]) {
            case S_X: soa[GSR_A_X * n + i] = v; break;
            case S_Y: soa[GSR_A_Y * n + i] = v; break;
            case S_Z: soa[GSR_A_Z * n + i] = v; break;
            case S_DC: soa[(GSR_A_SH0 + idxs[p]) * n + i] = v; break;
            case S_REST:
                if (narrays == GSR_SCENE_SH3_NARRAYS)   /* SH-3 mode: f_rest channel-major (15 per channel) */
                    soa[(GSR_A_SH0 + 3 * (1 + idxs[p] % 15) + idxs[p] / 15) * n + i] = v;
                else
                    soa[(GSR_A_SH0 + 3 + idxs[p]) * n + i] = v;
                break;
            /* sigmoid<float>: 1.0f / (1.0f + std::exp(-x)) (gaussians.cpp:12-15) */
            case S_OPACITY: soa[GSR_A_OPACITY * n + i] = 1.0f / (1.0f + expf(-v)); break;
            /* exp(value) resolves to ::exp(double) (gaussians.cpp:26) */
            case S_SCALE: soa[(GSR_A_SCALE0 + idxs[p]) * n + i] = (float)exp((double)v); break;
            case S_ROT: soa[(GSR_A_ROT0 + idxs[p]) * n + i] = v; break;
            case S_TCENTER: if (narrays == GSR_SCENE4D_NARRAYS) soa[GSR_A_TCENTER * n + i] = v; break;
            case S_TSCALE: if (narrays == GSR_SCENE4D_NARRAYS) soa[GSR_A_TSCALE * n + i] = (float)exp((double)v); break;
            case S_MOTION: if (narrays == GSR_SCENE4D_NARRAYS) soa[(GSR_A_MOTION0 + idxs[p]) * n + i] = v; break;
            default: break;   /* normals are not used by the render path */
            }
        }
    }
    free(row);
    fclose(f);
    return rc;
}

int orc_ply_read(const char* path, float* soa, int64_t capacity, int64_t* n_out) {
    return orc_ply_read_ex(path, soa, GSR_SCENE_NARRAYS, capacity, n_out);
}

/*
 * Config 5 (own spec; Spacetime-Gaussian style): the 3D arrays of a
 * 4D scene at time t, with NO temporal cull — every Gaussian keeps its slot,
 * its position moved by the cubic motion and its opacity scaled by the
 * temporal RBF:
 *   dt = t - trbf_center; dt2 = dt*dt; dt3 = dt2*dt
 *   x_t = ((x + m0*dt) + m3*dt2) + m6*dt3      (y: m1 m4 m7, z: m2 m5 m8)
 *   u = dt / trbf_scale; opacity_t = opacity * exp(-(u*u))
 * out38 gets all 38 arrays of the time-t 3D scene (n elements each).
 */
void orc_temporal(const float* soa49, int64_t n, float t, float* out38) {
    memcpy(out38, soa49, sizeof(float) * (size_t)GSR_SCENE_NARRAYS * (size_t)n);
    for (int64_t i = 0; i < n; i++) {
        const float dt = t - soa49[GSR_A_TCENTER * n + i];
        const float dt2 = dt * dt, dt3 = dt2 * dt;
        for (int a = 0; a < 3; a++) {
            const float m1 = soa49[(GSR_A_MOTION0 + a) * n + i];
            const float m2 = soa49[(GSR_A_MOTION0 + 3 + a) * n + i];
            const float m3 = soa49[(GSR_A_MOTION0 + 6 + a) * n + i];
            out38[(GSR_A_X + a) * n + i] = ((soa49[(GSR_A_X + a) * n + i] + m1 * dt) + m2 * dt2) + m3 * dt3;
        }
        const float u = dt / soa49[GSR_A_TSCALE * n + i];
        out38[GSR_A_OPACITY * n + i] = soa49[GSR_A_OPACITY * n + i] * orc_expf(-(u * u));
    }
}

/* ------------------------------------------------------------ math.cu */

static void o_normalize(float v[3]) {                   /* math.cu:7-18 */
    float n = sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (n > 1e-8f) {
        v[0] /= n;
        v[1] /= n;
        v[2] /= n;
    } else {
        v[0] = 0.0f;
        v[1] = 0.0f;
        v[2] = 0.0f;
    }
}

static void o_matmul3(const float* A, const float* B, float* out) {   /* math.cu:120-129 */
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            out[i * 3 + j] = 0.0f;
            for (int k = 0; k < 3; ++k) out[i * 3 + j] += A[i * 3 + k] * B[k * 3 + j];
        }
}

static void o_matvec4(const float* M, const float* v, float* out) {   /* math.cu:131-138 */
    for (int i = 0; i < 4; ++i) {
        out[i] = 0.0f;
        for (int j = 0; j < 4; ++j) out[i] += M[i * 4 + j] * v[j];
    }
}

static void o_transpose3(const float* A, float* At) {                 /* math.cu:147-151 */
    At[0] = A[0]; At[1] = A[3]; At[2] = A[6];
    At[3] = A[1]; At[4] = A[4]; At[5] = A[7];
    At[6] = A[2]; At[7] = A[5]; At[8] = A[8];
}

static void o_rot_from_quat(const float* q, float* R) {              /* math.cu:153-164 */
    float w = q[0], x = q[1], y = q[2], z = q[3];
    float n = sqrtf(x * x + y * y + z * z + w * w);
    x /= n; y /= n; z /= n; w /= n;
    R[0] = 1 - 2 * y * y - 2 * z * z; R[1] = 2 * x * y - 2 * w * z;     R[2] = 2 * x * z + 2 * w * y;
    R[3] = 2 * x * y + 2 * w * z;     R[4] = 1 - 2 * x * x - 2 * z * z; R[5] = 2 * y * z - 2 * w * x;
    R[6] = 2 * x * z - 2 * w * y;     R[7] = 2 * y * z + 2 * w * x;     R[8] = 1 - 2 * x * x - 2 * y * y;
}

static void o_diag3(const float* a, float* D) {                       /* math.cu:166-170 */
    D[0] = a[0]; D[1] = 0.0f; D[2] = 0.0f;
    D[3] = 0.0f; D[4] = a[1]; D[5] = 0.0f;
    D[6] = 0.0f; D[7] = 0.0f; D[8] = a[2];
}

static void o_gemm(const float* A, const float* B, int M, int N, int K, float* out) {  /* math.cu:172-186 */
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < N; ++j) {
            out[i * N + j] = 0.0f;
            for (int k = 0; k < K; ++k) out[i * N + j] += A[i * K + k] * B[k * N + j];
        }
}

/* ------------------------------------------------------------ render.cu */

void orc_project(const float V[16], const float P[16], const float xyz[3], float tmp[4], float ndc[4]) {
    float old_xyz[4] = {xyz[0], xyz[1], xyz[2], 1.0f};
    o_matvec4(V, old_xyz, tmp);
    o_matvec4(P, tmp, ndc);
    ndc[0] = ndc[0] / ndc[3];
    ndc[1] = ndc[1] / ndc[3];
    ndc[2] = ndc[2] / ndc[3];
}

void orc_covariance_chain(const float quat[4], const float scale[3], const float XYZ[3], float fx,
                          float fy, const float r_cam[9], const float r_cam_T[9], float sigma2d[4]) {
    const float X = XYZ[0], Y = XYZ[1], Z = XYZ[2];
    float jac[6], jacT[6], R[9], RT[9], S[9], tmp[9], cov[9];
    jac[0] = fx / Z; jac[1] = 0.0f;
    jac[2] = -fx * X / (Z * Z); jac[3] = 0.0f;
    jac[4] = fy / Z; jac[5] = -fy * Y / (Z * Z);
    jacT[0] = jac[0]; jacT[1] = jac[3]; jacT[2] = jac[1];
    jacT[3] = jac[4]; jacT[4] = jac[2]; jacT[5] = jac[5];
    o_rot_from_quat(quat, R);
    o_transpose3(R, RT);
    o_diag3(scale, S);
    o_matmul3(R, S, tmp);
    o_matmul3(tmp, S, R);
    o_matmul3(R, RT, cov);
    o_matmul3(r_cam, cov, tmp);
    o_matmul3(tmp, r_cam_T, cov);
    o_gemm(jac, cov, 2, 3, 3, tmp);
    o_gemm(tmp, jacT, 2, 2, 3, sigma2d);
}

static const float SH_C0 = 0.28209479177387814f;                      /* render.cu:369-377 */
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};

/* SH-3 ("Inria-correct") mode: the soa holds 59 arrays, sh[3k + c] for k < 16,
 * and the colour is the degree-3 evaluation of the 3DGS training code
 * (bands 0..3 left to right, + 0.5, clamped at 0 only). */
static int g_sh3 = 0;
void orc_set_sh3(int on) { g_sh3 = on != 0; }

static void color_sh3(const float* soa, int64_t n, int64_t i, const float dir[3], float color[3]) {
    static const float C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                                0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                                -0.5900435899266435f};
    const float x = dir[0], y = dir[1], z = dir[2];
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    for (int c = 0; c < 3; c++) {
        float S[16];
        for (int k = 0; k < 16; k++) S[k] = soa[(GSR_A_SH0 + 3 * k + c) * n + i];
        float r = SH_C0 * S[0];
        r = r - SH_C1 * y * S[1] + SH_C1 * z * S[2] - SH_C1 * x * S[3];
        r = r + SH_C2[0] * xy * S[4] + SH_C2[1] * yz * S[5] + SH_C2[2] * (2.0f * zz - xx - yy) * S[6] +
            SH_C2[3] * xz * S[7] + SH_C2[4] * (xx - yy) * S[8];
        r = r + C3[0] * y * (3.0f * xx - yy) * S[9] + C3[1] * xy * z * S[10] + C3[2] * y * (4.0f * zz - xx - yy) * S[11] +
            C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * S[12] + C3[4] * x * (4.0f * zz - xx - yy) * S[13] +
            C3[5] * z * (xx - yy) * S[14] + C3[6] * x * (xx - 3.0f * yy) * S[15];
        r += 0.5f;
        color[c] = fmaxf(r, 0.0f);
    }
}

void orc_intrinsics(const gsr_camera* cam, float* fx, float* fy) {
    /* fy = 1.0f / tanf(fovY * 0.5f * (CUDART_PI_F / 180.0f)) (render.cu:620);
       tanf taken correctly rounded via double. */
    const float PI_F = 3.141592654f;                                   /* CUDART_PI_F */
    const float arg = cam->fovY * 0.5f * (PI_F / 180.0f);
    const float t = (float)tan((double)arg);
    *fy = 1.0f / t;
    *fx = *fy / cam->aspectRatio;                                      /* render.cu:621 */
}

int orc_preprocess(const float* soa, int64_t n, const gsr_camera* cam, int W, int H, float k,
                   orc_splat* out) {
    float fx, fy;
    orc_intrinsics(cam, &fx, &fy);
    const float* V = cam->V_matrix;
    const float* P = cam->P_matrix;
    const float znear = cam->nearClip;
    for (int64_t i = 0; i < n; i++) {
        orc_splat* s = &out[i];
        memset(s, 0, sizeof *s);
        s->depth_key = 0xffffffffu;
        float gx = soa[GSR_A_X * n + i], gy = soa[GSR_A_Y * n + i], gz = soa[GSR_A_Z * n + i];
        float sh[27];
        for (int c = 0; c < 27; c++) sh[c] = soa[(GSR_A_SH0 + c) * n + i];

        /* ---- advancedCullGaussians (render.cu:500-561) ---- */
        float dir[3] = {gx - cam->position[0], gy - cam->position[1], gz - cam->position[2]};
        o_normalize(dir);
        float color[3];
        if (g_sh3) {
            color_sh3(soa, n, i, dir, color);
            for (int c = 0; c < 3; c++) s->color[c] = color[c];
        } else {
        for (int c = 0; c < 3; c++) color[c] = sh[c] * SH_C0;
        {
            const float x = dir[0], y = dir[1], z = dir[2];
            for (int c = 0; c < 3; c++) {
                color[c] += SH_C1 * z * sh[2 * 3 + c];
                color[c] -= SH_C1 * y * sh[3 + c];
                color[c] -= SH_C1 * x * sh[3 * 3 + c];
            }
            const float xx = x * x, yy = y * y, zz = z * z;
            const float xy = x * y, yz = y * z, xz = x * z;
            for (int c = 0; c < 3; c++) {
                color[c] += SH_C2[0] * xy * sh[4 * 3 + c];
                color[c] += SH_C2[1] * yz * sh[5 * 3 + c];
                color[c] += SH_C2[2] * (2.0f * zz - xx - yy) * sh[6 * 3 + c];
                color[c] += SH_C2[3] * xz * sh[7 * 3 + c];
                color[c] += SH_C2[4] * (xx - yy) * sh[8 * 3 + c];
            }
        }
        for (int c = 0; c < 3; c++) {
            color[c] += 0.5f;
            color[c] = fminf(fmaxf(color[c], 0.0f), 1.0f);
            s->color[c] = color[c];
        }
        }   /* reference SH (bands 0..2) */
        float old_xyz[4] = {gx, gy, gz, 1.0f};
        float tmp_xyz[4], new_xyz[4];
        o_matvec4(V, old_xyz, tmp_xyz);
        s->view[0] = tmp_xyz[0]; s->view[1] = tmp_xyz[1]; s->view[2] = tmp_xyz[2];
        if (!isfinite(tmp_xyz[0]) || !isfinite(tmp_xyz[1]) || !isfinite(tmp_xyz[2])) continue;
        o_matvec4(P, tmp_xyz, new_xyz);
        new_xyz[0] = new_xyz[0] / new_xyz[3];
        new_xyz[1] = new_xyz[1] / new_xyz[3];
        new_xyz[2] = new_xyz[2] / new_xyz[3];
        s->ndc[0] = new_xyz[0]; s->ndc[1] = new_xyz[1]; s->ndc[2] = new_xyz[2];
        if (!isfinite(new_xyz[0]) || !isfinite(new_xyz[1]) || !isfinite(new_xyz[2])) continue;
        if (tmp_xyz[2] >= -znear || new_xyz[2] < -1.0f || new_xyz[2] > 1.0f) continue;
        s->status = 1;

        /* ---- prepareGaussians (render.cu:637-775) ---- */
        const float X = tmp_xyz[0], Y = tmp_xyz[1], Z = tmp_xyz[2];
        float jac[6], jacT[6], R[9], RT[9], S[9], sc[3], tmp[9], cov[9];
        jac[0] = fx / Z; jac[1] = 0.0f;
        jac[2] = -fx * X / (Z * Z); jac[3] = 0.0f;
        jac[4] = fy / Z; jac[5] = -fy * Y / (Z * Z);
        jacT[0] = jac[0]; jacT[1] = jac[3]; jacT[2] = jac[1];
        jacT[3] = jac[4]; jacT[4] = jac[2]; jacT[5] = jac[5];
        float rot[4];
        for (int c = 0; c < 4; c++) rot[c] = soa[(GSR_A_ROT0 + c) * n + i];
        o_rot_from_quat(rot, R);
        o_transpose3(R, RT);
        /* render.cu:664-667 multiplies by a constant 1 (exact): omitted */
        sc[0] = soa[(GSR_A_SCALE0 + 0) * n + i];
        sc[1] = soa[(GSR_A_SCALE0 + 1) * n + i];
        sc[2] = soa[(GSR_A_SCALE0 + 2) * n + i];
        o_diag3(sc, S);
        o_matmul3(R, S, tmp);
        o_matmul3(tmp, S, R);
        o_matmul3(R, RT, cov);
        o_matmul3(cam->r_cam, cov, tmp);
        o_matmul3(tmp, cam->r_cam_T, cov);
        o_gemm(jac, cov, 2, 3, 3, tmp);
        float S2[4];
        o_gemm(tmp, jacT, 2, 2, 3, S2);
        S2[0] = (W * 0.5f) * (W * 0.5f) * S2[0];
        S2[1] = (W * 0.5f) * (H * 0.5f) * S2[1];
        S2[2] = (H * 0.5f) * (W * 0.5f) * S2[2];
        S2[3] = (H * 0.5f) * (H * 0.5f) * S2[3];
        const float det = S2[0] * S2[3] - S2[1] * S2[2];
        if (!isfinite(det) || det < 1e-8f) continue;
        const float invDet = 1.0f / det;
        s->inv_covar[0] = S2[3] * invDet;
        s->inv_covar[1] = -S2[1] * invDet;
        s->inv_covar[2] = -S2[2] * invDet;
        s->inv_covar[3] = S2[0] * invDet;
        const float Sxx = S2[0], Sxy = S2[1], Syx = S2[2], Syy = S2[3];
        const float sxy = 0.5f * (Sxy + Syx);
        const float tr = Sxx + Syy;
        const float dif = Sxx - Syy;
        const float rad = sqrtf(fmaxf(0.0f, dif * dif + 4 * sxy * sxy));
        float l1 = 0.5f * (tr + rad);
        float l2 = 0.5f * (tr - rad);
        const float eps = 1e-8f;
        l1 = fmaxf(l1, eps);
        l2 = fmaxf(l2, eps);
        const float theta = 0.5f * gsr_atan2f(2 * sxy, dif);
        const float r1 = k * sqrtf(l1);
        const float r2 = k * sqrtf(l2);
        const float c = gsr_cosf(theta);
        const float sn = gsr_sinf(theta);
        float ex = fabsf(r1 * c) + fabsf(r2 * sn);
        float ey = fabsf(r1 * sn) + fabsf(r2 * c);
        ex /= W / 2.0f;
        ey /= H / 2.0f;
        float xmin = new_xyz[0] - ex, xmax = new_xyz[0] + ex;
        float ymin = new_xyz[1] - ey, ymax = new_xyz[1] + ey;
        if (xmax < -0.99f || xmin > 0.99f || ymax < -0.99f || ymin > 0.99f) continue;
        xmin = fmaxf(xmin, -1.0f);
        xmax = fminf(xmax, 1.0f);
        ymin = fmaxf(ymin, -1.0f);
        ymax = fminf(ymax, 1.0f);
        s->aabb[0] = gsr_f2i_sat(floorf(((xmin + 1.0f) * 0.5f) * W));
        s->aabb[1] = gsr_f2i_sat(floorf(((ymin + 1.0f) * 0.5f) * H));
        s->aabb[2] = gsr_f2i_sat(ceilf(((xmax + 1.0f) * 0.5f) * W));
        s->aabb[3] = gsr_f2i_sat(ceilf(((ymax + 1.0f) * 0.5f) * H));
        s->px_x = gsr_f2i_sat(roundf(((new_xyz[0] + 1.0f) * 0.5f) * W));
        s->px_y = gsr_f2i_sat(roundf(((new_xyz[1] + 1.0f) * 0.5f) * H));
        s->depth_key = gsr_f2u_sat(-Z * 1e6f);                    /* render.cu:850 */
        s->opacity = soa[GSR_A_OPACITY * n + i];
        s->status = 2;
    }
    return 0;
}

/* ------------------------------------------------------------ blend */

typedef struct { uint32_t key; uint32_t idx; } orc_kv;

static int cmp_kv(const void* a, const void* b) {
    const orc_kv* x = (const orc_kv*)a;
    const orc_kv* y = (const orc_kv*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

/* One pixel-splat step of renderGaussians (render.cu:326-340).  take (optional): the
 * pixel's take-map entry (gsr_blend_take_map: count | index-mix sum << 32). */
/* Which FMA contractions the reference's compiler applied to render.cu:331 and 337 cannot
 * be observed here (the CUDA path cannot be built).  orc_set_blend_variant selects
 * another plausible choice, so the parity hole can be measured
 * (tests/test_oracle_contraction.py, tools/contraction_parity.py):
 *   md2: 0 no contraction; 1 the first product of each sum fused (shipped, = the
 *        kernels); 2 the second product of each sum fused; 3 the inner sums only
 *        (first product); 4 the outer sum only (first product);
 *   rgb: 0 rgb + (color * alpha) * T rounded twice; 1 fmaf(color * alpha, T, rgb) (shipped);
 *   exp: 0 gsr_blend_expf (shipped); 1 the host libm expf (glibc: correctly rounded);
 *        2 gsr_expf (Cephes, the blend's exp up to round 3). */
static int g_var_md2 = 1, g_var_rgb = 1, g_var_exp = 0;
void orc_set_blend_variant(int md2, int rgb, int expm) {
    g_var_md2 = md2;
    g_var_rgb = rgb;
    g_var_exp = expm;
}

static inline float md2_variant(float dx, float dy, const float* ic) {
    switch (g_var_md2) {
    case 0: return dx * (ic[0] * dx + ic[1] * dy) + dy * (ic[2] * dx + ic[3] * dy);
    case 2: return __builtin_fmaf(dy, __builtin_fmaf(ic[3], dy, ic[2] * dx), dx * __builtin_fmaf(ic[1], dy, ic[0] * dx));
    case 3: return dx * __builtin_fmaf(ic[0], dx, ic[1] * dy) + dy * __builtin_fmaf(ic[2], dx, ic[3] * dy);
    case 4: return __builtin_fmaf(dx, ic[0] * dx + ic[1] * dy, dy * (ic[2] * dx + ic[3] * dy));
    default: return gsr_blend_md2(dx, dy, ic[0], ic[1], ic[2], ic[3]);
    }
}

/* blend_step with the contraction variant of orc_set_blend_variant (never the CPU
 * baseline's path: orc_render_takes takes blend_step when the variant is the shipped one) */
static void blend_step_var(const orc_splat* g, int gx, int gy, float* T, float* rgb, uint64_t* take,
                           uint32_t gid) {
    if (gx < g->aabb[0] || gx > g->aabb[2] || gy < g->aabb[1] || gy > g->aabb[3]) return;
    if (*T < 1e-3f) return;
    const float dx = ((float)gx - (float)g->px_x);
    const float dy = ((float)gy - (float)g->px_y);
    const float md2 = md2_variant(dx, dy, g->inv_covar);
    const float x = -0.5f * md2;
    float opacity = g->opacity * (g_var_exp == 1 ? expf(x) : g_var_exp == 2 ? gsr_expf(x) : gsr_blend_expf(x));
    opacity = fminf(opacity, 0.99f);
    if (opacity < 1e-3f) return;
    for (int c = 0; c < 3; ++c)
        rgb[c] = g_var_rgb ? __builtin_fmaf(g->color[c] * opacity, *T, rgb[c]) : rgb[c] + g->color[c] * opacity * *T;
    *T *= (1.0f - opacity);
    if (take) {
        const uint32_t cnt = (uint32_t)*take + 1u, hs = (uint32_t)(*take >> 32) + (gid + 1u) * 2654435761u;
        *take = (uint64_t)cnt | ((uint64_t)hs << 32);
    }
}

static inline void blend_step(const orc_splat* g, int gx, int gy, float* T, float* rgb, uint64_t* take,
                              uint32_t gid) {
    if (gx < g->aabb[0] || gx > g->aabb[2] || gy < g->aabb[1] || gy > g->aabb[3]) return;
    if (*T < 1e-3f) return;
    const float dx = ((float)gx - (float)g->px_x);
    const float dy = ((float)gy - (float)g->px_y);
    const float* ic = g->inv_covar;
    /* render.cu:331 and 337 with nvcc's default FMA contraction (gsr_blend_md2) */
    const float md2 = gsr_blend_md2(dx, dy, ic[0], ic[1], ic[2], ic[3]);
    float opacity = g->opacity * gsr_blend_expf(-0.5f * md2);
    opacity = fminf(opacity, 0.99f);
    if (opacity < 1e-3f) return;
    for (int c = 0; c < 3; ++c) rgb[c] = __builtin_fmaf(g->color[c] * opacity, *T, rgb[c]);
    *T *= (1.0f - opacity);
    if (take) {
        const uint32_t cnt = (uint32_t)*take + 1u, hs = (uint32_t)(*take >> 32) + (gid + 1u) * 2654435761u;
        *take = (uint64_t)cnt | ((uint64_t)hs << 32);
    }
}

static int cover_dims(int W, int H, int nx, int ny, int ws, int hs, int* cw, int* ch) {
    if (W <= 0 || H <= 0 || nx <= 0 || ny <= 0 || ws <= 0 || hs <= 0) return -1;
    long long a = (long long)nx * ws, b = (long long)ny * hs;
    *cw = a < W ? (int)a : W;
    *ch = b < H ? (int)b : H;
    return 0;
}

/* orc_render plus the per-pixel take map (W * H entries, row-major; pixels outside
 * the covered area stay 0), the GPU's gsr_blend_take_map. */
int orc_render_takes(const float* soa, int64_t n, const gsr_camera* cam, int W, int H, int nx, int ny,
                     int ws, int hs, float k, float* out, uint64_t* takes, int threads);

int orc_render(const float* soa, int64_t n, const gsr_camera* cam, int W, int H, int nx, int ny,
               int ws, int hs, float k, float* out, int threads) {
    return orc_render_takes(soa, n, cam, W, H, nx, ny, ws, hs, k, out, NULL, threads);
}

int orc_render_takes(const float* soa, int64_t n, const gsr_camera* cam, int W, int H, int nx, int ny,
                     int ws, int hs, float k, float* out, uint64_t* takes, int threads) {
    int cw, ch;
    if (cover_dims(W, H, nx, ny, ws, hs, &cw, &ch)) return -1;
    orc_splat* sp = (orc_splat*)malloc(sizeof(orc_splat) * (size_t)(n > 0 ? n : 1));
    orc_preprocess(soa, n, cam, W, H, k, sp);
    int64_t m = 0;
    for (int64_t i = 0; i < n; i++) m += sp[i].status == 2;
    orc_kv* order = (orc_kv*)malloc(sizeof(orc_kv) * (size_t)(m > 0 ? m : 1));
    m = 0;
    for (int64_t i = 0; i < n; i++)
        if (sp[i].status == 2) { order[m].key = sp[i].depth_key; order[m].idx = (uint32_t)i; m++; }
    qsort(order, (size_t)m, sizeof(orc_kv), cmp_kv);

    const size_t npx = (size_t)W * (size_t)H;
    memset(out, 0, sizeof(float) * 3 * npx);
    if (takes) memset(takes, 0, sizeof(uint64_t) * npx);
    const int band = 8;
    const int nbands = (ch + band - 1) / band;
    const int shipped = g_var_md2 == 1 && g_var_rgb == 1 && g_var_exp == 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int b = 0; b < nbands; b++) {
        const int y0 = b * band;
        const int y1 = (y0 + band < ch ? y0 + band : ch) - 1;
        float* T = (float*)malloc(sizeof(float) * (size_t)band * (size_t)cw);
        float* rgb = (float*)calloc((size_t)band * (size_t)cw * 3, sizeof(float));
        for (size_t q = 0; q < (size_t)band * (size_t)cw; q++) T[q] = 1.0f;
        for (int64_t s = 0; s < m; s++) {
            const orc_splat* g = &sp[order[s].idx];
            if (g->aabb[3] < y0 || g->aabb[1] > y1) continue;
            const int ya = g->aabb[1] > y0 ? g->aabb[1] : y0;
            const int yb = g->aabb[3] < y1 ? g->aabb[3] : y1;
            const int xa = g->aabb[0] > 0 ? g->aabb[0] : 0;
            const int xb = g->aabb[2] < cw - 1 ? g->aabb[2] : cw - 1;
            for (int y = ya; y <= yb; y++)
                for (int x = xa; x <= xb; x++) {
                    const size_t q = (size_t)(y - y0) * cw + x;
                    if (shipped)
                        blend_step(g, x, y, &T[q], &rgb[3 * q], takes ? &takes[(size_t)y * W + x] : NULL,
                                   order[s].idx);
                    else
                        blend_step_var(g, x, y, &T[q], &rgb[3 * q], takes ? &takes[(size_t)y * W + x] : NULL,
                                       order[s].idx);
                }
        }
        for (int y = y0; y <= y1; y++)
            for (int x = 0; x < cw; x++) {
                const size_t q = (size_t)(y - y0) * cw + x;
                for (int c = 0; c < 3; c++) out[c * npx + (size_t)y * W + x] += rgb[3 * q + c];
            }
        free(T);
        free(rgb);
    }
    free(order);
    free(sp);
    return 0;
}

typedef struct { uint64_t key; uint32_t idx; } orc_pair;

static int cmp_pair(const void* a, const void* b) {
    const orc_pair* x = (const orc_pair*)a;
    const orc_pair* y = (const orc_pair*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

int orc_render_tiled(const float* soa, int64_t n, const gsr_camera* cam, int W, int H, int nx, int ny,
                     int ws, int hs, float k, float* out) {
    int cw, ch;
    if (cover_dims(W, H, nx, ny, ws, hs, &cw, &ch)) return -1;
    orc_splat* sp = (orc_splat*)malloc(sizeof(orc_splat) * (size_t)(n > 0 ? n : 1));
    orc_preprocess(soa, n, cam, W, H, k, sp);
    /* buildLwgs (render.cu:829-856): one pair per covered reference tile. */
    size_t np = 0, capp = 1024;
    orc_pair* pairs = (orc_pair*)malloc(sizeof(orc_pair) * capp);
    for (int64_t i = 0; i < n; i++) {
        const orc_splat* g = &sp[i];
        if (g->status != 2) continue;
        if (g->aabb[0] > g->aabb[2] || g->aabb[1] > g->aabb[3]) continue;
        const int min_x = (int)fmaxf(0, (float)(g->aabb[0] / ws));
        const int max_x = (int)fminf((float)(nx - 1), (float)(g->aabb[2] / ws));
        const int min_y = (int)fmaxf(0, (float)(g->aabb[1] / hs));
        const int max_y = (int)fminf((float)(ny - 1), (float)(g->aabb[3] / hs));
        for (int tx = min_x; tx <= max_x; tx++)
            for (int ty = min_y; ty <= max_y; ty++) {
                if (np == capp) { capp *= 2; pairs = (orc_pair*)realloc(pairs, sizeof(orc_pair) * capp); }
                pairs[np].key = ((uint64_t)(uint32_t)(tx + ty * nx) << 32) | g->depth_key;
                pairs[np].idx = (uint32_t)i;
                np++;
            }
    }
    qsort(pairs, np, sizeof(orc_pair), cmp_pair);
    const size_t npx = (size_t)W * (size_t)H;
    memset(out, 0, sizeof(float) * 3 * npx);
    const int bs = ws * hs;
    float* T = (float*)malloc(sizeof(float) * (size_t)bs);
    float* rgb = (float*)malloc(sizeof(float) * 3 * (size_t)bs);
    size_t p = 0;
    for (int t = 0; t < nx * ny; t++) {                 /* renderGaussians (render.cu:285-365) */
        const int x_off = (t % nx) * ws, y_off = (t / nx) * hs;
        for (int j = 0; j < bs; j++) { T[j] = 1.0f; rgb[3 * j] = rgb[3 * j + 1] = rgb[3 * j + 2] = 0.0f; }
        while (p < np && (pairs[p].key >> 32) == (uint64_t)t) {
            const orc_splat* g = &sp[pairs[p].idx];
            for (int j = 0; j < bs; j++) {
                const int gx = j % ws + x_off, gy = j / ws + y_off;
                if (gx >= W || gy >= H) continue;
                blend_step(g, gx, gy, &T[j], &rgb[3 * j], NULL, 0u);
            }
            p++;
        }
        for (int j = 0; j < bs; j++) {
            const int gx = x_off + j % ws, gy = y_off + j / ws;
            if (gx < W && gy < H)
                for (int c = 0; c < 3; c++) out[c * npx + (size_t)gy * W + gx] += rgb[3 * j + c];
        }
    }
    free(T);
    free(rgb);
    free(pairs);
    free(sp);
    return 0;
}
