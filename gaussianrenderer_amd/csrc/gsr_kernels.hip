// gsr_kernels.hip — gfx950 (CDNA4) kernels of the 3DGS rasterizer.
//
// Pipeline per frame (all stream-ordered, no host round trip):
//   k_preprocess      one thread per Gaussian, SoA coalesced loads: cull + SH
//                     colour + view/clip + 2D covariance + extent + AABB, writes a
//                     64-B splat record and the (depth_key << 32 | index) item
//                     [render.cu:472-786]
//   radix passes      stable LSD sort of the N items by depth key (4 x 8 bits)
//   k_emit_*          scan of per-Gaussian tile counts in depth order, then one
//                     (tile << 32 | index) pair per covered 16x16 tile
//                     [render.cu:811-857, 788-809]
//   radix passes      stable LSD sort of the pairs by tile id (2 x <= 8 bits)
//                     (the last tile pass also records each tile's [start, end))
//   k_blend           one workgroup per 16x16 tile, one pixel per lane, 8x8 pixel
//                     block per wave64; LDS-staged batches of 256 splat records;
//                     exact per-pixel early termination [render.cu:266-367]
//
// Every float expression restates render.cu / math.cu in the same operation
// order; the file is compiled with -ffp-contract=off so no FMA is formed
// implicitly, and the transcendental functions come from gsr_detmath.h, so the
// results are bit-identical to the CPU oracle (oracle/gsr_oracle.c).
#include <hip/hip_runtime.h>

#include "gsr_detmath.h"
#include "gsr.h"
#include "gsr_internal.h"

namespace gsr {

namespace {

__constant__ float kShC0 = 0.28209479177387814f;      // render.cu:369-377
__constant__ float kShC1 = 0.4886025119029199f;

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// ------------------------------------------------------------------ helpers

// Exclusive scan across a 256-thread workgroup (4 waves).  `scratch` holds 4
// entries.  Contains two barriers; every thread of the block must call it.
template <typename T>
__device__ __forceinline__ T block_exclusive_scan(T v, T* scratch, T& total) {
    const uint32_t lane = lane_id();
    const uint32_t w = threadIdx.x >> 6;
    T x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        T y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) scratch[w] = x;
    __syncthreads();
    T pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const T s = scratch[k];
        if ((uint32_t)k < w) pre += s;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return pre + x - v;
}

// [begin, end) of workgroup g when n items are split over `groups` workgroups in
// chunks that are multiples of `gran`.
__device__ __forceinline__ void chunk_range(uint64_t n, int groups, int g, uint64_t gran,
                                            uint64_t& b, uint64_t& e) {
    uint64_t per = (n + (uint64_t)groups - 1) / (uint64_t)groups;
    per = (per + gran - 1) / gran * gran;
    b = per * (uint64_t)g;
    if (b > n) b = n;
    e = b + per;
    if (e > n) e = n;
}

// --------------------------------------------------------------- AoS -> SoA

// Accepts the reference's Gaussian[] (gaussians.hpp:16-30) as input.
__global__ __launch_bounds__(256) void k_aos_to_soa(const gsr_gaussian* __restrict__ g, int64_t n,
                                                    float* __restrict__ a, int64_t stride) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const gsr_gaussian& q = g[i];
    a[GSR_A_X * stride + i] = q.x;
    a[GSR_A_Y * stride + i] = q.y;
    a[GSR_A_Z * stride + i] = q.z;
    a[GSR_A_OPACITY * stride + i] = q.opacity;
#pragma unroll
    for (int c = 0; c < 3; c++) a[(GSR_A_SCALE0 + c) * stride + i] = q.scale[c];
#pragma unroll
    for (int c = 0; c < 4; c++) a[(GSR_A_ROT0 + c) * stride + i] = q.rot[c];
#pragma unroll
    for (int c = 0; c < 27; c++) a[(GSR_A_SH0 + c) * stride + i] = q.sh[c];
}

// ------------------------------------------------------------------ preprocess

// math.cu:120-129 (matMul3D_cuda): out = 0; out += A[ik]*B[kj], k ascending.
__device__ __forceinline__ void mm3(const float* A, const float* B, float* out) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            float acc = 0.0f;
#pragma unroll
            for (int k = 0; k < 3; ++k) acc += A[i * 3 + k] * B[k * 3 + j];
            out[i * 3 + j] = acc;
        }
}

// math.cu:172-186 (geMatMul_cuda), A MxK, B KxN.
template <int M, int N, int K>
__device__ __forceinline__ void gemm(const float* A, const float* B, float* out) {
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
        for (int j = 0; j < N; ++j) {
            float acc = 0.0f;
#pragma unroll
            for (int k = 0; k < K; ++k) acc += A[i * K + k] * B[k * N + j];
            out[i * N + j] = acc;
        }
}

// math.cu:131-138 (matVecMul4D_cuda).
__device__ __forceinline__ void mv4(const float* M, const float* v, float* out) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float acc = 0.0f;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc += M[i * 4 + j] * v[j];
        out[i] = acc;
    }
}

__device__ __forceinline__ uint4 dead_record_d() {
    // tile ranges empty, count 0, depth key 0xFFFFFFFF (sorts last)
    return make_uint4(0u, 0u, 0u, 0xffffffffu);
}

__global__ __launch_bounds__(256) void k_preprocess(const float* __restrict__ arr, int64_t stride,
                                                    int64_t n, Frame fr, uint4* __restrict__ rec,
                                                    uint64_t* __restrict__ items) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float gx = arr[GSR_A_X * stride + i];
    const float gy = arr[GSR_A_Y * stride + i];
    const float gz = arr[GSR_A_Z * stride + i];
    uint4* R = rec + 4 * i;
    items[i] = ((uint64_t)0xffffffffu << 32) | (uint64_t)(uint32_t)i;

    // ---- view + clip transform and cull (render.cu:535-556) ----
    const float old_xyz[4] = {gx, gy, gz, 1.0f};
    float tmp_xyz[4], new_xyz[4];
    mv4(fr.V, old_xyz, tmp_xyz);
    if (!isfinite(tmp_xyz[0]) || !isfinite(tmp_xyz[1]) || !isfinite(tmp_xyz[2])) {
        R[3] = dead_record_d();
        return;
    }
    mv4(fr.P, tmp_xyz, new_xyz);
    new_xyz[0] = new_xyz[0] / new_xyz[3];
    new_xyz[1] = new_xyz[1] / new_xyz[3];
    new_xyz[2] = new_xyz[2] / new_xyz[3];
    if (!isfinite(new_xyz[0]) || !isfinite(new_xyz[1]) || !isfinite(new_xyz[2]) ||
        tmp_xyz[2] >= -fr.znear || new_xyz[2] < -1.0f || new_xyz[2] > 1.0f) {
        R[3] = dead_record_d();
        return;
    }

    // ---- 2D covariance (render.cu:655-686) ----
    const float X = tmp_xyz[0], Y = tmp_xyz[1], Z = tmp_xyz[2];
    const float fx = fr.fx, fy = fr.fy;
    float jac[6], jacT[6];
    jac[0] = fx / Z; jac[1] = 0.0f;
    jac[2] = -fx * X / (Z * Z); jac[3] = 0.0f;
    jac[4] = fy / Z; jac[5] = -fy * Y / (Z * Z);
    jacT[0] = jac[0]; jacT[1] = jac[3]; jacT[2] = jac[1];
    jacT[3] = jac[4]; jacT[4] = jac[2]; jacT[5] = jac[5];

    // buildRotMatFromQuat_cuda (math.cu:153-164)
    float qw = arr[(GSR_A_ROT0 + 0) * stride + i];
    float qx = arr[(GSR_A_ROT0 + 1) * stride + i];
    float qy = arr[(GSR_A_ROT0 + 2) * stride + i];
    float qz = arr[(GSR_A_ROT0 + 3) * stride + i];
    const float qn = sqrtf(qx * qx + qy * qy + qz * qz + qw * qw);
    qx /= qn; qy /= qn; qz /= qn; qw /= qn;
    float Rm[9], RT[9], S[9], tmp[9], cov[9];
    Rm[0] = 1 - 2 * qy * qy - 2 * qz * qz; Rm[1] = 2 * qx * qy - 2 * qw * qz;     Rm[2] = 2 * qx * qz + 2 * qw * qy;
    Rm[3] = 2 * qx * qy + 2 * qw * qz;     Rm[4] = 1 - 2 * qx * qx - 2 * qz * qz; Rm[5] = 2 * qy * qz - 2 * qw * qx;
    Rm[6] = 2 * qx * qz - 2 * qw * qy;     Rm[7] = 2 * qy * qz + 2 * qw * qx;     Rm[8] = 1 - 2 * qx * qx - 2 * qy * qy;
    RT[0] = Rm[0]; RT[1] = Rm[3]; RT[2] = Rm[6];
    RT[3] = Rm[1]; RT[4] = Rm[4]; RT[5] = Rm[7];
    RT[6] = Rm[2]; RT[7] = Rm[5]; RT[8] = Rm[8];
    const float scale_mod = 1.0f;
    S[0] = scale_mod * arr[(GSR_A_SCALE0 + 0) * stride + i]; S[1] = 0.0f; S[2] = 0.0f;
    S[3] = 0.0f; S[4] = scale_mod * arr[(GSR_A_SCALE0 + 1) * stride + i]; S[5] = 0.0f;
    S[6] = 0.0f; S[7] = 0.0f; S[8] = scale_mod * arr[(GSR_A_SCALE0 + 2) * stride + i];
    mm3(Rm, S, tmp);
    mm3(tmp, S, Rm);
    mm3(Rm, RT, cov);
    mm3(fr.Rc, cov, tmp);
    mm3(tmp, fr.RcT, cov);
    gemm<2, 3, 3>(jac, cov, tmp);
    float S2[4];
    gemm<2, 2, 3>(tmp, jacT, S2);
    const int W = fr.W, H = fr.H;
    S2[0] = (W * 0.5f) * (W * 0.5f) * S2[0];
    S2[1] = (W * 0.5f) * (H * 0.5f) * S2[1];
    S2[2] = (H * 0.5f) * (W * 0.5f) * S2[2];
    S2[3] = (H * 0.5f) * (H * 0.5f) * S2[3];
    const float det = S2[0] * S2[3] - S2[1] * S2[2];
    if (!isfinite(det) || det < 1e-8f) {                        // render.cu:690
        R[3] = dead_record_d();
        return;
    }
    const float invDet = 1.0f / det;
    const float ic0 = S2[3] * invDet, ic1 = -S2[1] * invDet;
    const float ic2 = -S2[2] * invDet, ic3 = S2[0] * invDet;

    // ---- extent (render.cu:704-764) ----
    const float sxy = 0.5f * (S2[1] + S2[2]);
    const float tr = S2[0] + S2[3];
    const float dif = S2[0] - S2[3];
    const float rad = sqrtf(fmaxf(0.0f, dif * dif + 4 * sxy * sxy));
    float l1 = 0.5f * (tr + rad);
    float l2 = 0.5f * (tr - rad);
    l1 = fmaxf(l1, 1e-8f);
    l2 = fmaxf(l2, 1e-8f);
    const float theta = 0.5f * gsr_atan2f(2 * sxy, dif);
    const float r1 = fr.k * sqrtf(l1);
    const float r2 = fr.k * sqrtf(l2);
    const float c = gsr_cosf(theta);
    const float sn = gsr_sinf(theta);
    float ex = fabsf(r1 * c) + fabsf(r2 * sn);
    float ey = fabsf(r1 * sn) + fabsf(r2 * c);
    ex /= W / 2.0f;
    ey /= H / 2.0f;
    float xmin = new_xyz[0] - ex, xmax = new_xyz[0] + ex;
    float ymin = new_xyz[1] - ey, ymax = new_xyz[1] + ey;
    if (xmax < -0.99f || xmin > 0.99f || ymax < -0.99f || ymin > 0.99f) {   // render.cu:737
        R[3] = dead_record_d();
        return;
    }
    xmin = fmaxf(xmin, -1.0f);
    xmax = fminf(xmax, 1.0f);
    ymin = fmaxf(ymin, -1.0f);
    ymax = fminf(ymax, 1.0f);
    const int xmin_px = gsr_f2i_sat(floorf(((xmin + 1.0f) * 0.5f) * W));
    const int xmax_px = gsr_f2i_sat(ceilf(((xmax + 1.0f) * 0.5f) * W));
    const int ymin_px = gsr_f2i_sat(floorf(((ymin + 1.0f) * 0.5f) * H));
    const int ymax_px = gsr_f2i_sat(ceilf(((ymax + 1.0f) * 0.5f) * H));
    const int px_x = gsr_f2i_sat(roundf(((new_xyz[0] + 1.0f) * 0.5f) * W));
    const int px_y = gsr_f2i_sat(roundf(((new_xyz[1] + 1.0f) * 0.5f) * H));
    const uint32_t key = gsr_f2u_sat(-Z * 1e6f);                // render.cu:850

    // internal GSR_TILE_PX tiles covered (output is tile-invariant)
    const int tx0 = xmin_px / GSR_TILE_PX;
    const int tx1 = min(fr.tiles_x - 1, xmax_px / GSR_TILE_PX);
    const int ty0 = ymin_px / GSR_TILE_PX;
    const int ty1 = min(fr.tiles_y - 1, ymax_px / GSR_TILE_PX);
    const uint32_t count = (uint32_t)((tx1 - tx0 + 1) * (ty1 - ty0 + 1));

    // ---- SH colour, bands 0..2 (render.cu:500-534), only for survivors ----
    float dir[3] = {gx - fr.campos[0], gy - fr.campos[1], gz - fr.campos[2]};
    {
        const float nn = sqrtf(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);  // math.cu:7-18
        if (nn > 1e-8f) {
            dir[0] /= nn; dir[1] /= nn; dir[2] /= nn;
        } else {
            dir[0] = 0.0f; dir[1] = 0.0f; dir[2] = 0.0f;
        }
    }
    const float x = dir[0], y = dir[1], z = dir[2];
    const float xx = x * x, yy = y * y, zz = z * z;
    const float xy = x * y, yz = y * z, xz = x * z;
    const float C2_0 = 1.0925484305920792f, C2_1 = -1.0925484305920792f, C2_2 = 0.31539156525252005f,
                C2_3 = -1.0925484305920792f, C2_4 = 0.5462742152960396f;
    float col[3];
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
        const float* sh = arr + (GSR_A_SH0 + ch) * stride + i;   // sh[ch], sh[3+ch], ...
        float cc = sh[0] * kShC0;
        cc += kShC1 * z * sh[6 * stride];
        cc -= kShC1 * y * sh[3 * stride];
        cc -= kShC1 * x * sh[9 * stride];
        cc += C2_0 * xy * sh[12 * stride];
        cc += C2_1 * yz * sh[15 * stride];
        cc += C2_2 * (2.0f * zz - xx - yy) * sh[18 * stride];
        cc += C2_3 * xz * sh[21 * stride];
        cc += C2_4 * (xx - yy) * sh[24 * stride];
        cc += 0.5f;
        col[ch] = fminf(fmaxf(cc, 0.0f), 1.0f);
    }
    const float opacity = arr[GSR_A_OPACITY * stride + i];

    R[0] = make_uint4(__float_as_uint(ic0), __float_as_uint(ic1), __float_as_uint(ic2), __float_as_uint(ic3));
    R[1] = make_uint4(__float_as_uint(opacity), __float_as_uint(col[0]), __float_as_uint(col[1]),
                      __float_as_uint(col[2]));
    R[2] = make_uint4((uint32_t)px_x, (uint32_t)px_y, (uint32_t)xmin_px | ((uint32_t)xmax_px << 16),
                      (uint32_t)ymin_px | ((uint32_t)ymax_px << 16));
    R[3] = make_uint4((uint32_t)tx0 | ((uint32_t)tx1 << 16), (uint32_t)ty0 | ((uint32_t)ty1 << 16), count, key);
    items[i] = ((uint64_t)key << 32) | (uint64_t)(uint32_t)i;
}

// ------------------------------------------------------------------ radix sort
//
// Stable LSD pass, reduce-then-scan (no inter-workgroup spin waits, so no
// forward-progress assumption): upsweep histograms per workgroup chunk,
// per-digit scan over workgroups, downsweep that ranks each 4096-item tile with
// wave64 ballot matching (the AMD stand-in for __match_any), scatters into LDS
// in digit order and writes runs out coalesced.

template <int ITEMS>
__global__ __launch_bounds__(kSortThreads) void k_radix_upsweep(const uint64_t* __restrict__ in,
                                                                const uint32_t* __restrict__ n_dev,
                                                                uint32_t n_host, int shift, uint32_t mask,
                                                                int groups, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[4][256];
    const uint32_t t = threadIdx.x;
    const uint32_t w = t >> 6;
#pragma unroll
    for (int k = 0; k < 4; k++) h[k][t] = 0;
    __syncthreads();
    const uint64_t n = n_dev ? (uint64_t)*n_dev : (uint64_t)n_host;
    uint64_t b, e;
    chunk_range(n, groups, blockIdx.x, kSortThreads * ITEMS, b, e);
    uint64_t i = b + t;
    for (; i + 3 * kSortThreads < e; i += 4 * kSortThreads) {
        const uint64_t v0 = in[i], v1 = in[i + kSortThreads], v2 = in[i + 2 * kSortThreads],
                       v3 = in[i + 3 * kSortThreads];
        atomicAdd(&h[w][(uint32_t)(v0 >> shift) & mask], 1u);
        atomicAdd(&h[w][(uint32_t)(v1 >> shift) & mask], 1u);
        atomicAdd(&h[w][(uint32_t)(v2 >> shift) & mask], 1u);
        atomicAdd(&h[w][(uint32_t)(v3 >> shift) & mask], 1u);
    }
    for (; i < e; i += kSortThreads) atomicAdd(&h[w][(uint32_t)(in[i] >> shift) & mask], 1u);
    __syncthreads();
    hist[t * (uint32_t)groups + blockIdx.x] = h[0][t] + h[1][t] + h[2][t] + h[3][t];
}

// One workgroup per digit: exclusive scan of hist[d][0..groups) in place.
__global__ __launch_bounds__(256) void k_radix_scan(uint32_t* __restrict__ hist, int groups,
                                                     uint32_t* __restrict__ totals) {
    __shared__ uint32_t scratch[4];
    uint32_t* row = hist + (size_t)blockIdx.x * groups;
    const int per = (groups + 255) / 256;
    const int b = threadIdx.x * per;
    uint32_t local = 0;
    for (int k = 0; k < per; k++)
        if (b + k < groups) local += row[b + k];
    uint32_t total;
    uint32_t run = block_exclusive_scan<uint32_t>(local, scratch, total);
    for (int k = 0; k < per; k++)
        if (b + k < groups) {
            const uint32_t v = row[b + k];
            row[b + k] = run;
            run += v;
        }
    if (threadIdx.x == 0) totals[blockIdx.x] = total;
}

template <int ITEMS>
__global__ __launch_bounds__(kSortThreads) void k_radix_downsweep(
    const uint64_t* __restrict__ in, uint64_t* __restrict__ out, const uint32_t* __restrict__ n_dev,
    uint32_t n_host, int shift, int bits, int groups, const uint32_t* __restrict__ hist,
    const uint32_t* __restrict__ totals, uint2* __restrict__ ranges) {
    constexpr int kTile = kSortThreads * ITEMS;
    __shared__ uint64_t s_items[kTile];
    __shared__ uint32_t s_wc[4][256];           // per-wave digit counters, then wave bases
    __shared__ uint32_t s_gbase[256];           // running global offset per digit
    __shared__ uint32_t s_lbase[256];           // tile-local exclusive base per digit
    __shared__ uint32_t s_scr[4];
    const uint32_t t = threadIdx.x;
    const uint32_t lane = lane_id();
    const uint32_t w = t >> 6;
    const uint32_t mask = (1u << bits) - 1u;
    const uint64_t n = n_dev ? (uint64_t)*n_dev : (uint64_t)n_host;
    uint64_t b, e;
    chunk_range(n, groups, blockIdx.x, kTile, b, e);
    if (b >= e) return;                          // uniform per workgroup

    // global base of each digit for this workgroup
    {
        uint32_t tot;
        const uint32_t dig_excl = block_exclusive_scan<uint32_t>(totals[t], s_scr, tot);
        s_gbase[t] = dig_excl + hist[t * (uint32_t)groups + blockIdx.x];
    }
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

    for (uint64_t tb = b; tb < e; tb += kTile) {
        const uint32_t tn = (uint32_t)min((uint64_t)kTile, e - tb);
#pragma unroll
        for (int k = 0; k < 4; k++) s_wc[k][t] = 0;
        __syncthreads();

        uint64_t it[ITEMS];
        uint32_t rk[ITEMS];
        const uint32_t wbase = w * 64 * ITEMS;
#pragma unroll
        for (int k = 0; k < ITEMS; k++) {
            const uint32_t el = wbase + k * 64 + lane;
            it[k] = (el < tn) ? in[tb + el] : 0ull;
        }
#pragma unroll
        for (int k = 0; k < ITEMS; k++) {
            const uint32_t el = wbase + k * 64 + lane;
            const bool valid = el < tn;
            const uint32_t d = (uint32_t)(it[k] >> shift) & mask;
            uint64_t peers = __ballot(valid);
            for (int bit = 0; bit < bits; bit++) {
                const bool on = (d >> bit) & 1u;
                const uint64_t bm = __ballot(on);
                peers &= on ? bm : ~bm;
            }
            uint32_t r = 0;
            if (valid) {
                const uint32_t before = s_wc[w][d];
                r = before + (uint32_t)__popcll(peers & lt_mask);
                if ((uint32_t)(__ffsll((unsigned long long)peers) - 1) == lane)
                    s_wc[w][d] = before + (uint32_t)__popcll(peers);
            }
            rk[k] = r;
        }
        __syncthreads();
        // per digit t: exclusive prefix over the four waves, tile count, tile-local base
        uint32_t tcount;
        {
            const uint32_t c0 = s_wc[0][t], c1 = s_wc[1][t], c2 = s_wc[2][t], c3 = s_wc[3][t];
            s_wc[0][t] = 0;
            s_wc[1][t] = c0;
            s_wc[2][t] = c0 + c1;
            s_wc[3][t] = c0 + c1 + c2;
            tcount = c0 + c1 + c2 + c3;
            uint32_t tot;
            s_lbase[t] = block_exclusive_scan<uint32_t>(tcount, s_scr, tot);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < ITEMS; k++) {
            const uint32_t el = wbase + k * 64 + lane;
            if (el < tn) {
                const uint32_t d = (uint32_t)(it[k] >> shift) & mask;
                s_items[s_lbase[d] + s_wc[w][d] + rk[k]] = it[k];
            }
        }
        __syncthreads();
        for (uint32_t q = t; q < tn; q += kSortThreads) {
            const uint64_t v = s_items[q];
            const uint32_t d = (uint32_t)(v >> shift) & mask;
            const uint32_t dst = s_gbase[d] + (q - s_lbase[d]);
            out[dst] = v;
            if (ranges) {
                // final pass of the tile sort: the LDS tile is fully sorted, so each
                // run of one tile key is contiguous; record its global [start, end)
                // as {~start, end} with atomicMax, so a zeroed array means "empty"
                // (replaces a separate boundary-detection kernel).
                const uint32_t key = (uint32_t)(v >> 32);
                if (q == 0 || (uint32_t)(s_items[q - 1] >> 32) != key) atomicMax(&ranges[key].x, ~dst);
                if (q == tn - 1 || (uint32_t)(s_items[q + 1] >> 32) != key) atomicMax(&ranges[key].y, dst + 1);
            }
        }
        __syncthreads();
        s_gbase[t] += tcount;
        // next iteration's first barrier orders this update before its use
    }
}

// ------------------------------------------------------------------ emission

__global__ __launch_bounds__(256) void k_emit_count(const uint64_t* __restrict__ sorted, uint32_t n,
                                                     const uint4* __restrict__ rec, int groups,
                                                     unsigned long long* __restrict__ wg_sum) {
    __shared__ unsigned long long scr[4];
    uint64_t b, e;
    chunk_range(n, groups, blockIdx.x, 256, b, e);
    unsigned long long s = 0;
    for (uint64_t j = b + threadIdx.x; j < e; j += 256) {
        const uint32_t i = (uint32_t)sorted[j];
        s += rec[4 * (uint64_t)i + 3].z;
    }
    unsigned long long tot;
    block_exclusive_scan<unsigned long long>(s, scr, tot);
    if (threadIdx.x == 0) wg_sum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void k_emit_scan(unsigned long long* __restrict__ wg, int groups,
                                                    uint32_t cap, Stats* __restrict__ st,
                                                    Stats* host_st) {
    __shared__ unsigned long long scr[4];
    const int per = (groups + 255) / 256;
    const int b = threadIdx.x * per;
    unsigned long long local = 0;
    for (int k = 0; k < per; k++)
        if (b + k < groups) local += wg[b + k];
    unsigned long long total;
    unsigned long long run = block_exclusive_scan<unsigned long long>(local, scr, total);
    for (int k = 0; k < per; k++)
        if (b + k < groups) {
            const unsigned long long v = wg[b + k];
            wg[b + k] = run;
            run += v;
        }
    if (threadIdx.x == 0) {
        Stats s;
        s.pairs_total = total;
        s.pairs_eff = (uint32_t)(total < cap ? total : cap);
        s.overflow = total > cap ? 1u : 0u;
        st[0] = s;
        // st[1]: sticky record (max P, overflow seen) until the host clears it
        Stats k = st[1];
        if (s.pairs_total > k.pairs_total) k.pairs_total = s.pairs_total;
        k.pairs_eff = s.pairs_eff;
        k.overflow |= s.overflow;
        st[1] = k;
        if (host_st) {
            host_st->pairs_total = k.pairs_total;
            host_st->pairs_eff = k.pairs_eff;
            host_st->overflow = k.overflow;
            __threadfence_system();
        }
    }
}

__global__ __launch_bounds__(256) void k_emit_pairs(const uint64_t* __restrict__ sorted, uint32_t n,
                                                     const uint4* __restrict__ rec, int groups,
                                                     const unsigned long long* __restrict__ wg_base,
                                                     uint32_t cap, int tiles_x,
                                                     uint64_t* __restrict__ pairs) {
    __shared__ unsigned long long scr[4];
    uint64_t b, e;
    chunk_range(n, groups, blockIdx.x, 256, b, e);
    unsigned long long run = wg_base[blockIdx.x];
    for (uint64_t rb = b; rb < e; rb += 256) {
        const uint64_t j = rb + threadIdx.x;
        uint32_t cnt = 0, i = 0;
        uint4 D = make_uint4(0, 0, 0, 0);
        if (j < e) {
            i = (uint32_t)sorted[j];
            D = rec[4 * (uint64_t)i + 3];
            cnt = D.z;
        }
        unsigned long long tot;
        unsigned long long pos = run + block_exclusive_scan<unsigned long long>(cnt, scr, tot);
        if (cnt) {
            const uint32_t tx0 = D.x & 0xffffu, tx1 = D.x >> 16;
            const uint32_t ty0 = D.y & 0xffffu, ty1 = D.y >> 16;
            for (uint32_t ty = ty0; ty <= ty1; ty++)
                for (uint32_t tx = tx0; tx <= tx1; tx++) {
                    if (pos < cap) pairs[pos] = ((uint64_t)(ty * (uint32_t)tiles_x + tx) << 32) | i;
                    pos++;
                }
        }
        run += tot;
    }
}

// ------------------------------------------------------------------ blend


// Bijective XCD-aware remap: blocks that share an XCD (b % 8) get one
// contiguous run of tiles, so neighbouring tiles' shared splats hit one L2.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int xcd = b & 7, q = nb >> 3, r = nb & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// md2 cutoff of one splat: alpha = fminf(op * exp(-md2/2), 0.99) < 1e-3 holds
// for every md2 > 2 ln(1000 op) (exp and the product are within a few ulp), so
// lanes beyond the returned bound can never composite.  The bound is padded by
// 1e-5 relative + 1e-3 absolute — orders of magnitude above the rounding of
// gsr_expf, the product and the hardware log2 used here — and is NaN (never
// skip) for NaN opacity, +inf for infinite opacity, -inf for op <= 0.  It only
// decides whether a wave may SKIP work; it never changes a composited value.
__device__ __forceinline__ float md2_cutoff(float op) {
    const float l = __log2f(op * 1000.0f);                   // v_log_f32
    return (l * 1.38629436111989061f) * 1.00001f + 1e-3f;     // 2 ln2 log2(1000 op)
}

// Can any pixel of an integer rectangle reach md2 <= cut?  dx0..dy1 bound the
// (float)pixel - (float)centre offsets of the rectangle's pixels (monotone, so
// every pixel's dx lies in [dx0, dx1]).  Returns false only when the exact
// minimum of the quadratic form a dx^2 + (b+c) dx dy + e dy^2 over that
// rectangle exceeds cut by more than a bound on the float rounding of md2
// (<= ~6 ulp of |a|dx^2 + (|b|+|c|)|dx dy| + |e|dy^2, padded 10x) — so a culled
// splat could never have composited onto this block.  Not positive definite
// (robustly), NaN or inf inputs: never culled.
__device__ __forceinline__ bool block_may_reach(float a, float b, float c, float e, float dx0, float dx1,
                                                float dy0, float dy1, float cut) {
    if (dx0 <= 0.0f && dx1 >= 0.0f && dy0 <= 0.0f && dy1 >= 0.0f) return true;
    const float h = 0.5f * (b + c);
    const float det = a * e - h * h;
    if (!(a > 0.0f && e > 0.0f && det > 1e-4f * (a * e)) || !(cut < 3.0e38f)) return true;
    const float ih = -h / e, iv = -h / a;
    auto q = [&](float x, float y) { return a * x * x + 2.0f * h * x * y + e * y * y; };
    float qm = q(dx0, fminf(fmaxf(ih * dx0, dy0), dy1));
    qm = fminf(qm, q(dx1, fminf(fmaxf(ih * dx1, dy0), dy1)));
    qm = fminf(qm, q(fminf(fmaxf(iv * dy0, dx0), dx1), dy0));
    qm = fminf(qm, q(fminf(fmaxf(iv * dy1, dx0), dx1), dy1));
    const float M = fmaxf(fmaxf(fabsf(dx0), fabsf(dx1)), fmaxf(fabsf(dy0), fabsf(dy1)));
    const float err = 4e-6f * (fabsf(a) + fabsf(b) + fabsf(c) + fabsf(e)) * M * M + 1e-3f;
    return !(qm - err > cut);
}

// One wave64 per 8x8 pixel block, four per 16x16 tile (one tile per 256-thread
// workgroup), and NO workgroup barrier: each wave streams its tile's splat list
// on its own in 64-record batches (lane l holds record l of the batch), with
// the next batch's pair indices and records prefetched into registers while the
// current one is composited, and a private LDS slice for the broadcast reads.
template <bool DIAG>
__global__ __launch_bounds__(256) void k_blend_v5(const uint64_t* __restrict__ pairs,
                                                const uint2* __restrict__ ranges,
                                                const uint4* __restrict__ rec, int tiles_x, int tiles_y,
                                                int W, int H, int cover_w, int cover_h,
                                                float* __restrict__ out,
                                                unsigned long long* __restrict__ counters) {
    __shared__ uint4 sA[4][64], sB[4][64], sC[4][64];
    __shared__ float sCut[4][64];
    const int ntiles = tiles_x * tiles_y;
    const int tile = xcd_remap(blockIdx.x, ntiles);
    const int tx = tile % tiles_x, ty = tile / tiles_x;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int bx = tx * GSR_TILE_PX + (w & 1) * 8;
    const int by = ty * GSR_TILE_PX + (w >> 1) * 8;
    const int px = bx + (lane & 7), py = by + (lane >> 3);
    const bool inside = px < cover_w && py < cover_h;
    const float fpx = (float)px, fpy = (float)py;
    // transmittance; a pixel is saturated ("done", render.cu:328) iff T < 1e-3.
    // Pixels outside the covered area start saturated (T = 0) and write 0.
    float T = inside ? 1.0f : 0.0f;
    float cr = 0.0f, cg = 0.0f, cb = 0.0f;
    const uint2 rr = ranges[tile];                       // {~start, end}, zero = empty
    const uint32_t beg = rr.y ? ~rr.x : 0u, end = rr.y;
    uint64_t d_loaded = 0, d_iter = 0, d_active = 0, d_taken = 0, d_skipped = 0;
    uint4* wA = sA[w];
    uint4* wB = sB[w];
    uint4* wC = sC[w];
    float* wCut = sCut[w];

    // software pipeline: records of batch k in (ra, rb, rc); pair index of batch k+1 in nidx
    uint4 ra = make_uint4(0, 0, 0, 0), rb = ra, rc = ra;
    uint32_t nidx = 0;
    if (beg + lane < end) {
        const uint32_t gi = (uint32_t)pairs[beg + lane];
        const uint4* R = rec + 4 * (uint64_t)gi;
        ra = R[0];
        rb = R[1];
        rc = R[2];
    }
    if (beg + 64 + lane < end) nidx = (uint32_t)pairs[beg + 64 + lane];
    bool alive = __ballot(!(T < 1e-3f)) != 0ull;
    for (uint32_t base = beg; base < end && alive; base += 64) {
        const uint32_t cnt = min(64u, end - base);
        // stage the current batch in this wave's LDS slice (same-wave LDS ops are in order)
        wA[lane] = ra;
        wB[lane] = rb;
        wC[lane] = rc;
        wCut[lane] = md2_cutoff(__uint_as_float(rb.x));
        // cull: lane = record; AABB vs block, then exact ellipse test on block n AABB
        bool h = false;
        if ((uint32_t)lane < cnt) {
            const int xmin = (int)(rc.z & 0xffffu), xmax = (int)(rc.z >> 16);
            const int ymin = (int)(rc.w & 0xffffu), ymax = (int)(rc.w >> 16);
            h = !(xmax < bx || xmin > bx + 7 || ymax < by || ymin > by + 7);
            if (h) {
                const float cx = (float)(int)rc.x, cy = (float)(int)rc.y;
                h = block_may_reach(__uint_as_float(ra.x), __uint_as_float(ra.y), __uint_as_float(ra.z),
                                    __uint_as_float(ra.w), (float)max(bx, xmin) - cx, (float)min(bx + 7, xmax) - cx,
                                    (float)max(by, ymin) - cy, (float)min(by + 7, ymax) - cy,
                                    md2_cutoff(__uint_as_float(rb.x)));
            }
        }
        uint64_t m = __ballot(h);
        if (DIAG) d_loaded += cnt;
        // prefetch: records of batch k+1 (indices already in nidx), indices of batch k+2
        if (base + 64 + lane < end) {
            const uint4* R = rec + 4 * (uint64_t)nidx;
            ra = R[0];
            rb = R[1];
            rc = R[2];
        }
        if (base + 128 + lane < end) nidx = (uint32_t)pairs[base + 128 + lane];
        while (m && alive) {
            // two splats per iteration: their md2/exp are independent (ILP);
            // compositing stays strictly in list order, per pixel
            const int s0 = __builtin_ctzll(m);
            m &= m - 1;
            const bool has1 = m != 0ull;
            const int s1 = has1 ? __builtin_ctzll(m) : s0;
            if (has1) m &= m - 1;
            const uint4 C0 = wC[s0], C1 = wC[s1];
            const uint4 A0 = wA[s0], A1 = wA[s1];
            const float cut0 = wCut[s0], cut1 = wCut[s1];
            const bool box0 = (px >= (int)(C0.z & 0xffffu)) & (px <= (int)(C0.z >> 16)) &
                              (py >= (int)(C0.w & 0xffffu)) & (py <= (int)(C0.w >> 16));
            const bool box1 = (px >= (int)(C1.z & 0xffffu)) & (px <= (int)(C1.z >> 16)) &
                              (py >= (int)(C1.w & 0xffffu)) & (py <= (int)(C1.w >> 16)) & has1;
            // render.cu:329-332, same operation order
            const float dx0 = fpx - (float)(int)C0.x, dy0 = fpy - (float)(int)C0.y;
            const float dx1 = fpx - (float)(int)C1.x, dy1 = fpy - (float)(int)C1.y;
            const float md0 = dx0 * (__uint_as_float(A0.x) * dx0 + __uint_as_float(A0.y) * dy0) +
                              dy0 * (__uint_as_float(A0.z) * dx0 + __uint_as_float(A0.w) * dy0);
            const float md1 = dx1 * (__uint_as_float(A1.x) * dx1 + __uint_as_float(A1.y) * dy1) +
                              dy1 * (__uint_as_float(A1.z) * dx1 + __uint_as_float(A1.w) * dy1);
            const bool unsat = !(T < 1e-3f);
            if (DIAG) {
                d_iter += has1 ? 2 : 1;
                d_active += (uint64_t)__popcll(__ballot(box0 & unsat)) + (uint64_t)__popcll(__ballot(box1 & unsat));
            }
            // no lane can reach alpha >= 1e-3 for either splat: skip both
            if (__ballot(unsat & ((box0 & !(md0 > cut0)) | (box1 & !(md1 > cut1)))) == 0ull) {
                if (DIAG) d_skipped += has1 ? 2 : 1;
                continue;
            }
            const uint4 B0 = wB[s0], B1 = wB[s1];
            const float e0 = gsr_expf(-0.5f * md0);
            const float e1 = gsr_expf(-0.5f * md1);
            {   // splat s0 (render.cu:333-340)
                float alpha = __uint_as_float(B0.x) * e0;
                alpha = fminf(alpha, 0.99f);
                const bool take = box0 & unsat & !(alpha < 1e-3f);
                const float wr = __uint_as_float(B0.y) * alpha * T;
                const float wg = __uint_as_float(B0.z) * alpha * T;
                const float wb = __uint_as_float(B0.w) * alpha * T;
                const float Tn = T * (1.0f - alpha);
                cr = take ? cr + wr : cr;
                cg = take ? cg + wg : cg;
                cb = take ? cb + wb : cb;
                T = take ? Tn : T;
                if (DIAG) d_taken += (uint64_t)__popcll(__ballot(take));
            }
            {   // splat s1, against the transmittance left by s0
                float alpha = __uint_as_float(B1.x) * e1;
                alpha = fminf(alpha, 0.99f);
                const bool take = box1 & !(T < 1e-3f) & !(alpha < 1e-3f);
                const float wr = __uint_as_float(B1.y) * alpha * T;
                const float wg = __uint_as_float(B1.z) * alpha * T;
                const float wb = __uint_as_float(B1.w) * alpha * T;
                const float Tn = T * (1.0f - alpha);
                cr = take ? cr + wr : cr;
                cg = take ? cg + wg : cg;
                cb = take ? cb + wb : cb;
                T = take ? Tn : T;
                if (DIAG) d_taken += (uint64_t)__popcll(__ballot(take));
            }
            alive = __ballot(!(T < 1e-3f)) != 0ull;   // whole block saturated -> stop
        }
    }
    if (DIAG && lane == 0) {
        if (w == 0 && d_loaded) atomicAdd(counters, (unsigned long long)d_loaded);
        atomicAdd(counters + 1, (unsigned long long)d_iter);
        atomicAdd(counters + 2, (unsigned long long)d_active);
        atomicAdd(counters + 3, (unsigned long long)d_taken);
        atomicAdd(counters + 5, (unsigned long long)d_skipped);
        atomicAdd(counters + 6, (unsigned long long)(d_iter * 64));
    }
    if (px < W && py < H) {
        const size_t o = (size_t)py * (size_t)W + (size_t)px;
        const size_t hw = (size_t)W * (size_t)H;
        out[o] = inside ? cr : 0.0f;
        out[hw + o] = inside ? cg : 0.0f;
        out[2 * hw + o] = inside ? cb : 0.0f;
    }
}

typedef float f2 __attribute__((ext_vector_type(2)));

// gsr_expf on two lanes at once (v_pk_* for every float op that has a packed
// form), for inputs the caller has PROVEN finite and <= 88.75: there the upper
// clamp and the NaN select of gsr_expf are no-ops, and every remaining step is
// the same IEEE operation in the same order, so each half is bit-identical to
// gsr_expf of that half.
__device__ __forceinline__ f2 gsr_expf_x2(f2 x) {
    f2 xc;
    xc.x = fmaxf(x.x, -104.0f);
    xc.y = fmaxf(x.y, -104.0f);
    const f2 t = xc * 1.44269504088896341f;
    f2 n;
    n.x = rintf(t.x);
    n.y = rintf(t.y);
    f2 r = __builtin_elementwise_fma(-n, (f2)0.693359375f, xc);
    r = __builtin_elementwise_fma(-n, (f2)-2.12194440e-4f, r);
    f2 p = __builtin_elementwise_fma((f2)1.9875691500e-4f, r, (f2)1.3981999507e-3f);
    p = __builtin_elementwise_fma(p, r, (f2)8.3334519073e-3f);
    p = __builtin_elementwise_fma(p, r, (f2)4.1665795894e-2f);
    p = __builtin_elementwise_fma(p, r, (f2)1.6666665459e-1f);
    p = __builtin_elementwise_fma(p, r, (f2)5.0000001201e-1f);
    const f2 r2 = r * r;
    const f2 y = __builtin_elementwise_fma(p, r2, r) + 1.0f;
    f2 res;
    res.x = __builtin_amdgcn_ldexpf(y.x, (int)n.x);
    res.y = __builtin_amdgcn_ldexpf(y.y, (int)n.y);
    return res;
}

// Fast-path proof for one splat on one block (exactness, not a heuristic):
// finite conic that is robustly positive definite with |a|+|b|+|c|+|e| times
// the squared largest block offset <= 4e7 keeps every in-box md2 finite and
// >= -10 (float error of the 9-op form < 10), so -md2/2 lies in gsr_expf_x2's
// proven range; finite colours make "alpha = 0 when not taken" leave the
// accumulators bit-identical (c + (col*0)*T == c, T*(1-0) == T).
__device__ __forceinline__ bool fast_safe(float a, float b, float c, float e, float M, float r, float g,
                                          float bl) {
    const float h = 0.5f * (b + c);
    const float S = fabsf(a) + fabsf(b) + fabsf(c) + fabsf(e);
    return a > 0.0f && e > 0.0f && (a * e - h * h) > 1e-4f * (a * e) && S * M * M <= 4e7f &&
           isfinite(S) && isfinite(r) && isfinite(g) && isfinite(bl);
}

// One wave64 per 8x8 pixel block (four per 16x16 tile, one tile per
// workgroup), no workgroup barrier.  Each wave streams its tile's splat list in
// 64-record batches (records of batch k+1 and indices of batch k+2 prefetched
// into registers).  Per batch, lane l culls record l (AABB, then the exact
// ellipse-vs-block test) and computes its 64-bit in-AABB pixel mask; the
// survivors are compacted, in list order, into PAIR SLOTS of the wave's LDS
// slice so that {parameter of splat 2j, parameter of splat 2j+1} are adjacent
// and feed v_pk_* instructions directly.  The compositing loop takes two
// splats per iteration: md2, exp and alpha packed, then the two composites in
// list order.  Batches holding a survivor without the fast-path proof run an
// exact one-splat path instead (same values, full gsr_expf, plain selects).
//
// Pair slot dwords (h = 0 / 1 for the first / second splat of the pair):
//   [0+h] cx  [2+h] cy  [4+h] a  [6+h] b  [8+h] c  [10+h] e  [12+h] opacity
//   [14+2h] red  [15+2h] green  [18+h] blue
template <bool DIAG>
__global__ __launch_bounds__(256) void k_blend(const uint64_t* __restrict__ pairs,
                                                const uint2* __restrict__ ranges,
                                                const uint4* __restrict__ rec, int tiles_x, int tiles_y,
                                                int W, int H, int cover_w, int cover_h,
                                                float* __restrict__ out,
                                                unsigned long long* __restrict__ counters) {
    constexpr int kSlot = 20;                               // dwords per pair slot
    __shared__ float4 sP[4][32 * kSlot / 4];
    const int ntiles = tiles_x * tiles_y;
    const int tile = xcd_remap(blockIdx.x, ntiles);
    const int tx = tile % tiles_x, ty = tile / tiles_x;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int bx = tx * GSR_TILE_PX + (w & 1) * 8;
    const int by = ty * GSR_TILE_PX + (w >> 1) * 8;
    const int px = bx + (lane & 7), py = by + (lane >> 3);
    const bool inside = px < cover_w && py < cover_h;
    const float fpx = (float)px, fpy = (float)py;
    // transmittance; a pixel is saturated ("done", render.cu:328) iff T < 1e-3.
    // Pixels outside the covered area start saturated (T = 0) and write 0.
    float T = inside ? 1.0f : 0.0f;
    f2 crg = (f2)0.0f;
    float cb = 0.0f;
    const uint2 rr = ranges[tile];                          // {~start, end}, zero = empty
    const uint32_t beg = rr.y ? ~rr.x : 0u, end = rr.y;
    uint64_t d_loaded = 0, d_iter = 0, d_active = 0, d_taken = 0, d_slow = 0;
    float* wP = reinterpret_cast<float*>(sP[w]);
    const float4* wP4 = sP[w];

    uint4 ra = make_uint4(0, 0, 0, 0), rb = ra, rc = ra;
    uint32_t nidx = 0;
    if (beg + lane < end) {
        const uint32_t gi = (uint32_t)pairs[beg + lane];
        const uint4* R = rec + 4 * (uint64_t)gi;
        ra = R[0];
        rb = R[1];
        rc = R[2];
    }
    if (beg + 64 + lane < end) nidx = (uint32_t)pairs[beg + 64 + lane];
    bool alive = __ballot(!(T < 1e-3f)) != 0ull;
    for (uint32_t base = beg; base < end && alive; base += 64) {
        const uint32_t cnt = min(64u, end - base);
        // ---- cull + lane masks + compaction (lane = record) ----
        bool hit = false, fast = true;
        uint32_t mlo = 0, mhi = 0;
        if ((uint32_t)lane < cnt) {
            const int xmin = (int)(rc.z & 0xffffu), xmax = (int)(rc.z >> 16);
            const int ymin = (int)(rc.w & 0xffffu), ymax = (int)(rc.w >> 16);
            hit = !(xmax < bx || xmin > bx + 7 || ymax < by || ymin > by + 7);
            if (hit) {
                const float cx = (float)(int)rc.x, cy = (float)(int)rc.y;
                const float a = __uint_as_float(ra.x), b = __uint_as_float(ra.y);
                const float c = __uint_as_float(ra.z), e = __uint_as_float(ra.w);
                const int x0 = max(xmin - bx, 0), x1 = min(xmax - bx, 7);
                const int y0 = max(ymin - by, 0), y1 = min(ymax - by, 7);
                const float dx0 = (float)(bx + x0) - cx, dx1 = (float)(bx + x1) - cx;
                const float dy0 = (float)(by + y0) - cy, dy1 = (float)(by + y1) - cy;
                hit = block_may_reach(a, b, c, e, dx0, dx1, dy0, dy1, md2_cutoff(__uint_as_float(rb.x)));
                const float M = fmaxf(fmaxf(fabsf(dx0), fabsf(dx1)), fmaxf(fabsf(dy0), fabsf(dy1)));
                fast = fast_safe(a, b, c, e, M, __uint_as_float(rb.y), __uint_as_float(rb.z),
                                 __uint_as_float(rb.w));
                // bit (row * 8 + col) of the block: pixel inside the AABB
                const uint32_t rep = ((0xffu >> (7 - (x1 - x0))) << x0) * 0x01010101u;
                const uint64_t rows = (y1 == 7 ? ~0ull : ((1ull << (8 * (y1 + 1))) - 1ull)) & (~0ull << (8 * y0));
                mlo = rep & (uint32_t)rows;
                mhi = rep & (uint32_t)(rows >> 32);
            }
        }
        const uint64_t m = __ballot(hit);
        const bool all_fast = __ballot(hit & !fast) == 0ull;
        if (hit) {
            const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            float* S = wP + (k >> 1) * kSlot;
            const int h = (int)(k & 1u);
            S[0 + h] = (float)(int)rc.x;
            S[2 + h] = (float)(int)rc.y;
            S[4 + h] = __uint_as_float(ra.x);
            S[6 + h] = __uint_as_float(ra.y);
            S[8 + h] = __uint_as_float(ra.z);
            S[10 + h] = __uint_as_float(ra.w);
            S[12 + h] = __uint_as_float(rb.x);
            S[14 + 2 * h] = __uint_as_float(rb.y);
            S[15 + 2 * h] = __uint_as_float(rb.z);
            S[18 + h] = __uint_as_float(rb.w);
        }
        const uint32_t nsurv = (uint32_t)__popcll(m);
        if ((nsurv & 1u) && lane < 10) {
            // odd count: zero the unused second half of the last slot (mask 0 keeps it inert)
            static constexpr int kHalf1[10] = {1, 3, 5, 7, 9, 11, 13, 16, 17, 19};
            wP[(nsurv >> 1) * kSlot + kHalf1[lane]] = 0.0f;
        }
        if (DIAG) d_loaded += cnt;
        // ---- prefetch: records of batch k+1, indices of batch k+2 ----
        if (base + 64 + lane < end) {
            const uint4* R = rec + 4 * (uint64_t)nidx;
            ra = R[0];
            rb = R[1];
            rc = R[2];
        }
        if (base + 128 + lane < end) nidx = (uint32_t)pairs[base + 128 + lane];

        uint64_t mm = m;
        if (all_fast) {
            for (uint32_t j = 0; mm && alive; ++j) {
                const int s0 = __builtin_ctzll(mm);
                mm &= mm - 1;
                const bool has1 = mm != 0ull;
                const int s1 = has1 ? __builtin_ctzll(mm) : s0;
                if (has1) mm &= mm - 1;
                const uint64_t box0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)mhi, s0) << 32) |
                                      (uint32_t)__builtin_amdgcn_readlane((int)mlo, s0);
                uint64_t box1 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)mhi, s1) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)mlo, s1);
                box1 = has1 ? box1 : 0ull;
                const float4 q0 = wP4[j * 5 + 0], q1 = wP4[j * 5 + 1], q2 = wP4[j * 5 + 2];
                const float4 q3 = wP4[j * 5 + 3], q4 = wP4[j * 5 + 4];
                // render.cu:329-332, same operation order, both splats at once
                const f2 dx = (f2)fpx - (f2){q0.x, q0.y};
                const f2 dy = (f2)fpy - (f2){q0.z, q0.w};
                const f2 md = dx * ((f2){q1.x, q1.y} * dx + (f2){q1.z, q1.w} * dy) +
                              dy * ((f2){q2.x, q2.y} * dx + (f2){q2.z, q2.w} * dy);
                const f2 ee = gsr_expf_x2(-0.5f * md);
                const f2 al = (f2){q3.x, q3.y} * ee;
                const float al0 = fminf(al.x, 0.99f), al1 = fminf(al.y, 0.99f);
                // render.cu:333-340: splat 2j, then splat 2j+1 against what 2j left
                const bool in0 = __builtin_amdgcn_inverse_ballot_w64(box0);
                const bool in1 = __builtin_amdgcn_inverse_ballot_w64(box1);
                const bool take0 = in0 & !(T < 1e-3f) & !(al0 < 1e-3f);
                const float a0 = take0 ? al0 : 0.0f;
                const float T1 = T * (1.0f - a0);
                const bool take1 = in1 & !(T1 < 1e-3f) & !(al1 < 1e-3f);
                const float a1 = take1 ? al1 : 0.0f;
                const float T2 = T1 * (1.0f - a1);
                crg = crg + ((f2){q3.z, q3.w} * a0) * T;
                crg = crg + ((f2){q4.x, q4.y} * a1) * T1;
                const f2 wb = ((f2){q4.z, q4.w} * (f2){a0, a1}) * (f2){T, T1};
                cb = (cb + wb.x) + wb.y;
                if (DIAG) {
                    d_iter += has1 ? 2 : 1;
                    d_active += (uint64_t)__popcll(__ballot(in0 & !(T < 1e-3f))) +
                                (uint64_t)__popcll(__ballot(in1 & !(T1 < 1e-3f)));
                    d_taken += (uint64_t)__popcll(__ballot(take0)) + (uint64_t)__popcll(__ballot(take1));
                }
                T = T2;
                alive = __ballot(!(T < 1e-3f)) != 0ull;   // whole block saturated -> stop
            }
        } else {
            // exact one-splat path (render.cu:329-340 with gsr_expf and selects)
            for (uint32_t k = 0; mm && alive; ++k) {
                const int s = __builtin_ctzll(mm);
                mm &= mm - 1;
                const uint64_t box = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)mhi, s) << 32) |
                                     (uint32_t)__builtin_amdgcn_readlane((int)mlo, s);
                const float* S = wP + (k >> 1) * kSlot;
                const int h = (int)(k & 1u);
                const float dx = fpx - S[0 + h], dy = fpy - S[2 + h];
                const float md = dx * (S[4 + h] * dx + S[6 + h] * dy) + dy * (S[8 + h] * dx + S[10 + h] * dy);
                const float ee = gsr_expf(-0.5f * md);
                float alpha = S[12 + h] * ee;
                alpha = fminf(alpha, 0.99f);
                const bool in = __builtin_amdgcn_inverse_ballot_w64(box);
                const bool take = in & !(T < 1e-3f) & !(alpha < 1e-3f);
                const float wr = S[14 + 2 * h] * alpha * T;
                const float wg = S[15 + 2 * h] * alpha * T;
                const float wb = S[18 + h] * alpha * T;
                const float Tn = T * (1.0f - alpha);
                if (DIAG) {
                    d_iter += 1;
                    d_slow += 1;
                    d_active += (uint64_t)__popcll(__ballot(in & !(T < 1e-3f)));
                    d_taken += (uint64_t)__popcll(__ballot(take));
                }
                crg.x = take ? crg.x + wr : crg.x;
                crg.y = take ? crg.y + wg : crg.y;
                cb = take ? cb + wb : cb;
                T = take ? Tn : T;
                alive = __ballot(!(T < 1e-3f)) != 0ull;
            }
        }
    }
    if (DIAG && lane == 0) {
        if (w == 0 && d_loaded) atomicAdd(counters, (unsigned long long)d_loaded);
        atomicAdd(counters + 1, (unsigned long long)d_iter);
        atomicAdd(counters + 2, (unsigned long long)d_active);
        atomicAdd(counters + 3, (unsigned long long)d_taken);
        atomicAdd(counters + 4, (unsigned long long)d_slow);
        atomicAdd(counters + 6, (unsigned long long)(d_iter * 64));
    }
    if (px < W && py < H) {
        const size_t o = (size_t)py * (size_t)W + (size_t)px;
        const size_t hw = (size_t)W * (size_t)H;
        out[o] = inside ? crg.x : 0.0f;
        out[hw + o] = inside ? crg.y : 0.0f;
        out[2 * hw + o] = inside ? cb : 0.0f;
    }
}

// Pixel-chain blend: each lane owns PPL pixels of one column (rows y0 + R*j),
// so one broadcast splat read feeds PPL independent md2/exp/composite chains.
// Block = BW x (R*PPL) pixels per wave; PPL 1: 8x8 (4 waves per 16x16 tile),
// PPL 2: 8x16 (2 waves), PPL 4: 16x16 (1 wave).  One splat per iteration; the
// exact ellipse-vs-block cull of the batch is the only skip.
template <bool DIAG, int PPL>
__global__ __launch_bounds__(256) void k_blend_px(const uint64_t* __restrict__ pairs,
                                                   const uint2* __restrict__ ranges,
                                                   const uint4* __restrict__ rec, int tiles_x, int tiles_y,
                                                   int W, int H, int cover_w, int cover_h,
                                                   float* __restrict__ out,
                                                   unsigned long long* __restrict__ counters) {
    constexpr int BW = PPL == 4 ? 16 : 8;          // block width
    constexpr int R = 64 / BW;                     // rows per pixel pass
    constexpr int BH = R * PPL;                    // block height
    constexpr int WPT = (GSR_TILE_PX / BW) * (GSR_TILE_PX / BH);   // waves per tile
    constexpr int TPB = 256 / (64 * WPT);          // tiles per 256-thread workgroup
    __shared__ uint4 sA[4][64], sB[4][64], sC[4][64];
    const int ntiles = tiles_x * tiles_y;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int tslot = blockIdx.x * TPB + w / WPT;
    if (tslot >= ntiles) return;                   // whole wave exits (no barrier in this kernel)
    const int tile = xcd_remap(tslot, ntiles);
    const int tx = tile % tiles_x, ty = tile / tiles_x;
    const int wt = w % WPT;                        // wave within its tile
    const int bx = tx * GSR_TILE_PX + (wt % (GSR_TILE_PX / BW)) * BW;
    const int by = ty * GSR_TILE_PX + (wt / (GSR_TILE_PX / BW)) * BH;
    const int px = bx + (lane % BW), py0 = by + lane / BW;
    const float fpx = (float)px;
    float T[PPL], cr[PPL], cg[PPL], cb[PPL];
    bool inside[PPL];
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
        inside[j] = px < cover_w && py0 + R * j < cover_h;
        T[j] = inside[j] ? 1.0f : 0.0f;
        cr[j] = cg[j] = cb[j] = 0.0f;
    }
    const uint2 rr = ranges[tile];
    const uint32_t beg = rr.y ? ~rr.x : 0u, end = rr.y;
    uint64_t d_loaded = 0, d_iter = 0, d_active = 0, d_taken = 0;
    uint4* wA = sA[w];
    uint4* wB = sB[w];
    uint4* wC = sC[w];

    uint4 ra = make_uint4(0, 0, 0, 0), rb = ra, rc = ra;
    uint32_t nidx = 0;
    if (beg + lane < end) {
        const uint32_t gi = (uint32_t)pairs[beg + lane];
        const uint4* Rp = rec + 4 * (uint64_t)gi;
        ra = Rp[0];
        rb = Rp[1];
        rc = Rp[2];
    }
    if (beg + 64 + lane < end) nidx = (uint32_t)pairs[beg + 64 + lane];
    auto unsat_any = [&]() {
        bool u = false;
#pragma unroll
        for (int j = 0; j < PPL; ++j) u |= !(T[j] < 1e-3f);
        return __ballot(u) != 0ull;
    };
    bool alive = unsat_any();
    for (uint32_t base = beg; base < end && alive; base += 64) {
        const uint32_t cnt = min(64u, end - base);
        wA[lane] = ra;
        wB[lane] = rb;
        wC[lane] = rc;
        bool h = false;
        if ((uint32_t)lane < cnt) {
            const int xmin = (int)(rc.z & 0xffffu), xmax = (int)(rc.z >> 16);
            const int ymin = (int)(rc.w & 0xffffu), ymax = (int)(rc.w >> 16);
            h = !(xmax < bx || xmin > bx + BW - 1 || ymax < by || ymin > by + BH - 1);
            if (h) {
                const float cx = (float)(int)rc.x, cy = (float)(int)rc.y;
                h = block_may_reach(__uint_as_float(ra.x), __uint_as_float(ra.y), __uint_as_float(ra.z),
                                    __uint_as_float(ra.w), (float)max(bx, xmin) - cx,
                                    (float)min(bx + BW - 1, xmax) - cx, (float)max(by, ymin) - cy,
                                    (float)min(by + BH - 1, ymax) - cy, md2_cutoff(__uint_as_float(rb.x)));
            }
        }
        uint64_t m = __ballot(h);
        if (DIAG) d_loaded += cnt;
        if (base + 64 + lane < end) {
            const uint4* Rp = rec + 4 * (uint64_t)nidx;
            ra = Rp[0];
            rb = Rp[1];
            rc = Rp[2];
        }
        if (base + 128 + lane < end) nidx = (uint32_t)pairs[base + 128 + lane];
        while (m && alive) {
            const int s = __builtin_ctzll(m);
            m &= m - 1;
            const uint4 C = wC[s], A = wA[s], B = wB[s];
            const int xmin = (int)(C.z & 0xffffu), xmax = (int)(C.z >> 16);
            const int ymin = (int)(C.w & 0xffffu), ymax = (int)(C.w >> 16);
            const bool xin = (px >= xmin) & (px <= xmax);
            const float dx = fpx - (float)(int)C.x;
            const float cy = (float)(int)C.y;
            const float a = __uint_as_float(A.x), b = __uint_as_float(A.y);
            const float c = __uint_as_float(A.z), e = __uint_as_float(A.w);
            const float ax = a * dx, cx = c * dx;
            if (DIAG) d_iter += 1;
#pragma unroll
            for (int j = 0; j < PPL; ++j) {
                const int py = py0 + R * j;
                const float dy = (float)py - cy;
                // render.cu:329-340, same operation order
                const float md = dx * (ax + b * dy) + dy * (cx + e * dy);
                const float ee = gsr_expf(-0.5f * md);
                float alpha = __uint_as_float(B.x) * ee;
                alpha = fminf(alpha, 0.99f);
                const bool box = xin & (py >= ymin) & (py <= ymax);
                const bool take = box & !(T[j] < 1e-3f) & !(alpha < 1e-3f);
                const float wr = __uint_as_float(B.y) * alpha * T[j];
                const float wg = __uint_as_float(B.z) * alpha * T[j];
                const float wb = __uint_as_float(B.w) * alpha * T[j];
                const float Tn = T[j] * (1.0f - alpha);
                if (DIAG) {
                    d_active += (uint64_t)__popcll(__ballot(box & !(T[j] < 1e-3f)));
                    d_taken += (uint64_t)__popcll(__ballot(take));
                }
                cr[j] = take ? cr[j] + wr : cr[j];
                cg[j] = take ? cg[j] + wg : cg[j];
                cb[j] = take ? cb[j] + wb : cb[j];
                T[j] = take ? Tn : T[j];
            }
            alive = unsat_any();
        }
    }
    if (DIAG && lane == 0) {
        if (wt == 0 && d_loaded) atomicAdd(counters, (unsigned long long)d_loaded);
        atomicAdd(counters + 1, (unsigned long long)d_iter);
        atomicAdd(counters + 2, (unsigned long long)d_active);
        atomicAdd(counters + 3, (unsigned long long)d_taken);
        atomicAdd(counters + 6, (unsigned long long)(d_iter * 64 * PPL));
    }
    const size_t hw = (size_t)W * (size_t)H;
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
        const int py = py0 + R * j;
        if (px < W && py < H) {
            const size_t o = (size_t)py * (size_t)W + (size_t)px;
            out[o] = inside[j] ? cr[j] : 0.0f;
            out[hw + o] = inside[j] ? cg[j] : 0.0f;
            out[2 * hw + o] = inside[j] ? cb[j] : 0.0f;
        }
    }
}

// ------------------------------------------------------------------ standalone sort ABI helpers

// (u32(key) << 32 | i): the reference sorts int keys as unsigned 8-bit digits
// over all 32 bits (onesweep.cu:190-250, numPasses = 4).
__global__ void k_items_from_keys(const int* __restrict__ keys, uint32_t n, uint64_t* __restrict__ items) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) items[i] = ((uint64_t)(uint32_t)keys[i] << 32) | i;
}

__global__ void k_keys_from_items(const uint64_t* __restrict__ items, uint32_t n, int* __restrict__ keys) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) keys[i] = (int)(uint32_t)(items[i] >> 32);
}

// Stage items for lightWeightGaussian records: (bits [shift, shift+32) of
// radix_id << 32 | position).  src_perm (nullable) maps position -> record.
__global__ void k_items_from_lwg(const gsr_lwg* __restrict__ rec, const uint64_t* __restrict__ src_perm,
                                 uint32_t n, int shift, uint32_t mask, uint64_t* __restrict__ items) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = src_perm ? (uint32_t)src_perm[i] : i;
    const uint32_t k = (uint32_t)(rec[r].radix_id >> shift) & mask;
    items[i] = ((uint64_t)k << 32) | i;
}

__global__ void k_gather_lwg(const gsr_lwg* __restrict__ in, const uint64_t* __restrict__ stage1,
                             const uint64_t* __restrict__ stage2, uint32_t n, gsr_lwg* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t r = (uint32_t)stage2[i];
    if (stage1) r = (uint32_t)stage1[r];
    out[i] = in[r];
}

// ------------------------------------------------------------------ math probe

__global__ void k_math_probe(const float* __restrict__ in, int n, float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = in[2 * i], y = in[2 * i + 1];
    float* o = out + 8 * i;
    o[0] = gsr_expf(x);
    o[1] = gsr_sinf(x);
    o[2] = gsr_cosf(x);
    o[3] = gsr_atan2f(x, y);
    o[4] = sqrtf(x);
    o[5] = x / y;
    o[6] = roundf(x);
    o[7] = __int_as_float(gsr_f2i_sat(x * 1000.0f));
}

inline int grid_for(int64_t n, int block) { return (int)((n + block - 1) / block); }

}  // namespace

// ------------------------------------------------------------------ launchers

hipError_t launch_aos_to_soa(const gsr_gaussian* aos, int64_t n, float* arrays, int64_t stride,
                             hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_aos_to_soa, dim3(grid_for(n, 256)), dim3(256), 0, s, aos, n, arrays, stride);
    return hipGetLastError();
}

hipError_t launch_preprocess(const float* arrays, int64_t stride, int64_t n, const Frame& fr,
                             uint4* rec, uint64_t* items, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_preprocess, dim3(grid_for(n, 256)), dim3(256), 0, s, arrays, stride, n, fr, rec,
                       items);
    return hipGetLastError();
}

template <int ITEMS>
static void radix_pass(const uint64_t* in, uint64_t* out, const uint32_t* n_dev, uint32_t n_host, int shift,
                       int bits, int groups, uint32_t* hist, uint32_t* totals, uint2* ranges, hipStream_t s) {
    const uint32_t mask = (1u << bits) - 1u;
    hipLaunchKernelGGL(k_radix_upsweep<ITEMS>, dim3(groups), dim3(kSortThreads), 0, s, in, n_dev, n_host, shift,
                       mask, groups, hist);
    hipLaunchKernelGGL(k_radix_scan, dim3(256), dim3(256), 0, s, hist, groups, totals);
    hipLaunchKernelGGL(k_radix_downsweep<ITEMS>, dim3(groups), dim3(kSortThreads), 0, s, in, out, n_dev, n_host,
                       shift, bits, groups, hist, totals, ranges);
}

hipError_t launch_radix_pass(const uint64_t* in, uint64_t* out, const uint32_t* n_dev, uint32_t n_host,
                             int shift, int bits, int groups, int items, uint32_t* hist, uint32_t* totals,
                             uint2* ranges, hipStream_t s) {
    if (items == 8)
        radix_pass<8>(in, out, n_dev, n_host, shift, bits, groups, hist, totals, ranges, s);
    else
        radix_pass<16>(in, out, n_dev, n_host, shift, bits, groups, hist, totals, ranges, s);
    return hipGetLastError();
}

hipError_t launch_emit(const uint64_t* depth_sorted, uint32_t n, const uint4* rec, int groups,
                       unsigned long long* wg_scratch, Stats* stats, Stats* host_mapped_stats,
                       uint32_t pair_capacity, int tiles_x, uint64_t* pairs, hipStream_t s) {
    hipLaunchKernelGGL(k_emit_count, dim3(groups), dim3(256), 0, s, depth_sorted, n, rec, groups, wg_scratch);
    hipLaunchKernelGGL(k_emit_scan, dim3(1), dim3(256), 0, s, wg_scratch, groups, pair_capacity, stats,
                       host_mapped_stats);
    hipLaunchKernelGGL(k_emit_pairs, dim3(groups), dim3(256), 0, s, depth_sorted, n, rec, groups, wg_scratch,
                       pair_capacity, tiles_x, pairs);
    return hipGetLastError();
}

template <int PPL>
static void blend_px(const uint64_t* pairs, const uint2* ranges, const uint4* rec, const Frame& fr, float* out,
                     unsigned long long* consumed, hipStream_t s) {
    constexpr int TPB = PPL;   // tiles per 256-thread workgroup (waves per tile = 4 / PPL)
    const int nt = fr.tiles_x * fr.tiles_y;
    const dim3 grid((nt + TPB - 1) / TPB);
    if (consumed)
        hipLaunchKernelGGL((k_blend_px<true, PPL>), grid, dim3(256), 0, s, pairs, ranges, rec, fr.tiles_x,
                           fr.tiles_y, fr.W, fr.H, fr.cover_w, fr.cover_h, out, consumed);
    else
        hipLaunchKernelGGL((k_blend_px<false, PPL>), grid, dim3(256), 0, s, pairs, ranges, rec, fr.tiles_x,
                           fr.tiles_y, fr.W, fr.H, fr.cover_w, fr.cover_h, out, consumed);
}

hipError_t launch_blend(const uint64_t* pairs, const uint2* ranges, const uint4* rec, const Frame& fr,
                        float* out, unsigned long long* consumed, int variant, hipStream_t s) {
    const int nt = fr.tiles_x * fr.tiles_y;
    if (nt <= 0) return hipSuccess;
    switch (variant) {
    case 1: blend_px<1>(pairs, ranges, rec, fr, out, consumed, s); return hipGetLastError();
    case 2: blend_px<2>(pairs, ranges, rec, fr, out, consumed, s); return hipGetLastError();
    case 4: blend_px<4>(pairs, ranges, rec, fr, out, consumed, s); return hipGetLastError();
    case 5:
        if (consumed)
            hipLaunchKernelGGL(k_blend_v5<true>, dim3(nt), dim3(256), 0, s, pairs, ranges, rec, fr.tiles_x,
                               fr.tiles_y, fr.W, fr.H, fr.cover_w, fr.cover_h, out, consumed);
        else
            hipLaunchKernelGGL(k_blend_v5<false>, dim3(nt), dim3(256), 0, s, pairs, ranges, rec, fr.tiles_x,
                               fr.tiles_y, fr.W, fr.H, fr.cover_w, fr.cover_h, out, consumed);
        return hipGetLastError();
    default: break;
    }
    if (consumed)
        hipLaunchKernelGGL(k_blend<true>, dim3(nt), dim3(256), 0, s, pairs, ranges, rec, fr.tiles_x, fr.tiles_y,
                           fr.W, fr.H, fr.cover_w, fr.cover_h, out, consumed);
    else
        hipLaunchKernelGGL(k_blend<false>, dim3(nt), dim3(256), 0, s, pairs, ranges, rec, fr.tiles_x,
                           fr.tiles_y, fr.W, fr.H, fr.cover_w, fr.cover_h, out, consumed);
    return hipGetLastError();
}

hipError_t launch_items_from_keys(const int* keys, uint32_t n, uint64_t* items, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_items_from_keys, dim3((n + 255) / 256), dim3(256), 0, s, keys, n, items);
    return hipGetLastError();
}

hipError_t launch_keys_from_items(const uint64_t* items, uint32_t n, int* keys, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_keys_from_items, dim3((n + 255) / 256), dim3(256), 0, s, items, n, keys);
    return hipGetLastError();
}

hipError_t launch_items_from_lwg(const gsr_lwg* rec, const uint64_t* src_perm, uint32_t n, int shift,
                                 uint32_t mask, uint64_t* items, hipStream_t s) {
    if (n)
        hipLaunchKernelGGL(k_items_from_lwg, dim3((n + 255) / 256), dim3(256), 0, s, rec, src_perm, n, shift, mask,
                           items);
    return hipGetLastError();
}

hipError_t launch_gather_lwg(const gsr_lwg* in, const uint64_t* stage1, const uint64_t* stage2, uint32_t n,
                             gsr_lwg* out, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_gather_lwg, dim3((n + 255) / 256), dim3(256), 0, s, in, stage1, stage2, n, out);
    return hipGetLastError();
}

hipError_t launch_math_probe(const float* in, int n, float* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_math_probe, dim3(grid_for(n, 256)), dim3(256), 0, s, in, n, out);
    return hipGetLastError();
}

}  // namespace gsr
