// gsr_kernels.hip — gfx950 (CDNA4) kernels of the 3DGS rasterizer.
//
// Pipeline per frame (all stream-ordered, no host round trip):
//   k_preprocess      one thread per Gaussian, SoA coalesced loads: cull + SH
//                     colour + view/clip + 2D covariance + extent + AABB, writes a
//                     64-B splat record, the (depth_key << 32 | index) item and
//                     the tile rectangle (4 B packed on the binning path) [render.cu:472-786]
//   radix passes      stable LSD sort of the N items by depth key (8-bit digits,
//                     trailing identity passes skipped on the device); every pass
//                     carries the packed rectangles, so they end in depth order
//   k_bin_rows_*      tile binning, row pass: one item per covered tile row,
//                     binned stably by row [render.cu:811-857, 788-809, 1099-1118]
//   k_bin_cols_*      tile binning, column pass: one Gaussian index per covered
//                     tile column, binned stably inside the row; tile ranges
//   (k_emit_*, k_kv_*: pair emission + key-value tile sort, for grids over 256
//                     tiles per axis)
//   k_blend_w         one wave64 per 8x8 block, one pixel per lane; 64-record
//                     batches culled against the block, survivors compacted into
//                     LDS pair slots, two splats per iteration with packed math;
//                     exact per-pixel early termination [render.cu:266-367]
//
// Every float expression restates render.cu / math.cu in the same operation
// order; the file is compiled with -ffp-contract=off so no FMA is formed
// implicitly, and the transcendental functions come from gsr_detmath.h, so the
// results are bit-identical to the CPU oracle (oracle/gsr_oracle.c).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include <type_traits>

#include "gsr_detmath.h"
#include "gsr.h"
#include "gsr_internal.h"

namespace gsr {

namespace {

__constant__ float kShC0 = 0.28209479177387814f;      // render.cu:369-377
__constant__ float kShC1 = 0.4886025119029199f;

// Geometry kernels raise their waves' instruction-issue priority (s_setprio) above
// the blend's: with frames in flight, a geometry wave that shares a SIMD with blend
// waves would otherwise queue behind them for the VALU.  Issue priority only: no
// preemption, no effect on a kernel running alone (+0.8 % frames/s in flight,
// interleaved A/B of two builds: profiles/r02_ab_setprio.txt).
#ifndef GSR_GEOM_PRIORITY
#define GSR_GEOM_PRIORITY 3
#endif
#define GSR_GEOM_PRIO()                                                            \
    do {                                                                           \
        if (GSR_GEOM_PRIORITY > 0) __builtin_amdgcn_s_setprio(GSR_GEOM_PRIORITY); \
    } while (0)

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// ------------------------------------------------------------------ helpers

// Cross-lane moves on the DPP path (VALU) instead of ds_bpermute (the LDS crossbar,
// one LDS round trip per step): a wave64 scan is six dependent VALU ops.  CDNA4 is a
// GFX9 core, so row_bcast:15 / :31 and wave_shr:1 exist.  Lanes a control does not
// reach (row start for row_shr, rows outside row_mask) read 0, the identity of every
// scan below (add, unsigned max, or).
template <int CTRL, int ROWM, bool BC>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWM, 0xf, BC);
}
template <int CTRL, int ROWM, bool BC, typename T>
__device__ __forceinline__ T dpp_mov(T x) {
    if constexpr (sizeof(T) == 4) {
        return (T)dpp_u32<CTRL, ROWM, BC>((uint32_t)x);
    } else {
        const uint64_t u = (uint64_t)x;
        const uint32_t lo = dpp_u32<CTRL, ROWM, BC>((uint32_t)u), hi = dpp_u32<CTRL, ROWM, BC>((uint32_t)(u >> 32));
        return (T)(((uint64_t)hi << 32) | lo);
    }
}
struct OpAdd {
    template <typename T>
    __device__ T operator()(T a, T b) const { return a + b; }
};
struct OpMax {
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return max(a, b); }
};
struct OpOr {
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a | b; }
};
// Inclusive wave64 scan: Hillis-Steele inside each row of 16 lanes (row_shr 1, 2, 4, 8),
// then row 0's total into row 1 and row 2's into row 3 (row_bcast:15), then rows 0-1's
// into rows 2-3 (row_bcast:31).
template <typename T, typename Op>
__device__ __forceinline__ T wave_incl_scan(T x, Op op) {
    x = op(x, dpp_mov<0x111, 0xf, true>(x));
    x = op(x, dpp_mov<0x112, 0xf, true>(x));
    x = op(x, dpp_mov<0x114, 0xf, true>(x));
    x = op(x, dpp_mov<0x118, 0xf, true>(x));
    x = op(x, dpp_mov<0x142, 0xa, false>(x));
    x = op(x, dpp_mov<0x143, 0xc, false>(x));
    return x;
}
// The value of the lane below (0 at lane 0): wave_shr:1.
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x) { return dpp_u32<0x138, 0xf, true>(x); }

// Exclusive scan across a workgroup of NW waves (4 = 256 threads unless a kernel says
// otherwise); `scratch` holds NW entries.  Contains two barriers; every thread of the
// block must call it.
template <typename T, int NW = 4>
__device__ __forceinline__ T block_exclusive_scan(T v, T* scratch, T& total) {
    const uint32_t lane = lane_id();
    const uint32_t w = threadIdx.x >> 6;
    const T x = wave_incl_scan(v, OpAdd{});
    if (lane == 63) scratch[w] = x;
    __syncthreads();
    T pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NW; k++) {
        const T s = scratch[k];
        if ((uint32_t)k < w) pre += s;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return pre + x - v;
}

// block_exclusive_scan without its trailing barrier: the caller barriers before `scratch`
// is written again (and before anything it publishes from the result is read).
template <typename T, int NW = 4>
__device__ __forceinline__ T block_exclusive_scan_lead(T v, T* scratch, T& total) {
    const uint32_t lane = lane_id();
    const uint32_t w = threadIdx.x >> 6;
    const T x = wave_incl_scan(v, OpAdd{});
    if (lane == 63) scratch[w] = x;
    __syncthreads();
    T pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NW; k++) {
        const T s = scratch[k];
        if ((uint32_t)k < w) pre += s;
        tot += s;
    }
    total = tot;
    return pre + x - v;
}

// Wave64-wide max / or (every lane gets the result: lane 63 of the inclusive scan).
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(v, OpMax{}), 63);
}
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(v, OpOr{}), 63);
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

// Chunk handled by workgroup b of G when the chunks are dealt so that each XCD
// takes one contiguous run of them (a bijection on [0, G); hardware dispatch sends
// workgroup b to XCD b mod 8).  The partial cache lines at the seams between
// consecutive chunks' output runs are then written through one L2.  Used by the
// depth sort's downsweep at 16 items per thread (scenes of 4M+ Gaussians: config
// 3 depth sort 173 -> 163 us); not by the binning scatters, whose chunks carry
// uneven work (near splats cover more rows and columns) that contiguous runs would
// pile onto one XCD (config 3 rows 100 -> 143 us, columns 143 -> 199 us;
// profiles/r02_ab_xcd_chunks.txt).
#ifndef GSR_XCD_DEPTH
#define GSR_XCD_DEPTH 1   // 0: round-robin chunks in the depth downsweep too (A/B builds)
#endif
__device__ __forceinline__ int xcd_chunk(int b, int G) {
    const int xcd = b & 7, q = G >> 3, r = G & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
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

// Compact tile rectangle of one Gaussian for the emission: tx0 | tx1 << 16 |
// ty0 << 32 | ty1 << 48; tile count (tx1 - tx0 + 1) * (ty1 - ty0 + 1), which
// is 0 for the dead value below (tx0 = ty0 = 1, tx1 = ty1 = 0).
constexpr uint64_t kDeadRect = 0x0000000100000001ull;
__device__ __forceinline__ uint32_t rect_count(uint64_t r) {
    const int tx0 = (int)(r & 0xffffu), tx1 = (int)((r >> 16) & 0xffffu);
    const int ty0 = (int)((r >> 32) & 0xffffu), ty1 = (int)(r >> 48);
    return (uint32_t)((tx1 - tx0 + 1) * (ty1 - ty0 + 1));
}

// 4-B form of a tile rectangle for grids of at most 256 tiles per axis (the
// binning path): tx0 | tx1 << 8 | ty0 << 16 | ty1 << 24.  Lossless there (every
// coordinate is < 256; the dead value packs to 0x00010001 and unpacks to kDeadRect).
__device__ __forceinline__ uint32_t pack_rect(uint64_t r) {
    return (uint32_t)(r & 0xffu) | (uint32_t)((r >> 8) & 0xff00u) | (uint32_t)((r >> 16) & 0xff0000u) |
           (uint32_t)((r >> 24) & 0xff000000u);
}
__device__ __forceinline__ uint64_t unpack_rect(uint32_t p) {
    return (uint64_t)(p & 0xffu) | ((uint64_t)((p >> 8) & 0xffu) << 16) | ((uint64_t)((p >> 16) & 0xffu) << 32) |
           ((uint64_t)(p >> 24) << 48);
}

// The preprocess's tile rect of Gaussian i: 8 B, or packed to 4 B (pack_rect) for the
// binning path (`packed`: the buffer then holds u32 rects in index order).
__device__ __forceinline__ void put_rect(uint64_t* rect, int64_t i, uint64_t r, int packed) {
    if (packed)
        reinterpret_cast<uint32_t*>(rect)[i] = pack_rect(r);
    else
        rect[i] = r;
}

// ------------------------------------------------------------------ blend cull words
//
// The blend culls every record of its tile list against each 8x8 block (the
// ellipse-vs-block test and the fast-path proof below).  Everything in those
// tests that depends on the record alone is computed once here, in
// k_preprocess, and stored as the record's fourth 16-B word (the blend's record
// gather fetches the whole 64-B line anyway: profiles/r01_fetch_calibration.txt):
//   { xs, ih, iv, S }
// xs   gsr_alpha_take_min_x(op): the alpha test passes on a pixel iff its exp
//      argument -md2/2 >= xs (exact, gsr_detmath.h).  The block test's md2 cutoff is
//      -2 xs (+1e-6, block_cut) when the conic is robustly positive definite; the
//      blend's fast-exp mode takes its alpha decisions from xs
//      (-inf: every pixel passes, the block test never culls)
// ih   -h / e, iv = -h / a (edge minimisers of the quadratic form), h = (b + c) / 2
// S    |a| + |b| + |c| + |e| if the record passes the per-record part of the
//      fast-path proof (robustly PD, finite S and colour, coefficients 0 or
//      >= 2^-60), else +inf (then the per-block part S M^2 <= 4e7 fails, and the
//      block test's rounding margin is infinite: conservative, never culls)

// md2 cutoff of one splat: alpha = fminf(op * exp(-md2/2), 0.99) < 1e-3 holds
// for every md2 > 2 ln(1000 op) (exp and the product are within a few ulp), so
// lanes beyond the returned bound can never composite.  The bound is padded by
// 1e-5 relative + 1e-3 absolute — orders of magnitude above the rounding of
// gsr_blend_expf, the product and the hardware log2 used here — and is NaN (never
// skip) for NaN opacity, +inf for infinite opacity, -inf for op <= 0.  It only
// decides whether a wave may SKIP work; it never changes a composited value.
__device__ __forceinline__ float md2_cutoff(float op) {
    const float l = __log2f(op * 1000.0f);                   // v_log_f32
    return (l * 1.38629436111989061f) * 1.00001f + 1e-3f;     // 2 ln2 log2(1000 op)
}

// Fast-path proof for one splat on one block (exactness, not a heuristic):
// finite conic that is robustly positive definite with |a|+|b|+|c|+|e| times
// the squared largest block offset <= 4e7 keeps every in-box md2 finite and
// >= -10 (float error of the 9-op form < 10), so -md2/2 lies in gsr_blend_expf_x2's
// proven range; finite colours make "alpha = 0 when not taken" leave the
// accumulators bit-identical (c + (col*0)*T == c, T*(1-0) == T).
// Every coefficient is also 0 or of magnitude >= 2^-60: the pixel offsets are
// integers, so every intermediate of the md2 form is a multiple of 2^-83 —
// zero or a normal number — and scaling the coefficients by -0.5 scales every
// intermediate exactly: the form on (-a/2, -b/2, -c/2, -e/2) IS -0.5f * md2.
// The per-record part is the cull word's S; the per-block part, in the blend,
// is S * M * M <= 4e7.
__device__ __forceinline__ bool coef_ok(float v) { return v == 0.0f || fabsf(v) >= 0x1p-60f; }

__device__ __forceinline__ uint4 cull_word(float a, float b, float c, float e, float op, float r, float g,
                                           float bl) {
    const float inf = __builtin_huge_valf();
    const float h = 0.5f * (b + c);
    const bool pd = a > 0.0f && e > 0.0f && (a * e - h * h) > 1e-4f * (a * e);
    const float S = fabsf(a) + fabsf(b) + fabsf(c) + fabsf(e);
    const bool fast = pd && isfinite(S) && isfinite(r) && isfinite(g) && isfinite(bl) && coef_ok(a) &&
                      coef_ok(b) && coef_ok(c) && coef_ok(e);
    // edge minimisers; v_rcp_f32 (~1 ulp) moves them by ~1e-7 relative, which
    // changes an edge minimum only at second order (e * delta^2), far inside the
    // block test's rounding margin
    const float ih = pd ? -h * __builtin_amdgcn_rcpf(e) : 0.0f;
    const float iv = pd ? -h * __builtin_amdgcn_rcpf(a) : 0.0f;
    // a conic that is not robustly PD never culls: xs = -inf makes block_cut +inf.  Its
    // alpha decisions come from the exact one-splat path (no fast proof), never xs.
    const float xs = pd ? gsr_alpha_take_min_x(op) : -inf;
    return make_uint4(__float_as_uint(xs), __float_as_uint(ih), __float_as_uint(iv), __float_as_uint(fast ? S : inf));
}

// md2 cutoff of the block test from the record's xs: a lane with float md2 > -2 xs has
// -md2/2 < xs (exact scaling; the 1e-6 pad covers a subnormal -md2/2 rounding up to xs)
// and fails the alpha test.  xs = -inf: +inf (never culls); +inf: -inf (always culls).
__device__ __forceinline__ float block_cut(float xs) { return __builtin_fmaf(-2.0f, xs, 1e-6f); }

// Can any pixel of an integer rectangle reach md2 <= cut?  dx0..dy1 bound the
// (float)pixel - (float)centre offsets of the rectangle's pixels (monotone, so
// every pixel's dx lies in [dx0, dx1]).  Returns false only when the exact
// minimum of the quadratic form a dx^2 + (b+c) dx dy + e dy^2 over that
// rectangle exceeds cut by more than a bound on the float rounding of md2
// (<= ~6 ulp of |a|dx^2 + (|b|+|c|)|dx dy| + |e|dy^2, padded 10x) — so a culled
// splat could never have composited onto this block.  cut, ih and iv come from
// the record's cull word (cull_word), SMM = S M^2 with the word's S and M the largest
// |offset| of the rectangle: a conic that is not robustly positive definite has
// cut = +inf, a record without the per-record fast proof S = +inf (infinite margin);
// NaN anywhere: never culled.
__device__ __forceinline__ bool block_may_reach(float a, float b, float c, float e, float ih, float iv,
                                                float dx0, float dx1, float dy0, float dy1, float SMM, float cut) {
    // centre inside the rectangle: reachable.  Evaluated branch-free with the rest (the
    // blend's cull runs it on every lane; a branch only adds exec-mask work)
    const bool inside = (dx0 <= 0.0f) & (dx1 >= 0.0f) & (dy0 <= 0.0f) & (dy1 >= 0.0f);
    // q = a x^2 + (b + c) x y + e y^2 in Horner form with explicit fused multiply-adds
    // (5 VALU instead of 8): its rounding error stays a few ulp of the terms' magnitudes,
    // far inside the margin below (4e-6 relative)
    const float bc = b + c;
    auto q = [&](float x, float y) { return __builtin_fmaf(x, __builtin_fmaf(a, x, bc * y), (e * y) * y); };
    // The form is convex with its minimum at the splat centre (offset 0,0), which
    // lies outside the rectangle here.  A far edge never holds the rectangle's
    // minimum (from any of its points the segment toward the centre enters the
    // interior, where the form is smaller), so only the near x-edge (when 0 is not
    // in [dx0, dx1]) and the near y-edge (when 0 is not in [dy0, dy1]) are evaluated.
    const float xe = dx0 > 0.0f ? dx0 : dx1, ye = dy0 > 0.0f ? dy0 : dy1;
    // clamps as v_med3_f32: equal to fminf(fmaxf(v, lo), hi) here (lo <= hi; lo and hi
    // both NaN or neither; quiet NaN v gives lo either way), without the two
    // canonicalising v_max each fminf / fmaxf operand costs in IEEE mode
    const float qx = q(xe, __builtin_amdgcn_fmed3f(ih * xe, dy0, dy1));
    const float qy = q(__builtin_amdgcn_fmed3f(iv * ye, dx0, dx1), ye);
    const bool x_out = dx0 > 0.0f || dx1 < 0.0f, y_out = dy0 > 0.0f || dy1 < 0.0f;
    const float qm = fminf(x_out ? qx : 3.0e38f, y_out ? qy : 3.0e38f);
    const float err = __builtin_fmaf(4e-6f, SMM, 1e-3f);   // SMM = S M M (S, M: see above)
    return inside | !(qm - err > cut);
}

// Tile row spans (binning path, GSR_TUNE_TILE_SPANS).  A splat's tile rect is the
// box of its AABB, and an elongated or tilted ellipse reaches alpha >= 1e-3 on only
// part of it: config 2 lists 5.39M (tile, splat) pairs of which 4.12M can composite
// at all.  For each of the first four tile rows of the rect, nibble r of the 16-bit
// code counts the columns at the row's left end (bits 0-1) and right end (bits 2-3)
// that hold no in-box pixel of the ellipse q <= C; the row pass lists only the
// columns in between (none when left + right >= the row's width).  Rows past the
// fourth (4.1M of the 4.12M reachable pairs sit in the first four) keep every
// column; a count stops at 3, keeping the middle columns (conservative; counts up
// to 15 drop no more pairs on config 2, and 2 B per Gaussian keep the row pass's
// gather of the codes by index half the footprint of 4 B).
//
// Why a dropped pair changes no pixel.  q = a dx^2 + (b + c) dx dy + e dy^2 is the
// exact md2 of the record's float conic; the blend's float md2 is within
// 4e-6 S M^2 of it (block_may_reach's bound: S = |a|+|b|+|c|+|e|, M = largest
// |offset| in the AABB), so with C = cut + 4e-6 S M^2 + 1e-3 every pixel outside
// q <= C has float md2 > cut, alpha < 1e-3, and is never taken.  The x-extent of
// q <= C over a strip of offsets [u0, u1] is [L, R]: R is the ellipse's rightmost
// offset xr = sqrt(C e / det) when the strip holds its ordinate yr = -h xr / e,
// else (-h u + sqrt(a C - det u^2)) / a at the strip end nearer yr (R(dy) is
// concave); L mirrors it.  Float error: det = a e - h^2 is within 3e-7 k of itself
// relative (k = a e / det <= 1e4 for a finite cut), which moves xr, ym and the
// square root by at most sqrt(6e-7 (k + 1)) xr; the pads below cover that and the
// approximate rcp / sqrt (~1 ulp) with room.  A numpy restatement of this function
// (tools/sim/spans_check.py) keeps 78.7 % of config 2's pairs (the exact hull: 76.5 %)
// and every pair it drops peaks at alpha <= 0.9976e-3 on its tile.
__device__ __forceinline__ uint16_t tile_row_spans(float cx, float cy, float a, float b, float c, float e,
                                                   float cut, uint4 cw, int xmin_px, int xmax_px, int ymin_px,
                                                   int ymax_px, int tx0, int tx1, int ty0, int ty1) {
    const float S = __uint_as_float(cw.w);
    // not robustly positive definite (cut = inf) or without the fast proof (S = inf): keep all
    if (!(cut < 3.0e38f) || !(S < 3.0e38f)) return 0u;
    const float h = 0.5f * (b + c);
    const float det = a * e - h * h;   // > 1e-4 a e here (cull_word's pd test)
    const float M = fmaxf(fmaxf(fabsf((float)xmin_px - cx), fabsf((float)xmax_px - cx)),
                          fmaxf(fabsf((float)ymin_px - cy), fabsf((float)ymax_px - cy)));
    const float C = cut + (4e-6f * S * M * M + 1e-3f);
    const float rdet = __builtin_amdgcn_rcpf(det), ra = __builtin_amdgcn_rcpf(a);
    const float xr = __builtin_amdgcn_sqrtf(C * e * rdet);   // rightmost offset (leftmost: -xr)
    const float ym = __builtin_amdgcn_sqrtf(C * a * rdet);   // largest |dy| of the ellipse
    const float yr = -h * xr * __builtin_amdgcn_rcpf(e);     // its ordinate (leftmost: -yr)
    const float k = a * e * rdet;
    const float rel = __builtin_amdgcn_sqrtf(6e-7f * (k + 1.0f)) + 1e-4f;
    // offsets are exact (integer pixel minus integer-valued centre); cx + L rounds by
    // < 5e-4 px below 4096, hence the 1/64 px (a 2-px pad kept 6 % more pairs)
    const float padx = 0.015625f + rel * xr, ymp = ym * (1.0f + rel) + 0.015625f;
    const float aC = a * C;
    const int w = tx1 - tx0 + 1;
    const int rows = min(ty1 - ty0 + 1, 4);
    uint32_t code = 0;
    for (int r = 0; r < rows; r++) {
        const int ty = ty0 + r;
        const int y0 = max(ty * GSR_TILE_PX, ymin_px), y1 = min(ty * GSR_TILE_PX + (GSR_TILE_PX - 1), ymax_px);
        const float dy0 = (float)y0 - cy, dy1 = (float)y1 - cy;
        int c0 = tx1 + 1, c1 = tx0 - 1;   // empty
        if (!(dy0 > ymp || dy1 < -ymp)) {
            const float u0 = fminf(fmaxf(dy0, -ym), ym), u1 = fminf(fmaxf(dy1, -ym), ym);
            float R = xr, L = -xr;
            if (!(yr >= u0 && yr <= u1)) {
                const float u = yr < u0 ? u0 : u1;
                R = (-h * u + __builtin_amdgcn_sqrtf(fmaxf(aC - det * u * u, 0.0f))) * ra;
            }
            if (!(-yr >= u0 && -yr <= u1)) {
                const float u = -yr < u0 ? u0 : u1;
                L = (-h * u - __builtin_amdgcn_sqrtf(fmaxf(aC - det * u * u, 0.0f))) * ra;
            }
            const float xl = fmaxf(cx + L - padx, (float)xmin_px), xh = fminf(cx + R + padx, (float)xmax_px);
            if (xl <= xh) {
                c0 = max(tx0, (int)floorf(xl * (1.0f / GSR_TILE_PX)));
                c1 = min(tx1, (int)floorf(xh * (1.0f / GSR_TILE_PX)));
            }
        }
        int sl, sr;
        if (c0 > c1) {
            sl = sr = min(w, 3);   // no column reachable (w > 6: the middle ones stay)
        } else {
            sl = min(c0 - tx0, 3);
            sr = min(tx1 - c1, 3);
        }
        code |= (uint32_t)(sl | (sr << 2)) << (4 * r);
    }
    return (uint16_t)code;
}

// Temporal state of a 4D (Spacetime-Gaussian style) Gaussian at time t, in
// this exact operation order (the oracle restates it, oracle/gsr_oracle.c):
// dt = t - c; x_t = ((x + m0 dt) + m3 dt^2) + m6 dt^3 (dt^2 = dt dt, dt^3 =
// dt^2 dt; y, z with m1/m4/m7, m2/m5/m8); temporal factor exp(-(dt/s)^2).
// One Gaussian i < n; returns the depth key of its item (0xFFFFFFFF: culled or dead).
// Array k of the scene block for the workgroup's Gaussians: the base (arr + k stride + the
// workgroup's first index) is uniform, so it is formed by scalar instructions and the load
// takes it as an SGPR pair beside the lane's 32-bit byte offset (global_load ... saddr).
// Indexing arr[k * stride + i] with a 64-bit i made every load's address a per-lane
// 64-bit multiply-add (v_mad_u64_u32) — ~150 VALU per Gaussian for 38 arrays.
struct SoaWg {
    const float* base;   // arr + first index of the workgroup (uniform)
    int64_t stride;
    uint32_t off;        // lane byte offset: 4 * (i - first index)
    __device__ __forceinline__ float operator()(int64_t k) const {
        typedef const __attribute__((address_space(1))) char* gptr;
        gptr b = (gptr)(base + k * stride);
        asm("" : "+s"(b));   // keep the base whole (the compiler re-associates it into the lane part)
        return *(const __attribute__((address_space(1))) float*)(b + off);
    }
};

template <bool T4D, bool SH3>
__device__ __forceinline__ uint32_t preprocess_one(const SoaWg& A,
                                                   const Frame& fr, uint4* __restrict__ rec,
                                                   uint64_t* __restrict__ items, uint64_t* __restrict__ rect,
                                                   int packed, uint16_t* __restrict__ spans, float tnow,
                                                   const RecSplit& rs, int64_t i) {
    // depth split, key mode (RecSplit): 1 = records of the near Gaussians only, 2 = the
    // far ones' records only (no item, rect or span writes: those are sorted already)
    const bool far_pass = rs.mode == 2;
    if (far_pass && rs.gate && *rs.gate == 0u) return 0xffffffffu;
    const uint32_t kcut = rs.mode == 1 ? *rs.kcut : far_pass ? *rs.kcut_frame : 0xffffffffu;
    // the frame's threshold, for the far record pass (the near sort copies it too)
    if (rs.mode == 1 && i == 0) *rs.kcut_frame = kcut;
    float gx = A(GSR_A_X);
    float gy = A(GSR_A_Y);
    float gz = A(GSR_A_Z);
    float tfac = 1.0f;
    if (T4D) {
        const float dt = tnow - A(GSR_A_TCENTER);
        const float dt2 = dt * dt, dt3 = dt2 * dt;
        auto m = [&](int j) { return A(GSR_A_MOTION0 + j); };
        gx = ((gx + m(0) * dt) + m(3) * dt2) + m(6) * dt3;
        gy = ((gy + m(1) * dt) + m(4) * dt2) + m(7) * dt3;
        gz = ((gz + m(2) * dt) + m(5) * dt2) + m(8) * dt3;
        const float u = dt / A(GSR_A_TSCALE);
        tfac = gsr_expf(-(u * u));
    }
    // Every other load of this Gaussian is issued here, before the cull decides
    // whether it is needed: one memory round trip instead of three (position, then
    // rotation / scale, then SH).  Wasted bytes for culled Gaussians only (config 2:
    // 5 %).  The SH stays behind the cull in 4D (the temporal cull drops ~64 %) and
    // SH-3 (48 coefficients) modes.
    constexpr bool kEarlySH = !T4D && !SH3;
    float q_in[4], s_in[3], op_in, sh_in[kEarlySH ? 27 : 1];
#pragma unroll
    for (int k = 0; k < 4; k++) q_in[k] = A(GSR_A_ROT0 + k);
#pragma unroll
    for (int k = 0; k < 3; k++) s_in[k] = A(GSR_A_SCALE0 + k);
    op_in = A(GSR_A_OPACITY);
    if (kEarlySH) {
#pragma unroll
        for (int k = 0; k < 27; k++) sh_in[k] = A(GSR_A_SH0 + k);
    }
    uint4* R = rec + 4 * i;
    if (!far_pass) items[i] = ((uint64_t)0xffffffffu << 32) | (uint64_t)(uint32_t)i;

    // ---- view + clip transform and cull (render.cu:535-556) ----
    const float old_xyz[4] = {gx, gy, gz, 1.0f};
    float tmp_xyz[4], new_xyz[4];
    mv4(fr.V, old_xyz, tmp_xyz);
    if (!isfinite(tmp_xyz[0]) || !isfinite(tmp_xyz[1]) || !isfinite(tmp_xyz[2])) {
        if (!far_pass) put_rect(rect, i, kDeadRect, packed);
        return 0xffffffffu;
    }
    mv4(fr.P, tmp_xyz, new_xyz);
    new_xyz[0] = new_xyz[0] / new_xyz[3];
    new_xyz[1] = new_xyz[1] / new_xyz[3];
    new_xyz[2] = new_xyz[2] / new_xyz[3];
    if (!isfinite(new_xyz[0]) || !isfinite(new_xyz[1]) || !isfinite(new_xyz[2]) ||
        tmp_xyz[2] >= -fr.znear || new_xyz[2] < -1.0f || new_xyz[2] > 1.0f) {
        if (!far_pass) put_rect(rect, i, kDeadRect, packed);
        return 0xffffffffu;
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
    float qw = q_in[0];
    float qx = q_in[1];
    float qy = q_in[2];
    float qz = q_in[3];
    const float qn = sqrtf(qx * qx + qy * qy + qz * qz + qw * qw);
    qx /= qn; qy /= qn; qz /= qn; qw /= qn;
    float Rm[9], RT[9], S[9], tmp[9], cov[9];
    Rm[0] = 1 - 2 * qy * qy - 2 * qz * qz; Rm[1] = 2 * qx * qy - 2 * qw * qz;     Rm[2] = 2 * qx * qz + 2 * qw * qy;
    Rm[3] = 2 * qx * qy + 2 * qw * qz;     Rm[4] = 1 - 2 * qx * qx - 2 * qz * qz; Rm[5] = 2 * qy * qz - 2 * qw * qx;
    Rm[6] = 2 * qx * qz - 2 * qw * qy;     Rm[7] = 2 * qy * qz + 2 * qw * qx;     Rm[8] = 1 - 2 * qx * qx - 2 * qy * qy;
    RT[0] = Rm[0]; RT[1] = Rm[3]; RT[2] = Rm[6];
    RT[3] = Rm[1]; RT[4] = Rm[4]; RT[5] = Rm[7];
    RT[6] = Rm[2]; RT[7] = Rm[5]; RT[8] = Rm[8];
    S[0] = s_in[0]; S[1] = 0.0f; S[2] = 0.0f;
    S[3] = 0.0f; S[4] = s_in[1]; S[5] = 0.0f;
    S[6] = 0.0f; S[7] = 0.0f; S[8] = s_in[2];
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
        if (!far_pass) put_rect(rect, i, kDeadRect, packed);
        return 0xffffffffu;
    }
    const float invDet = 1.0f / det;
    const float ic0 = S2[3] * invDet, ic1 = -S2[1] * invDet;
    const float ic2 = -S2[2] * invDet, ic3 = S2[0] * invDet;
    if (T4D) {
        // temporal cull (exact): opacity below 0.9e-3 with a robustly positive
        // definite conic keeps md2 >= -0.05 at every pixel of the AABB, so alpha
        // = min(op exp(-md2/2), 0.99) < 1e-3 everywhere and the splat never composites
        const float opt = op_in * tfac;
        const float hh = 0.5f * (ic1 + ic2);
        if (opt < 0.9e-3f && ic0 > 0.0f && ic3 > 0.0f && (ic0 * ic3 - hh * hh) > 1e-4f * (ic0 * ic3)) {
            if (!far_pass) put_rect(rect, i, kDeadRect, packed);
            return 0xffffffffu;
        }
    }

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
        if (!far_pass) put_rect(rect, i, kDeadRect, packed);
        return 0xffffffffu;
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
    const uint64_t trect =
        (uint64_t)((uint32_t)tx0 | ((uint32_t)tx1 << 16)) | ((uint64_t)((uint32_t)ty0 | ((uint32_t)ty1 << 16)) << 32);
    if (rs.mode == 1 && key >= kcut && !spans) {
        // far (key mode): no record unless phase B needs it (mode 2 writes it then)
        put_rect(rect, i, trect, packed);
        items[i] = ((uint64_t)key << 32) | (uint64_t)(uint32_t)i;
        return key;
    }
    if (far_pass && key < kcut) return key;

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
    if (!SH3) {
#pragma unroll
        for (int ch = 0; ch < 3; ch++) {
            auto SH = [&](int k) { return kEarlySH ? sh_in[ch + k] : A(GSR_A_SH0 + ch + k); };   // sh[ch], sh[3+ch], ...
            float cc = SH(0) * kShC0;
            cc += kShC1 * z * SH(6);
            cc -= kShC1 * y * SH(3);
            cc -= kShC1 * x * SH(9);
            cc += C2_0 * xy * SH(12);
            cc += C2_1 * yz * SH(15);
            cc += C2_2 * (2.0f * zz - xx - yy) * SH(18);
            cc += C2_3 * xz * SH(21);
            cc += C2_4 * (xx - yy) * SH(24);
            cc += 0.5f;
            col[ch] = fminf(fmaxf(cc, 0.0f), 1.0f);
        }
    } else {
        // "Inria-correct" mode: degree-3 SH as the 3DGS training code evaluates it
        // (left-to-right, bands 0..3), + 0.5, clamped at 0 only
        const float C3_0 = -0.5900435899266435f, C3_1 = 2.890611442640554f, C3_2 = -0.4570457994644658f,
                    C3_3 = 0.3731763325901154f, C3_4 = -0.4570457994644658f, C3_5 = 1.445305721320277f,
                    C3_6 = -0.5900435899266435f;
#pragma unroll
        for (int ch = 0; ch < 3; ch++) {
            auto S = [&](int k) { return A(GSR_A_SH0 + ch + 3 * k); };   // coefficient k of channel ch
            float r = kShC0 * S(0);
            r = r - kShC1 * y * S(1) + kShC1 * z * S(2) - kShC1 * x * S(3);
            r = r + C2_0 * xy * S(4) + C2_1 * yz * S(5) + C2_2 * (2.0f * zz - xx - yy) * S(6) +
                C2_3 * xz * S(7) + C2_4 * (xx - yy) * S(8);
            r = r + C3_0 * y * (3.0f * xx - yy) * S(9) + C3_1 * xy * z * S(10) +
                C3_2 * y * (4.0f * zz - xx - yy) * S(11) + C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * S(12) +
                C3_4 * x * (4.0f * zz - xx - yy) * S(13) + C3_5 * z * (xx - yy) * S(14) +
                C3_6 * x * (xx - 3.0f * yy) * S(15);
            r += 0.5f;
            col[ch] = fmaxf(r, 0.0f);
        }
    }
    const float opacity = T4D ? op_in * tfac : op_in;

    R[0] = make_uint4(__float_as_uint(ic0), __float_as_uint(ic1), __float_as_uint(ic2), __float_as_uint(ic3));
    R[1] = make_uint4(__float_as_uint(opacity), __float_as_uint(col[0]), __float_as_uint(col[1]),
                      __float_as_uint(col[2]));
    // centre pixel stored as the float the blend computes with ((float)px, render.cu:329)
    R[2] = make_uint4(__float_as_uint((float)px_x), __float_as_uint((float)px_y), (uint32_t)xmin_px | ((uint32_t)xmax_px << 16),
                      (uint32_t)ymin_px | ((uint32_t)ymax_px << 16));
    const uint4 cw = cull_word(ic0, ic1, ic2, ic3, opacity, col[0], col[1], col[2]);
    R[3] = cw;
    if (far_pass) return key;
    if (spans)
        spans[i] = tile_row_spans((float)px_x, (float)px_y, ic0, ic1, ic2, ic3,
                                  cw.x == __float_as_uint(-__builtin_huge_valf()) ? __builtin_huge_valf()
                                                                                 : md2_cutoff(opacity),
                                  cw, xmin_px, xmax_px, ymin_px, ymax_px, tx0, tx1, ty0, ty1);
    put_rect(rect, i, trect, packed);
    items[i] = ((uint64_t)key << 32) | (uint64_t)(uint32_t)i;
    return key;
}

template <bool T4D, bool SH3>
__global__ __launch_bounds__(256) void k_preprocess(const float* __restrict__ arr, int64_t stride,
                                                    int64_t n, Frame fr, uint4* __restrict__ rec,
                                                    uint64_t* __restrict__ items, uint64_t* __restrict__ rect,
                                                    int packed, uint16_t* __restrict__ spans,
                                                    float tnow, RecSplit rs) {
    GSR_GEOM_PRIO();
    const int64_t i0 = (int64_t)blockIdx.x * 256;
    const int64_t i = i0 + threadIdx.x;
    if (i >= n) return;
    const SoaWg A{arr + i0, stride, 4u * threadIdx.x};
    (void)preprocess_one<T4D, SH3>(A, fr, rec, items, rect, packed, spans, tnow, rs, i);
}

// Lanes of the wave whose `bits`-bit digit equals this lane's, among the lanes in
// `valid` (the wave64 stand-in for __match_any): one ballot per digit bit.  Per bit
// 4 VALU: v_bfe_i32 (the bit as a 0 / -1 mask m), the ballot's v_cmp, and one
// v_bitop3_b32 per mask half computing peers & ~(ballot ^ m) — truth table 0x90 for
// (peers, ballot, m), index S0*4 + S1*2 + S2 (tools/microbench/bitop3_probe.hip) —
// where the select-and-mask form compiles to 8.
// (MAXB: compile-time bound on `bits`, so the loop unrolls; bits <= MAXB.)
template <int MAXB>
__device__ __forceinline__ uint64_t match_peers(uint32_t d, bool valid, int bits) {
    const uint64_t v = __ballot(valid);
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
    for (int bit = 0; bit < MAXB; bit++) {
        if (bit >= bits) break;
        const int m = __builtin_amdgcn_sbfe((int)d, bit, 1);
        const uint64_t bm = __ballot(m != 0);
        lo = __builtin_amdgcn_bitop3_b32(lo, (uint32_t)bm, (uint32_t)m, 0x90);
        hi = __builtin_amdgcn_bitop3_b32(hi, (uint32_t)(bm >> 32), (uint32_t)m, 0x90);
    }
    return ((uint64_t)hi << 32) | lo;
}

// Stable in-wave ranks from returning LDS atomics (template flag RA, runtime knob
// GSR_TUNE_RANK_ATOMIC): atomicAdd(&count[digit], 1) from one wave64 instruction
// returns the old values in LANE order when several lanes hit one address — measured
// on gfx950 with no exception in 1.5e10 lane-operations over uniform, skewed, run and
// interleaved digit patterns (tools/microbench/lds_atomic_order.hip) — so the returned
// value is the element's stable rank among the wave's earlier elements of its digit:
// one LDS op instead of ballot matching (4 VALU per digit bit, match_peers).  The ISA
// does not document that order, so the runtime only takes RA = true after
// k_rank_order_check (below) has found it on the device in this process; otherwise,
// or with the knob at 0, every kernel ranks with ballots (RA = false).

// ------------------------------------------------------------------ radix sort
//
// Stable LSD pass, reduce-then-scan (no inter-workgroup spin waits, so no
// forward-progress assumption): upsweep histograms per workgroup chunk,
// per-digit scan over workgroups, downsweep that ranks each 4096-item tile with
// wave64 ballot matching (the AMD stand-in for __match_any), scatters into LDS
// in digit order and writes runs out coalesced.

// Depth-sort pass plan.  dstats (zeroed per frame, filled by pass 0's upsweep
// over every key except 0xFFFFFFFF, which culled records carry): [0] max of ~key
// (= ~min key), [1] max key, [2] bit p set if some key has its low 8p bits all
// ones, [3] nonzero if any such key exists.  Pass p >= 1 is an identity (and is
// skipped) when every key shares the digits at and above p and no key has
// all-ones low 8p bits: the 0xFFFFFFFF keys then already trail in index order,
// exactly where the full sort puts them.  Skippable(p) implies skippable(p+1).
__device__ __forceinline__ bool depth_pass_skipped(const uint32_t* __restrict__ dstats, int pass) {
    if (!dstats || pass == 0) return false;
    if (dstats[3] == 0u) return true;
    const uint32_t kmin = ~dstats[0], kmax = dstats[1];
    return (kmin >> (8 * pass)) == (kmax >> (8 * pass)) && !((dstats[2] >> pass) & 1u);
}

__device__ __forceinline__ int depth_passes_run(const uint32_t* __restrict__ dstats) {
    int p = 1;
    while (p < 4 && !depth_pass_skipped(dstats, p)) ++p;
    return p;
}

// SortRange (depth split, key mode; all fields null / 0 otherwise):
//   base   the far part's positions [*base, n_host) are sorted on their own (n_dev unused)
//   gate   every kernel of the pass returns at once when *gate is 0 (phase B not needed)
//   filter pass 0 reads all n_host items of the preprocess order and keeps only those with
//          key < *kcut (1, the near part) or key >= *kcut (2, the far part), written from
//          position 0 (near) or *base (far); the near pass's downsweep stores the kept
//          count in *count_out, and its upsweep copies *kcut to *kcut_copy (the frame's
//          threshold, for phase B)
//   sat    (far pass 0) also drop an item whose tile rect (rect[position], packed) holds
//          no tile phase A left unsaturated: sat is the summed-area table of those tiles,
//          (tiles_y + 1) x sat_w words, sat_w = tiles_x + 1 (k_split_sat)
//   count  with base: the far part's length (the far pass 0's kept count), else n_host - base
struct SortRange {
    const uint32_t* base;
    const uint32_t* gate;
    const uint32_t* kcut;
    int filter;
    uint32_t* count_out;
    uint32_t* kcut_copy;
    const uint32_t* sat;
    int sat_w;
    const uint32_t* rect;
    const uint32_t* count;
};

// Some tile of the packed rect pr (tx0 | tx1 << 8 | ty0 << 16 | ty1 << 24) is counted
// in the summed-area table (dead rects hold none).
__device__ __forceinline__ bool rect_hits(const uint32_t* __restrict__ sat, int w, uint32_t pr) {
    const uint32_t x0 = pr & 0xffu, x1 = (pr >> 8) & 0xffu, y0 = (pr >> 16) & 0xffu, y1 = pr >> 24;
    if (x0 > x1 || y0 > y1) return false;
    const uint32_t* r0 = sat + (size_t)y0 * (uint32_t)w;
    const uint32_t* r1 = sat + (size_t)(y1 + 1u) * (uint32_t)w;
    return r1[x1 + 1u] - r0[x1 + 1u] - r1[x0] + r0[x0] != 0u;
}

__device__ __forceinline__ bool sort_keep(const SortRange& sr, uint32_t K, uint64_t v, uint32_t pr) {
    const uint32_t k = (uint32_t)(v >> 32);
    if (sr.filter == 1) return k < K;
    return sr.filter == 0 || (k >= K && (!sr.sat || rect_hits(sr.sat, sr.sat_w, pr)));
}

__device__ __forceinline__ uint64_t sort_len(const SortRange& sr, const uint32_t* n_dev, uint32_t n_host) {
    if (sr.base) {
        const uint32_t base = min(*sr.base, n_host);
        return sr.count ? (uint64_t)min(*sr.count, n_host - base) : (uint64_t)(n_host - base);
    }
    return n_dev ? (uint64_t)*n_dev : (uint64_t)n_host;
}

template <int ITEMS, bool FILT>   // FILT: a filtered pass 0 (SortRange::filter != 0)
__global__ __launch_bounds__(kSortThreads) void k_radix_upsweep(const uint64_t* __restrict__ in,
                                                                const uint32_t* __restrict__ n_dev,
                                                                uint32_t n_host, int shift, uint32_t mask,
                                                                int groups, uint32_t* __restrict__ hist,
                                                                uint32_t* __restrict__ dstats, int pass,
                                                                SortRange sr) {
    GSR_GEOM_PRIO();
    __shared__ uint32_t h[4][FILT ? 257 : 256];   // [256]: items a filtered pass 0 drops
    __shared__ uint32_t s_st[4];
    if (sr.gate && *sr.gate == 0u) return;
    if (depth_pass_skipped(dstats, pass)) return;
    const uint32_t t = threadIdx.x;
    const uint32_t w = t >> 6;
    const bool plan = dstats && pass == 0;
    uint32_t inv_min = 0, kmax = 0, lowones = 0, any = 0;
    if (plan && t < 4) s_st[t] = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) h[k][t] = 0;
    __syncthreads();
    const uint32_t K = FILT ? *sr.kcut : 0u;
    if (FILT && sr.filter == 1 && sr.kcut_copy && blockIdx.x == 0 && t == 0) *sr.kcut_copy = K;
    const uint32_t base = sr.base ? *sr.base : 0u;
    if (!FILT) in += base;
    const uint64_t n = FILT ? (uint64_t)n_host : sort_len(sr, n_dev, n_host);
    // (XCD-contiguous chunks, so that a histogram row's 64-B lines merge in one L2, measured
    // slower: config 3 upsweep 11.5 -> 16.5 us, profiles/r05_kt_xcd_hist.txt)
    const int chunk = (int)blockIdx.x;
    uint64_t b, e;
    chunk_range(n, groups, chunk, kSortThreads * ITEMS, b, e);
    const bool masked = FILT && sr.sat;   // the far pass 0's rect test reads rect[position]
    // the digit's counter, or the drop counter for an item a filtered pass 0 does not keep
    auto dig = [&](uint64_t v, uint64_t i) {
        return !FILT || sort_keep(sr, K, v, masked ? sr.rect[i] : 0u) ? ((uint32_t)(v >> shift) & mask) : 256u;
    };
    auto note = [&](uint64_t v, uint64_t i) {
        const uint32_t k = (uint32_t)(v >> 32);
        if (k != 0xffffffffu && (!FILT || sort_keep(sr, K, v, masked ? sr.rect[i] : 0u))) {
            inv_min = max(inv_min, ~k);
            kmax = max(kmax, k);
            any = 1u;
            lowones |= ((k & 0xffu) == 0xffu ? 2u : 0u) | ((k & 0xffffu) == 0xffffu ? 4u : 0u) |
                       ((k & 0xffffffu) == 0xffffffu ? 8u : 0u);
        }
    };
    uint64_t i = b + t;
    for (; i + 3 * kSortThreads < e; i += 4 * kSortThreads) {
        const uint64_t v0 = in[i], v1 = in[i + kSortThreads], v2 = in[i + 2 * kSortThreads],
                       v3 = in[i + 3 * kSortThreads];
        atomicAdd(&h[w][dig(v0, i)], 1u);
        atomicAdd(&h[w][dig(v1, i + kSortThreads)], 1u);
        atomicAdd(&h[w][dig(v2, i + 2 * kSortThreads)], 1u);
        atomicAdd(&h[w][dig(v3, i + 3 * kSortThreads)], 1u);
        if (plan) {
            note(v0, i);
            note(v1, i + kSortThreads);
            note(v2, i + 2 * kSortThreads);
            note(v3, i + 3 * kSortThreads);
        }
    }
    for (; i < e; i += kSortThreads) {
        const uint64_t v = in[i];
        atomicAdd(&h[w][dig(v, i)], 1u);
        if (plan) note(v, i);
    }
    if (plan) {   // wave reductions first: one LDS atomic per wave and word
        inv_min = wave_max_u32(inv_min);
        kmax = wave_max_u32(kmax);
        lowones = wave_or_u32(lowones);
        any = wave_or_u32(any);
        if ((t & 63u) == 0) {
            atomicMax(&s_st[0], inv_min);
            atomicMax(&s_st[1], kmax);
            atomicOr(&s_st[2], lowones);
            atomicOr(&s_st[3], any);
        }
    }
    __syncthreads();
    hist[t * (uint32_t)groups + chunk] = h[0][t] + h[1][t] + h[2][t] + h[3][t];
    // per-workgroup plan words after the 4 final ones; pass 0's scan kernel
    // reduces them (plain stores: ~500 device atomics on 4 addresses serialise)
    if (plan && t < 4) dstats[4 + 4 * blockIdx.x + t] = s_st[t];
}

// One workgroup per digit: exclusive scan of hist[d][0..groups) in place.
__global__ __launch_bounds__(256) void k_radix_scan(uint32_t* __restrict__ hist, int groups,
                                                     uint32_t* __restrict__ totals,
                                                     const uint32_t* __restrict__ dstats, int pass,
                                                     const uint32_t* __restrict__ gate) {
    GSR_GEOM_PRIO();
    __shared__ uint32_t scratch[4];
    if (gate && *gate == 0u) return;
    if (dstats && pass == 0 && blockIdx.x == 0) {
        // reduce the upsweep's per-workgroup plan words into dstats[0..3]
        __shared__ uint32_t r[4];
        if (threadIdx.x < 4) r[threadIdx.x] = 0;
        __syncthreads();
        uint32_t a = 0, b = 0, c = 0, d = 0;
        for (int g = threadIdx.x; g < groups; g += 256) {
            const uint32_t* q = dstats + 4 + 4 * g;
            a = max(a, q[0]);
            b = max(b, q[1]);
            c |= q[2];
            d |= q[3];
        }
        a = wave_max_u32(a);
        b = wave_max_u32(b);
        c = wave_or_u32(c);
        d = wave_or_u32(d);
        if ((threadIdx.x & 63u) == 0) {
            atomicMax(&r[0], a);
            atomicMax(&r[1], b);
            atomicOr(&r[2], c);
            atomicOr(&r[3], d);
        }
        __syncthreads();
        if (threadIdx.x < 4) const_cast<uint32_t*>(dstats)[threadIdx.x] = r[threadIdx.x];
    }
    if (depth_pass_skipped(dstats, pass)) return;
    uint32_t* row = hist + (size_t)blockIdx.x * groups;
    const int per = (groups + 255) / 256;
    const int b = threadIdx.x * per;
    // every load of the thread's segment in flight at once (a loop over `per` waited for
    // each in turn: 5 round trips at 5M items, 20 for the row scan below)
    constexpr int kPerMax = kMaxSortGroups / 256;
    uint32_t v[kPerMax], local = 0;
#pragma unroll
    for (int k = 0; k < kPerMax; k++) {
        v[k] = k < per && b + k < groups ? row[b + k] : 0u;
        local += v[k];
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan<uint32_t>(local, scratch, total);
#pragma unroll
    for (int k = 0; k < kPerMax; k++)
        if (k < per && b + k < groups) {
            row[b + k] = run;
            run += v[k];
        }
    if (threadIdx.x == 0) totals[blockIdx.x] = total;
}

// pay_out != nullptr (depth sort feeding the tile binning): every pass carries
// each item's tile rectangle as a 4-B payload (pack_rect: grids <= 256 tiles per
// axis) and writes it at the item's destination, so the pass that turns out to be
// the last one leaves the rects in depth order (pay_out[np & 1] for np passes run)
// for the row pass to read coalesced.  Pass 0 takes it from the live partition's
// payloads (pay_in), or from the preprocess's packed rects: rect[position] when its
// input is the preprocess order (rect_direct: item j has index j), else rect[index]
// (a repeated sort).
// Payloads leave through the items' LDS slots, in the same digit runs.
// (The rects used to be gathered in the last pass only: a random 8-B read per item
// that cost the 5M-Gaussian frame 76 us of its 110-us pass, profiles/r02_geom_pmc.txt.)
template <int ITEMS, bool RA, bool FILT>   // FILT: a filtered pass 0 (SortRange::filter != 0)
__global__ __launch_bounds__(kSortThreads) void k_radix_downsweep(
    const uint64_t* __restrict__ in, uint64_t* __restrict__ out, const uint32_t* __restrict__ n_dev,
    uint32_t n_host, int shift, int bits, int groups, const uint32_t* __restrict__ hist,
    const uint32_t* __restrict__ totals, uint2* __restrict__ ranges, const uint32_t* __restrict__ dstats,
    int pass, const uint32_t* __restrict__ rect, int rect_direct, const uint32_t* __restrict__ pay_in,
    uint32_t* __restrict__ pay_out, SortRange sr) {
    GSR_GEOM_PRIO();
    constexpr int kTile = kSortThreads * ITEMS;
    __shared__ uint64_t s_items[kTile];
    if (sr.gate && *sr.gate == 0u) return;
    if (depth_pass_skipped(dstats, pass)) return;
    if (sr.base) {   // far part: the outputs start at *base, and so do the inputs unless filtered
        const uint32_t base = *sr.base;
        out += base;
        if (pay_out) pay_out += base;
        if (!FILT) {
            in += base;
            if (pay_in) pay_in += base;
        }
    }
    const uint32_t K = FILT ? *sr.kcut : 0u;
    const bool carry = pay_out != nullptr;
    __shared__ uint32_t s_wc[4][256];           // per-wave digit counters, then wave slot bases
    __shared__ uint32_t s_gd[256];              // per digit: global offset minus tile slot
    __shared__ uint32_t s_scr[4];
    // up to 8 items per thread the payloads get slots of their own (+8 KB of LDS, no
    // occupancy change) and travel with the items; at 16 the LDS is the occupancy
    // limit, so they reuse the items' slots in a second round (two more barriers)
    constexpr bool kPaySlots = ITEMS <= 8;
    __shared__ uint32_t s_payd[kPaySlots ? kTile : 1];
    const uint32_t t = threadIdx.x;
    const uint32_t lane = lane_id();
    const uint32_t w = t >> 6;
    const uint32_t mask = (1u << bits) - 1u;
    const uint64_t n = FILT ? (uint64_t)n_host : sort_len(sr, n_dev, n_host);
    uint64_t b, e;
    const int chunk = GSR_XCD_DEPTH && ITEMS == 16 ? xcd_chunk((int)blockIdx.x, groups) : (int)blockIdx.x;
    chunk_range(n, groups, chunk, kTile, b, e);

    // global base of each digit for this workgroup (a filtered pass 0: the kept count is
    // the sum of the digit totals)
    uint32_t gb;   // digit t's running global offset (thread t owns digit t)
    {
        uint32_t tot;
        const uint32_t dig_excl = block_exclusive_scan<uint32_t>(totals[t], s_scr, tot);
        gb = dig_excl + hist[t * (uint32_t)groups + chunk];
        if (FILT && sr.count_out && blockIdx.x == 0 && t == 0) *sr.count_out = tot;
    }
    if (b >= e) return;                          // uniform per workgroup
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

    for (uint64_t tb = b; tb < e; tb += kTile) {
        const uint32_t tn = (uint32_t)min((uint64_t)kTile, e - tb);
#pragma unroll
        for (int k = 0; k < 4; k++) s_wc[k][t] = 0;
        __syncthreads();

        uint64_t it[ITEMS];
        uint32_t rk[ITEMS], pv[ITEMS];
        bool kp[ITEMS];   // in the tile and kept (a filtered pass 0 drops the other part)
        const uint32_t wbase = w * 64 * ITEMS;
        // tile-relative 32-bit offsets from a uniform base: one address VGPR for all ITEMS
        // loads (64-bit per-item addresses had the 16-item kernel at 164+ VGPRs)
        const uint64_t* __restrict__ in_t = in + tb;
#pragma unroll
        for (int k = 0; k < ITEMS; k++) {
            const uint32_t el = wbase + k * 64 + lane;
            it[k] = (el < tn) ? in_t[el] : 0ull;
        }
        auto load_pay = [&]() {
            if (!carry) return;
            // uniform branches: the position-indexed reads must not wait for the item loads
            const uint32_t* src = (pay_in ? pay_in : rect) + tb;
            if (pay_in || rect_direct) {
#pragma unroll
                for (int k = 0; k < ITEMS; k++) {
                    const uint32_t el = wbase + k * 64 + lane;
                    pv[k] = (el < tn) ? src[el] : 0u;
                }
            } else {
#pragma unroll
                for (int k = 0; k < ITEMS; k++) {
                    const uint32_t el = wbase + k * 64 + lane;
                    pv[k] = (el < tn) ? rect[(uint32_t)it[k]] : 0u;
                }
            }
        };
        // a filtered pass 0 ranks by the payloads; otherwise they are loaded after the
        // ranking (their latency hides behind the tile scan, and the ranking holds 16 fewer
        // VGPRs at 16 items per thread)
        if (FILT) load_pay();
        uint32_t before[ITEMS];
#pragma unroll
        for (int k = 0; k < ITEMS; k++) {
            const uint32_t el = wbase + k * 64 + lane;
            const bool valid = el < tn && (!FILT || sort_keep(sr, K, it[k], pv[k]));
            kp[k] = valid;
            const uint32_t d = (uint32_t)(it[k] >> shift) & mask;
            // returning atomics at 4-8 items per thread; at 16 (4M+ items) ballot matching
            if (RA && ITEMS < 16) {
                rk[k] = valid ? atomicAdd(&s_wc[w][d], 1u) : 0u;
                before[k] = 0;
            } else {
                // every lane reads its digit's running count and the digit's leader adds the
                // slot's count without a return: a wave's LDS ops execute in issue order, so
                // slot k's read sees slots < k and no read is waited on before the next slot
                // (reading, waiting and writing back per slot serialised 16 LDS round trips)
                // (digits of fewer than 8 bits are masked: their high ballots match all)
                const uint64_t peers = match_peers<8>(d, valid, 8);
                rk[k] = (uint32_t)__popcll(peers & lt_mask);
                before[k] = s_wc[w][d];
                if (valid && (uint32_t)(__ffsll((unsigned long long)peers) - 1) == lane)
                    atomicAdd(&s_wc[w][d], (uint32_t)__popcll(peers));
                // the reads fold into the ranks every 4 slots (the compiler places the waits
                // for them; the VGPR peak came from hoisted loop invariants, see below)
                if ((k & 3) == 3)
#pragma unroll
                    for (int j = k - 3; j <= k; j++) rk[j] += before[j];
            }
        }
        if (!FILT) load_pay();
        __syncthreads();
        // per digit t: tile count, tile-local base, and each wave's first slot (tile base
        // included, so an item reads one word for its slot); the write-back's base is kept
        // as global offset minus tile slot (one word per item there too)
        uint32_t tcount, tv;   // tv: the tile's kept items (tn unless filtered)
        {
            const uint32_t c0 = s_wc[0][t], c1 = s_wc[1][t], c2 = s_wc[2][t], c3 = s_wc[3][t];
            tcount = c0 + c1 + c2 + c3;
            const uint32_t lb = block_exclusive_scan<uint32_t>(tcount, s_scr, tv);   // barriers: reads done
            s_wc[0][t] = lb;
            s_wc[1][t] = lb + c0;
            s_wc[2][t] = lb + c0 + c1;
            s_wc[3][t] = lb + c0 + c1 + c2;
            s_gd[t] = gb - lb;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < ITEMS; k++) {
            if (kp[k]) {
                const uint32_t d = (uint32_t)(it[k] >> shift) & mask;
                const uint32_t slot = s_wc[w][d] + rk[k];
                s_items[slot] = it[k];
                if (kPaySlots && carry) s_payd[slot] = pv[k];
                rk[k] = slot;   // the payload round's slot (the items die here)
            }
        }
        __syncthreads();
        // the digits of the items this thread wrote, four per word: the payload round
        // rebuilds their destinations from them (16 destinations held across the round
        // took the 16-item kernel to 179 VGPRs, two workgroups per CU)
        uint32_t dpk[(ITEMS + 3) / 4];
#pragma unroll
        for (int k = 0; k < (ITEMS + 3) / 4; k++) dpk[k] = 0;
#pragma unroll
        for (int k = 0; k < ITEMS; k++) {
            const uint32_t q = t + k * kSortThreads;
            if (q < tv) {
                const uint64_t v = s_items[q];
                const uint32_t d = (uint32_t)(v >> shift) & mask;
                const uint32_t dst = s_gd[d] + q;
                out[dst] = v;
                if (kPaySlots && carry) pay_out[dst] = s_payd[q];
                dpk[k / 4] |= d << (8 * (k % 4));
                if (ranges) {
                    // final pass of the tile sort: the LDS tile is fully sorted, so each
                    // run of one tile key is contiguous; record its global [start, end)
                    // as {~start, end} with atomicMax, so a zeroed array means "empty"
                    // (replaces a separate boundary-detection kernel).
                    const uint32_t key = (uint32_t)(v >> 32);
                    if (q == 0 || (uint32_t)(s_items[q - 1] >> 32) != key) atomicMax(&ranges[key].x, ~dst);
                    if (q == tv - 1 || (uint32_t)(s_items[q + 1] >> 32) != key) atomicMax(&ranges[key].y, dst + 1);
                }
            }
        }
        if (!kPaySlots && carry) {
            // the payloads take the items' LDS slots once every item is read, so their
            // stores leave in the same digit runs as the items' (coalesced)
            uint32_t* s_pay = reinterpret_cast<uint32_t*>(s_items);
            __syncthreads();
#pragma unroll
            for (int k = 0; k < ITEMS; k++)
                if (kp[k]) s_pay[rk[k]] = pv[k];
            __syncthreads();
#pragma unroll
            for (int k = 0; k < ITEMS; k++) {
                const uint32_t q = t + k * kSortThreads;
                const uint32_t d = (dpk[k / 4] >> (8 * (k % 4))) & 0xffu;
                if (q < tv) pay_out[s_gd[d] + q] = s_pay[q];
            }
        }
        // 16 items per thread: one tile per workgroup (launch_radix_pass checks the grid),
        // so the loop is straight-line code and nothing is hoisted across tiles (the
        // loop-invariant slot offsets of the write-back held 15 VGPRs for the whole kernel)
        if (ITEMS == 16) break;
        __syncthreads();   // every read of s_gd / s_wc done before the next tile's writes
        gb += tcount;
    }
}

// Key-value variant for the tile sort: keys of type K (uint16_t when the frame
// has <= 65536 tiles, else uint32_t) and uint32_t values in separate arrays,
// so the upsweep reads only the keys and the final pass writes only the values
// (plus the tile ranges).  Same reduce-then-scan structure and ranking.
template <typename K, int ITEMS>
__global__ __launch_bounds__(kSortThreads) void k_kv_upsweep(const K* __restrict__ keys,
                                                             const uint32_t* __restrict__ n_dev, int shift,
                                                             uint32_t mask, int groups,
                                                             uint32_t* __restrict__ hist) {
    GSR_GEOM_PRIO();
    __shared__ uint32_t h[4][256];
    const uint32_t t = threadIdx.x;
    const uint32_t w = t >> 6;
#pragma unroll
    for (int k = 0; k < 4; k++) h[k][t] = 0;
    __syncthreads();
    const uint64_t n = (uint64_t)*n_dev;
    uint64_t b, e;
    chunk_range(n, groups, blockIdx.x, kSortThreads * ITEMS, b, e);
    uint64_t i = b + t;
    for (; i + 3 * kSortThreads < e; i += 4 * kSortThreads) {
        const uint32_t k0 = keys[i], k1 = keys[i + kSortThreads], k2 = keys[i + 2 * kSortThreads],
                       k3 = keys[i + 3 * kSortThreads];
        atomicAdd(&h[w][(k0 >> shift) & mask], 1u);
        atomicAdd(&h[w][(k1 >> shift) & mask], 1u);
        atomicAdd(&h[w][(k2 >> shift) & mask], 1u);
        atomicAdd(&h[w][(k3 >> shift) & mask], 1u);
    }
    for (; i < e; i += kSortThreads) atomicAdd(&h[w][((uint32_t)keys[i] >> shift) & mask], 1u);
    __syncthreads();
    hist[t * (uint32_t)groups + blockIdx.x] = h[0][t] + h[1][t] + h[2][t] + h[3][t];
}

// keys_out == nullptr: final pass — write values only and record each tile's
// global [start, end) as {~start, end} (atomicMax; a zeroed array = empty).
template <typename K, int ITEMS>
__global__ __launch_bounds__(kSortThreads) void k_kv_downsweep(
    const K* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, K* __restrict__ keys_out,
    uint32_t* __restrict__ vals_out, const uint32_t* __restrict__ n_dev, int shift, int bits, int groups,
    const uint32_t* __restrict__ hist, const uint32_t* __restrict__ totals, uint2* __restrict__ ranges) {
    GSR_GEOM_PRIO();
    constexpr int kTile = kSortThreads * ITEMS;
    __shared__ K s_keys[kTile];
    __shared__ uint32_t s_vals[kTile];
    __shared__ uint32_t s_wc[4][256];
    __shared__ uint32_t s_gbase[256];
    __shared__ uint32_t s_lbase[256];
    __shared__ uint32_t s_scr[4];
    const uint32_t t = threadIdx.x;
    const uint32_t lane = lane_id();
    const uint32_t w = t >> 6;
    const uint32_t mask = (1u << bits) - 1u;
    const uint64_t n = (uint64_t)*n_dev;
    uint64_t b, e;
    chunk_range(n, groups, blockIdx.x, kTile, b, e);
    if (b >= e) return;
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
        uint32_t kk[ITEMS], vv[ITEMS], rk[ITEMS];
        const uint32_t wbase = w * 64 * ITEMS;
#pragma unroll
        for (int k = 0; k < ITEMS; k++) {
            const uint32_t el = wbase + k * 64 + lane;
            kk[k] = (el < tn) ? (uint32_t)keys_in[tb + el] : 0u;
            vv[k] = (el < tn) ? vals_in[tb + el] : 0u;
        }
#pragma unroll
        for (int k = 0; k < ITEMS; k++) {
            const uint32_t el = wbase + k * 64 + lane;
            const bool valid = el < tn;
            const uint32_t d = (kk[k] >> shift) & mask;
            const uint64_t peers = match_peers<8>(d, valid, bits);
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
                const uint32_t d = (kk[k] >> shift) & mask;
                const uint32_t q = s_lbase[d] + s_wc[w][d] + rk[k];
                s_keys[q] = (K)kk[k];
                s_vals[q] = vv[k];
            }
        }
        __syncthreads();
        for (uint32_t q = t; q < tn; q += kSortThreads) {
            const uint32_t key = s_keys[q];
            const uint32_t d = (key >> shift) & mask;
            const uint32_t dst = s_gbase[d] + (q - s_lbase[d]);
            vals_out[dst] = s_vals[q];
            if (keys_out) {
                keys_out[dst] = (K)key;
            } else {
                if (q == 0 || (uint32_t)s_keys[q - 1] != key) atomicMax(&ranges[key].x, ~dst);
                if (q == tn - 1 || (uint32_t)s_keys[q + 1] != key) atomicMax(&ranges[key].y, dst + 1);
            }
        }
        __syncthreads();
        s_gbase[t] += tcount;
    }
}

// ------------------------------------------------------------------ emission

// Tile counts in depth order.  The one random access of the emission — the
// compact rect of Gaussian sorted[j] — happens here, once; the rects are
// written back in depth order (srect) so k_emit_pairs reads them coalesced.
// Each thread issues all four of its index loads, then all four rect gathers,
// so the dependent gathers overlap instead of running back to back.
// The depth sort ends in items[passes run & 1] (trailing identity passes are
// skipped on the device); the other buffer is free for srect.
__device__ __forceinline__ const uint64_t* depth_sorted(const uint64_t* items0, const uint64_t* items1,
                                                        const uint32_t* dstats) {
    return (depth_passes_run(dstats) & 1) ? items1 : items0;
}
// The depth-ordered rect payloads the binning's depth sort carries (k_radix_downsweep):
// same parity as the items.
__device__ __forceinline__ const uint32_t* depth_sorted_rects(const uint32_t* pay0, const uint32_t* pay1,
                                                             const uint32_t* dstats) {
    return (depth_passes_run(dstats) & 1) ? pay1 : pay0;
}

__global__ __launch_bounds__(256) void k_emit_count(const uint64_t* __restrict__ items0,
                                                     const uint64_t* __restrict__ items1,
                                                     const uint32_t* __restrict__ dstats, uint32_t n,
                                                     const uint64_t* __restrict__ rect, int groups,
                                                     unsigned long long* __restrict__ wg_sum,
                                                     uint2* __restrict__ ranges, int ntiles) {
    GSR_GEOM_PRIO();
    __shared__ unsigned long long scr[4];
    // zero the tile ranges for the tile sort's final pass (a slice per workgroup)
    for (int q = blockIdx.x * 256 + threadIdx.x; q < ntiles; q += groups * 256) ranges[q] = make_uint2(0u, 0u);
    const uint64_t* sorted = depth_sorted(items0, items1, dstats);
    uint64_t* srect = const_cast<uint64_t*>(sorted == items0 ? items1 : items0);
    uint64_t b, e;
    chunk_range(n, groups, blockIdx.x, 1024, b, e);
    unsigned long long s = 0;
    for (uint64_t c0 = b; c0 < e; c0 += 1024) {
        uint32_t gi[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t j = c0 + threadIdx.x + 256 * k;
            gi[k] = j < e ? (uint32_t)sorted[j] : 0u;
        }
        uint64_t r[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t j = c0 + threadIdx.x + 256 * k;
            r[k] = j < e ? rect[gi[k]] : kDeadRect;
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t j = c0 + threadIdx.x + 256 * k;
            if (j < e) srect[j] = r[k];
            s += rect_count(r[k]);
        }
    }
    unsigned long long tot;
    block_exclusive_scan<unsigned long long>(s, scr, tot);
    if (threadIdx.x == 0) wg_sum[blockIdx.x] = tot;
}

// Exclusive scan of the per-workgroup pair counts + the frame's pair stats.
// (Folding it into k_emit_count's last-arriving workgroup was measured slower:
// the agent-scope fences before each arrival ticket write back the L2 on gfx950.)
__global__ __launch_bounds__(256) void k_emit_scan(unsigned long long* __restrict__ wg, int groups,
                                                    uint32_t cap, Stats* __restrict__ st,
                                                    Stats* host_st, uint32_t* fstatus) {
    GSR_GEOM_PRIO();
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
        Stats s{};
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
        if (fstatus) *fstatus = s.overflow;
        if (host_st) {
            host_st->pairs_total = k.pairs_total;
            host_st->pairs_eff = k.pairs_eff;
            host_st->overflow = k.overflow;
            __threadfence_system();
        }
    }
}

// One (tile key, Gaussian index) pair per covered tile, in depth order, as
// separate key (K = uint16_t or uint32_t) and value (uint32_t) arrays for the
// key-value tile sort [render.cu:788-809].  Each wave owns 256 consecutive
// Gaussians of the workgroup's 1024 and writes their pairs cooperatively:
// per round of 64 Gaussians, lane l of a 64-pair step finds its Gaussian by a
// binary search over the round's inclusive count prefix, so every store
// instruction writes 64 consecutive pairs.
template <typename K>
__global__ __launch_bounds__(256) void k_emit_pairs(const uint64_t* __restrict__ items0,
                                                     const uint64_t* __restrict__ items1,
                                                     const uint32_t* __restrict__ dstats, uint32_t n, int groups,
                                                     const unsigned long long* __restrict__ wg_base,
                                                     uint32_t cap, int tiles_x, K* __restrict__ keys,
                                                     uint32_t* __restrict__ vals) {
    GSR_GEOM_PRIO();
    __shared__ unsigned long long scr[4];
    __shared__ uint32_t s_incl[4][64], s_idx[4][64];
    __shared__ uint64_t s_rect[4][64];
    const uint64_t* sorted = depth_sorted(items0, items1, dstats);
    const uint64_t* srect = sorted == items0 ? items1 : items0;
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    uint64_t b, e;
    chunk_range(n, groups, blockIdx.x, 1024, b, e);
    unsigned long long run = wg_base[blockIdx.x];
    for (uint64_t c0 = b; c0 < e; c0 += 1024) {
        // this wave's 256 Gaussians: [c0 + 256 w, +256), four rounds of 64
        uint32_t cnt[4], gi[4];
        uint64_t r[4];
        uint32_t wtot = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t j = c0 + 256 * w + 64 * k + lane;
            gi[k] = j < e ? (uint32_t)sorted[j] : 0u;
            r[k] = j < e ? srect[j] : kDeadRect;
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            cnt[k] = rect_count(r[k]);
            wtot += cnt[k];
        }
        // wave totals -> exclusive base of this wave inside the 1024-chunk
        unsigned long long chunk_tot;
        const unsigned long long wsum = (unsigned long long)__reduce_add_sync(~0ull, wtot);
        const unsigned long long wbase = block_exclusive_scan<unsigned long long>(lane == 0 ? wsum : 0ull, scr,
                                                                                  chunk_tot);
        unsigned long long pos = run + (unsigned long long)__shfl(wbase, 0, 64);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            // inclusive prefix of the round's counts
            const uint32_t incl = wave_incl_scan(cnt[k], OpAdd{});
            const uint32_t rtot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            s_incl[w][lane] = incl;
            s_idx[w][lane] = gi[k];
            s_rect[w][lane] = r[k];
            for (uint32_t q = lane; q < rtot; q += 64) {
                // Gaussian l: the first lane whose inclusive prefix exceeds q
                uint32_t l = 0;
#pragma unroll
                for (uint32_t st = 32; st >= 1; st >>= 1)
                    if (s_incl[w][l + st - 1] <= q) l += st;
                const uint64_t rr = s_rect[w][l];
                const uint32_t before = s_incl[w][l] - rect_count(rr);   // exclusive prefix of Gaussian l
                const uint32_t k2 = q - before;
                const uint32_t tx0 = (uint32_t)(rr & 0xffffu), tx1 = (uint32_t)((rr >> 16) & 0xffffu);
                const uint32_t ty0 = (uint32_t)((rr >> 32) & 0xffffu);
                const uint32_t wdt = tx1 - tx0 + 1u;
                const uint32_t dy = k2 / wdt, dx = k2 - dy * wdt;
                const unsigned long long p = pos + q;
                if (p < cap) {
                    keys[p] = (K)((ty0 + dy) * (uint32_t)tiles_x + tx0 + dx);
                    vals[p] = s_idx[w][l];
                }
            }
            pos += rtot;
        }
        run += chunk_tot;
    }
}

// ------------------------------------------------------------------ tile binning
//
// For tile grids up to 256 x 256, two stable counting passes replace "emit every
// (tile, Gaussian) pair in depth order, then LSD-sort the pairs by tile":
//   row pass     each depth-ordered Gaussian expands into one item per covered
//                tile ROW (index | tx0 << 32 | tx1 << 48), binned stably by row:
//                ~2.4 items per Gaussian instead of ~5.6 pairs
//   column pass  each row's items expand into one value per covered tile COLUMN,
//                binned stably by column inside the row: the final tile-major,
//                depth-ordered Gaussian indices; the tile ranges come straight
//                from the column scan and no tile key is ever stored
// Each pass is count (per-chunk histograms) -> scan -> scatter.  The scatters
// rank one tile of generated items at a time in LDS (wave ballots on the digit
// bits) and write them digit run by digit run, so the stores coalesce.  Every
// source is processed in order and chunks are scanned in order: the result is
// the same stable order as the pair sort [render.cu:788-857].

constexpr uint32_t kRowSources = 1024;              // Gaussians per row-pass sub-chunk
// Row items per column-pass chunk (a chunk never crosses a row): 1,024 or 2,048, chosen
// per frame by the runtime (GSR_TUNE_COL_CHUNK).  Smaller chunks halve the scatter's
// per-chunk LDS (config 2: column scatter 26.0 -> 21.6 us); on config 3's ~9M row items
// the doubled chunk count costs the count and scan more (+10 us), so 2,048 stays there
// (profiles/r05_ab_col_chunk.txt).
constexpr uint32_t kColChunkMin = 1024, kColChunkMax = 2048;

__device__ __forceinline__ uint32_t rect_rows(uint64_t r) {
    return rect_count(r) ? (uint32_t)((r >> 48) - ((r >> 32) & 0xffffu) + 1u) : 0u;
}
__device__ __forceinline__ uint32_t rect_cols(uint64_t r) {
    return rect_count(r) ? (uint32_t)(((r >> 16) & 0xffffu) - (r & 0xffffu) + 1u) : 0u;
}

// Stable rank of one tile of up to 256*ITEMS items with BITS-bit digits.  Item
// k of thread t is tile element w*64*ITEMS + k*64 + lane (each wave's items are
// contiguous).  On return pos[k] is the item's slot in the digit-sorted tile,
// s_lbase[d] the first slot of digit d; returns the tile's count of digit t.
// Per k-slot every lane reads its digit's running wave count and the slot's
// leader of each digit ADDS the slot's count (ds_add, no return): LDS ops of a
// wave execute in issue order, so slot k's read sees slots < k and nothing waits
// on a read before the next slot is issued.
template <int ITEMS, int BITS, bool RA>
__device__ __forceinline__ uint32_t bin_rank_tile(const uint32_t (&dig)[ITEMS], uint32_t tn,
                                                  uint32_t (&pos)[ITEMS], uint32_t (*s_wc)[256],
                                                  uint32_t* s_lbase, uint32_t* s_scr) {
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (int k = 0; k < 4; k++) s_wc[k][t] = 0;
    __syncthreads();
    if (RA) {
#pragma unroll
        for (int k = 0; k < ITEMS; k++) {
            const uint32_t el = w * 64 * ITEMS + k * 64 + lane;
            pos[k] = el < tn ? atomicAdd(&s_wc[w][dig[k]], 1u) : 0u;
        }
    } else {
        uint32_t before[ITEMS], inslot[ITEMS];
#pragma unroll
        for (int k = 0; k < ITEMS; k++) {
            const uint32_t el = w * 64 * ITEMS + k * 64 + lane;
            const bool valid = el < tn;
            const uint32_t d = dig[k];
            const uint64_t peers = match_peers<BITS>(d, valid, BITS);
            inslot[k] = (uint32_t)__popcll(peers & lt_mask);
            before[k] = s_wc[w][d];
            if (valid && (uint32_t)(__ffsll((unsigned long long)peers) - 1) == lane)
                atomicAdd(&s_wc[w][d], (uint32_t)__popcll(peers));
        }
#pragma unroll
        for (int k = 0; k < ITEMS; k++) pos[k] = before[k] + inslot[k];
    }
    __syncthreads();
    uint32_t tcount;
    {
        // each wave's first slot of digit t, tile base included (s_wc[w][t] = s_lbase[t] +
        // the earlier waves' counts), so an item reads one word for its slot, not two
        const uint32_t c0 = s_wc[0][t], c1 = s_wc[1][t], c2 = s_wc[2][t], c3 = s_wc[3][t];
        tcount = c0 + c1 + c2 + c3;
        uint32_t tot;
        const uint32_t lb = block_exclusive_scan<uint32_t>(tcount, s_scr, tot);   // barriers: reads done
        s_lbase[t] = lb;
        s_wc[0][t] = lb;
        s_wc[1][t] = lb + c0;
        s_wc[2][t] = lb + c0 + c1;
        s_wc[3][t] = lb + c0 + c1 + c2;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < ITEMS; k++) {
        const uint32_t el = w * 64 * ITEMS + k * 64 + lane;
        if (el < tn) pos[k] += s_wc[w][dig[k]];
    }
    return tcount;
}

// Exclusive starts (in source order) of per-source counts cnt[] (thread t owns sources
// PER*t .. PER*t + PER-1): returns them in start[] and the total, and writes each with
// an 8-bit tag (the source's first row or column) to s_ft[s] = start << 8 | tag, so an
// element reads one word for both (starts stay below 2^24: <= 2,048 sources x 256
// digits).  Two barriers.
template <int PER>
__device__ __forceinline__ uint32_t bin_source_starts(const uint32_t (&cnt)[PER], uint32_t (&start)[PER],
                                                      const uint32_t (&tag)[PER], uint32_t* s_ft, uint32_t* s_scr) {
    const uint32_t t = threadIdx.x;
    uint32_t loc = 0;
#pragma unroll
    for (int i = 0; i < PER; i++) loc += cnt[i];
    uint32_t tot;
    uint32_t run = block_exclusive_scan<uint32_t>(loc, s_scr, tot);
#pragma unroll
    for (int i = 0; i < PER; i++) {
        start[i] = run;
        s_ft[PER * t + i] = (run << 8) | tag[i];
        run += cnt[i];
    }
    return tot;
}

// Source of every element of the tile [tb, tb + tn) of a generated stream,
// without a per-element search: each source starting inside the tile marks its
// first element (slot + 1) in s_own (cleared beforehand), then an in-order
// inclusive max-scan fills the runs.  `carry` (slot + 1 owning the element
// before the tile; 0 at a stream's start) seeds the scan and becomes the owner
// of the tile's last element.  The scan runs thread-major inside each wave
// (lane handles elements w*64*ITEMS + lane*ITEMS + i), so every wave scans its
// own ITEMS*64 elements in order.  Three barriers.
template <int ITEMS, int PER>
__device__ __forceinline__ void bin_tile_owners(const uint32_t (&cnt)[PER], const uint32_t (&start)[PER],
                                                uint32_t tb, uint32_t tn, uint16_t* s_own, uint32_t& carry,
                                                uint32_t* s_wmax) {
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
#pragma unroll
    for (int i = 0; i < PER; i++)
        if (cnt[i] && start[i] >= tb && start[i] < tb + tn) s_own[start[i] - tb] = (uint16_t)(PER * t + i + 1);
    __syncthreads();
    const uint32_t base = w * 64 * ITEMS + lane * ITEMS;
    uint32_t v[ITEMS], run = 0;
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        run = max(run, (uint32_t)s_own[base + i]);
        v[i] = run;
    }
    // exclusive max over the earlier lanes of the wave, then over earlier waves
    const uint32_t x = wave_incl_scan(run, OpMax{});
    if (lane == 63) s_wmax[w] = x;
    const uint32_t before = wave_shr1(x);
    __syncthreads();
    uint32_t cin = carry;
    for (uint32_t k = 0; k < w; k++) cin = max(cin, s_wmax[k]);
    cin = max(cin, before);
#pragma unroll
    for (int i = 0; i < ITEMS; i++) s_own[base + i] = (uint16_t)max(cin, v[i]);
    carry = max(max(carry, max(s_wmax[0], s_wmax[1])), max(s_wmax[2], s_wmax[3]));
    __syncthreads();
}

// Frame pair statistics (st[0]) + the sticky copy (st[1], and the host-mapped
// mirror) the non-blocking overflow check reads.
// Binning path: `needed` = depth passes the device plan asked for, `launched` = passes
// the host launched (its pass budget); needed > launched leaves the depth order
// incomplete, so the frame is flagged (overflow bit 1) and re-rendered like a
// pair-buffer overflow.  depth_passes is the latest frame's, not sticky.
// fstatus (nullable): the frame's validity word (gsr_render_path_status): set to the
// frame's overflow bits by its first column scan (fst_first: phase A or one phase),
// or-ed in by phase B's.
__device__ __forceinline__ void publish_pair_stats(unsigned long long total, uint32_t cap, Stats* st,
                                                   Stats* host_st, uint32_t needed = 0, uint32_t launched = 4,
                                                   uint32_t* fstatus = nullptr, bool fst_first = true) {
    Stats s{};
    s.pairs_total = total;
    s.pairs_eff = (uint32_t)(total < cap ? total : cap);
    s.overflow = (total > cap ? 1u : 0u) | (needed > launched ? 2u : 0u);
    s.depth_passes = needed;
    st[0] = s;
    Stats k = st[1];
    if (s.pairs_total > k.pairs_total) k.pairs_total = s.pairs_total;
    k.pairs_eff = s.pairs_eff;
    k.overflow |= s.overflow;
    k.depth_passes = s.depth_passes;
    st[1] = k;
    if (fstatus) {
        if (fst_first) *fstatus = s.overflow;
        else if (s.overflow) atomicOr(fstatus, s.overflow);
    }
    if (host_st) {
        host_st->pairs_total = k.pairs_total;
        host_st->pairs_eff = k.pairs_eff;
        host_st->overflow = k.overflow;
        host_st->depth_passes = k.depth_passes;
        __threadfence_system();
    }
}

// Depth-order positions a row pass reads: [base, base + n) as the host passed them, or
// with the depth split's device-side cut (the near part's size after the threshold
// partition): mode 1 = [0, min(cut, n)) (phase A), mode 2 = [cut, n) (phase B).
// (mode 2 with cut_n: the far part's kept length *cut_n, a masked far sort's count.)
__device__ __forceinline__ void row_range(uint32_t& base, uint32_t& n, const uint32_t* cut, int mode,
                                          const uint32_t* cut_n) {
    if (mode == 1) {
        n = min(*cut, n);
    } else if (mode == 2) {
        base = min(*cut, n);
        n -= base;
        if (cut_n) n = min(*cut_n, n);
    }
}

// ------------------------------------------------------------------ bucket depth sort
//
// The binning path's global depth sort in two global steps instead of three or four
// LSD passes (GSR_TUNE_DEPTH_BUCKETS).  Stable order of (depth key, index), exactly
// the LSD passes' order:
//   k_bkt_count    per workgroup chunk, the histogram over B buckets: bucket(key) =
//                  the number of splitters <= key (B - 1 sorted splitters in LDS; the
//                  last is 0xFFFFFFFF, so bucket B - 1 holds exactly the keys equal to
//                  0xFFFFFFFF: culled items and saturated live keys, which tie)
//   k_bkt_scan     per bucket, exclusive scan over the chunks (a chunk-major histogram:
//                  every access a coalesced row segment)
//   k_bkt_scatter  stable scatter of the preprocess order into the buckets (per-wave
//                  returning LDS atomics on packed 16-bit counters, so the rank of an
//                  item is its order among the wave's earlier items of its bucket);
//                  every item lands at its bucket's range, index-ordered inside it; the
//                  tile rects ride along as payloads
//   k_bkt_local    one workgroup per live bucket: load it (<= kBktCap items), stable
//                  LSD in LDS over the bits (key - bucket min) spans (typically 11 on
//                  config 2: two 8-bit passes), write it back in place.  A bucket over
//                  capacity is sorted by the same workgroup through global memory
//                  (stable 8-bit passes ping-ponging with the scratch buffer), so any
//                  splitters give the exact order; they only set the speed
// Splitters are the previous frame's quantiles: k_bkt_local writes the key at each
// bkt_split_pos of the live order for the next frame (double-buffered; the open first and
// last live buckets a quarter share, the rest even), so the buckets hold about n / B
// items each while the camera moves smoothly.  A context's
// first frame runs the LSD passes and k_bkt_splitters takes the quantiles from them.
// Stability: the scatter keeps index order inside a bucket, the local passes are stable
// and buckets are key ranges in order, so ties stay in index order — the same order as
// render.cu's CUB SortPairs of (tile << 32 | depth) within each tile (render.cu:1099-1118).
constexpr int kBktThreads = 256;
constexpr int kBktItems = 8;                                  // items per thread per tile
constexpr uint32_t kBktTile = kBktThreads * kBktItems;        // 2048
constexpr uint32_t kBktCap = kBktTile;                        // local sort capacity (items)
static_assert(kBktCap == kMaxBucketCap && kMaxBuckets == 4096, "gsr_internal.h bucket sort limits");

// The splitters in LDS as an implicit search tree in breadth-first (Eytzinger) order:
// node i at depth d, position p = i + 1 - 2^d holds the sorted splitter of rank
// (2p + 1) 2^(h - 1 - d) - 1 (h = log2 B; the B - 1 splitters fill the tree exactly).  Each
// search step reads one tree level, and a level's nodes are consecutive words.  (The plain
// sorted array put every address of the first search steps on ONE LDS bank -- b + st - 1
// with b a multiple of 2 st -- up to 32-way conflicts: the count kernel took 10 us.)
template <int B, int TH = kBktThreads>
__device__ __forceinline__ void bkt_load_splitters(uint32_t* s_T, const uint32_t* __restrict__ splitters) {
    // B / TH nodes per thread, every load issued before the first LDS write: a rolled
    // loop waited for each load in turn (four serial memory round trips at B = 1,024)
    static_assert(B >= TH, "one node per thread at least");
    constexpr int h = __builtin_ctz(B);
    constexpr int kPer = B / TH;
    uint32_t v[kPer], jj[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const uint32_t i = threadIdx.x + (uint32_t)k * TH;
        const int d = 31 - __clz((int)(i + 1u));
        const uint32_t p = i + 1u - (1u << d);
        const int sh = h - 1 - d;                               // < 0 only for i = B - 1 (no node)
        jj[k] = sh >= 0 ? ((2u * p + 1u) << sh) - 1u : (uint32_t)B - 2u;   // sorted rank
        v[k] = splitters[min(jj[k], (uint32_t)B - 3u)];
    }
#pragma unroll
    for (int k = 0; k < kPer; k++)
        s_T[threadIdx.x + (uint32_t)k * TH] = jj[k] < (uint32_t)B - 2u ? v[k] : 0xffffffffu;
}

// The buckets of N keys: bucket(key) = the number of the B - 1 sorted splitters that are
// <= key (the last is 0xFFFFFFFF, so a key 0xFFFFFFFF lands in bucket B - 1), by a walk
// down the tree of bkt_load_splitters.  Level by level, so each level's N LDS reads are in
// flight together.
template <int B, int N>
__device__ __forceinline__ void bkt_of_n(const uint32_t* s_T, const uint32_t (&key)[N], uint32_t (&bk)[N]) {
#pragma unroll
    for (int k = 0; k < N; k++) bk[k] = 0;
#pragma unroll
    for (int lvl = 0; lvl < __builtin_ctz(B); lvl++) {
        uint32_t v[N];
#pragma unroll
        for (int k = 0; k < N; k++) v[k] = s_T[bk[k]];
#pragma unroll
        for (int k = 0; k < N; k++) bk[k] = 2u * bk[k] + (v[k] <= key[k] ? 2u : 1u);
    }
#pragma unroll
    for (int k = 0; k < N; k++) bk[k] -= (uint32_t)B - 1u;
}

template <int B>
__global__ __launch_bounds__(kBktThreads) void k_bkt_count(const uint64_t* __restrict__ in, uint32_t n,
                                                           const uint32_t* __restrict__ splitters, int groups,
                                                           uint32_t* __restrict__ hist,
                                                           uint16_t* __restrict__ bid = nullptr) {
    GSR_GEOM_PRIO();
    __shared__ uint32_t s_S[B], s_h[B];
    const uint32_t t = threadIdx.x, lane = t & 63u;
    uint64_t b, e;
    chunk_range(n, groups, blockIdx.x, kBktTile, b, e);
    uint32_t key[kBktItems];
    auto load = [&](uint64_t i0, uint32_t (&kk)[kBktItems]) {
#pragma unroll
        for (int k = 0; k < kBktItems; k++) {
            const uint64_t i = i0 + (uint64_t)k * kBktThreads + t;
            kk[k] = i < e ? (uint32_t)(in[i] >> 32) : 0xffffffffu;
        }
    };
    load(b, key);   // the first tile's keys travel together with the splitters: one memory round trip
    bkt_load_splitters<B>(s_S, splitters);
    for (uint32_t j = t; j < (uint32_t)B; j += kBktThreads) s_h[j] = 0;
    __syncthreads();
    uint32_t dead = 0;   // culled items all share the last bucket: counted by ballots, not 64-way atomics
    for (uint64_t i0 = b; i0 < e; i0 += kBktTile) {
        // the next tile's keys are in flight while this tile walks the tree (scenes above
        // 1M items give a workgroup several tiles)
        uint32_t nkey[kBktItems];
        if (i0 + kBktTile < e) load(i0 + kBktTile, nkey);
        uint32_t bk[kBktItems];
        bkt_of_n<B>(s_S, key, bk);
#pragma unroll
        for (int k = 0; k < kBktItems; k++) {
            const uint64_t i = i0 + (uint64_t)k * kBktThreads + t;
            const bool d = key[k] == 0xffffffffu;
            dead += (uint32_t)__popcll(__ballot(d && i < e));
            if (!d) atomicAdd(&s_h[bk[k]], 1u);
            if (bid && i < e) bid[i] = (uint16_t)bk[k];   // the scatter reads it instead of searching again
        }
        if (i0 + kBktTile < e) {
#pragma unroll
            for (int k = 0; k < kBktItems; k++) key[k] = nkey[k];
        }
    }
    if (lane == 0 && dead) atomicAdd(&s_h[B - 1], dead);
    __syncthreads();
    // chunk-major (hist[chunk][bucket]): this workgroup's row is one coalesced 4B-per-bucket run
    // (bucket-major, each of its B words went to another cache line: 15 us for 1M items)
    for (uint32_t j = t; j < (uint32_t)B; j += kBktThreads) hist[(size_t)blockIdx.x * B + j] = s_h[j];
}

// Per bucket, the exclusive scan over the chunks of the chunk-major histogram (in place)
// and the bucket's total.  64 buckets per workgroup (one per lane), 16 waves splitting the
// chunks: every load is a coalesced 256-B row segment.  groups <= kBktMaxGroups.
constexpr int kBktMaxGroups = kMaxBucketGroups;
template <int B, int MAXG = kBktMaxGroups>
__global__ __launch_bounds__(1024) void k_bkt_scan(uint32_t* __restrict__ hist, int groups,
                                                   uint32_t* __restrict__ totals) {
    GSR_GEOM_PRIO();
    constexpr int kPerMax = MAXG / 16;
    __shared__ uint32_t s_part[16][64];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint32_t b = blockIdx.x * 64u + lane;
    const uint32_t per = ((uint32_t)groups + 15u) / 16u;
    const uint32_t g0 = w * per;
    uint32_t v[kPerMax], sum = 0;
#pragma unroll
    for (int i = 0; i < kPerMax; i++) {
        const uint32_t g = g0 + (uint32_t)i;
        v[i] = (uint32_t)i < per && g < (uint32_t)groups ? hist[(size_t)g * B + b] : 0u;
        sum += v[i];
    }
    s_part[w][lane] = sum;
    __syncthreads();
    uint32_t run = 0, tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; k++) {
        const uint32_t p = s_part[k][lane];
        run += k < w ? p : 0u;
        tot += p;
    }
    if (w == 0) totals[b] = tot;
    // the frame's "a live item has key 0xFFFFFFFF" word (bkt_sat_word), raised by the scatter
    if (blockIdx.x == 0 && t == 0) totals[2 * B + 1] = 0u;
#pragma unroll
    for (int i = 0; i < kPerMax; i++) {
        const uint32_t g = g0 + (uint32_t)i;
        if ((uint32_t)i < per && g < (uint32_t)groups) {
            hist[(size_t)g * B + b] = run;
            run += v[i];
        }
    }
}

// Big buckets (many chunks): one wave per bucket, its lanes splitting the chunks (up to
// MAXG / 64 each, loads issued together), a wave scan over the lanes.  B / 4 workgroups of
// four waves: the per-bucket layout of k_bkt_scan put 1.25 MB through 8 workgroups (23 us at
// 611 chunks).
template <int B, int MAXG>
__global__ __launch_bounds__(256) void k_bkt_scan_w(uint32_t* __restrict__ hist, int groups,
                                                    uint32_t* __restrict__ totals) {
    GSR_GEOM_PRIO();
    constexpr int kPerMax = MAXG / 64;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t b = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t per = ((uint32_t)groups + 63u) / 64u;
    const uint32_t g0 = lane * per;
    uint32_t v[kPerMax], sum = 0;
#pragma unroll
    for (int i = 0; i < kPerMax; i++) {
        const uint32_t g = g0 + (uint32_t)i;
        v[i] = (uint32_t)i < per && g < (uint32_t)groups ? hist[(size_t)g * B + b] : 0u;
        sum += v[i];
    }
    const uint32_t incl = wave_incl_scan(sum, OpAdd{});
    uint32_t run = incl - sum;
    if (lane == 63) totals[b] = incl;
    if (b == 0 && lane == 0) totals[2 * B + 1] = 0u;   // bkt_sat_word (as k_bkt_scan)
#pragma unroll
    for (int i = 0; i < kPerMax; i++) {
        const uint32_t g = g0 + (uint32_t)i;
        if ((uint32_t)i < per && g < (uint32_t)groups) {
            hist[(size_t)g * B + b] = run;
            run += v[i];
        }
    }
}

// Big buckets (A/B, GSR_BB_SCANG=1): 16 buckets per 1,024-thread workgroup, each wave's four
// 16-lane quarters reading a 64-B row segment of four different chunks (64 chunk slices per
// workgroup), the slices' sums combined in LDS.  B / 16 workgroups.
template <int B, int MAXG>
__global__ __launch_bounds__(1024) void k_bkt_scan_g(uint32_t* __restrict__ hist, int groups,
                                                     uint32_t* __restrict__ totals) {
    GSR_GEOM_PRIO();
    constexpr int kPerMax = (MAXG + 63) / 64;
    __shared__ uint32_t s_part[64][16];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint32_t bl = lane & 15u, sl = w * 4u + (lane >> 4);   // bucket in the group, chunk slice
    const uint32_t b = blockIdx.x * 16u + bl;
    const uint32_t per = ((uint32_t)groups + 63u) / 64u;
    const uint32_t g0 = sl * per;
    uint32_t v[kPerMax], sum = 0;
#pragma unroll
    for (int i = 0; i < kPerMax; i++) {
        const uint32_t g = g0 + (uint32_t)i;
        v[i] = (uint32_t)i < per && g < (uint32_t)groups ? hist[(size_t)g * B + b] : 0u;
        sum += v[i];
    }
    s_part[sl][bl] = sum;
    __syncthreads();
    uint32_t run = 0, tot = 0;
    for (uint32_t k = 0; k < 64u; k++) {
        const uint32_t p = s_part[k][bl];
        run += k < sl ? p : 0u;
        tot += p;
    }
    if (sl == 0) totals[b] = tot;
    if (blockIdx.x == 0 && t == 0) totals[2 * B + 1] = 0u;   // bkt_sat_word (as k_bkt_scan)
#pragma unroll
    for (int i = 0; i < kPerMax; i++) {
        const uint32_t g = g0 + (uint32_t)i;
        if ((uint32_t)i < per && g < (uint32_t)groups) {
            hist[(size_t)g * B + b] = run;
            run += v[i];
        }
    }
}

// 16-bit half h of the packed counter word v.
__device__ __forceinline__ uint32_t half16(uint32_t v, uint32_t h) { return (v >> (16u * h)) & 0xffffu; }

// Bucket records: 16 B {index, key, rect, 0} (R12 false: one store request per item in the
// unstaged scatter), or 12 B {index, key, rect} (R12: the staged scatter writes runs, where
// the bytes, not the requests, bound it; a quarter fewer of them).
struct __attribute__((packed, aligned(4))) BktRec12 {
    uint32_t i, k, r;
};
template <bool R12>
__device__ __forceinline__ uint4 rec_get(const uint4* __restrict__ rec, uint32_t q) {
    if (R12) {
        const BktRec12 v = reinterpret_cast<const BktRec12*>(rec)[q];
        return make_uint4(v.i, v.k, v.r, 0u);
    }
    return rec[q];
}
template <bool R12>
__device__ __forceinline__ void rec_put(uint4* __restrict__ rec, uint32_t q, uint32_t i, uint32_t k, uint32_t r) {
    if (R12) reinterpret_cast<BktRec12*>(rec)[q] = BktRec12{i, k, r};
    else rec[q] = make_uint4(i, k, r, 0u);
}

// bstart (B + 2 words): written by chunk 0's workgroup, the first position of every bucket
// and bstart[B] = n (k_bkt_local reads its bucket's range there); bstart[B + 1] (cleared by
// k_bkt_scan) is raised when a live item (a tile rect that covers tiles) has key 0xFFFFFFFF.
// TH threads (512 from 512 buckets up: twice the waves of 256, half the items per wave, so
// each wave's latency chain is half as long; the grid is only ~n / 2,048 workgroups:
// 16.3-16.8 -> 15.6-15.8 us at config 2, profiles/r05_kt_bkt_scatter512.txt).
// Live items go out as one 16-B record {index, key, rect, 0} into rec (one store request per
// item: a 4,096-way scatter writes ~one item per bucket per tile, so every store of a wave hits
// its own cache line and the scatter is bound by the L2's request rate, not by bytes: two
// arrays, item and rect, were two requests per item); k_bkt_local reads a bucket's records
// back contiguously.  The last bucket (key 0xFFFFFFFF, never sorted) goes straight to its
// final place in out / pay_out.  The next tile's items and rects are loaded while this one
// is ranked.
// STAGE: the tile is laid out in LDS by bucket first (tile-local position = the bucket's
// offset in the tile + the item's stable rank in it), then written out by position, so the
// lanes of a store that hold items of one bucket write consecutive records (a run per bucket
// and tile: ~4 items at 512 buckets) instead of one store request each.
template <int B, bool RA, int TH, bool STAGE = false, uint32_t TILE = kBktTile, int WPE = 1, bool R12 = false,
          bool LEAN = false, bool BID = false>
__global__ __launch_bounds__(TH) __attribute__((amdgpu_waves_per_eu(WPE))) void k_bkt_scatter(const uint64_t* __restrict__ in,
                                                             uint64_t* __restrict__ out, uint32_t n,
                                                             const uint32_t* __restrict__ splitters, int groups,
                                                             const uint32_t* __restrict__ hist,
                                                             const uint32_t* __restrict__ totals,
                                                             const uint32_t* __restrict__ rect,
                                                             uint32_t* __restrict__ pay_out,
                                                             uint32_t* __restrict__ bstart,
                                                             uint4* __restrict__ rec,
                                                             const uint16_t* __restrict__ bid) {
    GSR_GEOM_PRIO();
    constexpr int NW = TH / 64, kIt = TILE / TH;  // waves; items per thread
    constexpr uint32_t kW = B / 2;                      // packed counter words per wave
    constexpr int kPer = B / TH;                        // buckets per thread (scan)
    constexpr int kWPer = (kW + TH - 1) / TH;           // counter words per thread
    static_assert(kPer >= 1 && kIt * TH == TILE && TILE % kBktTile == 0, "bucket / thread split");
    // LEAN (staged, one counter word per thread): thread t < kW owns word t (buckets 2t, 2t + 1),
    // so its wave prefix and the tile offsets' scan are one step (no s_tc, one barrier fewer);
    // the scan keeps only its first barrier, and the counters are cleared for the next tile
    // after their last read (the stage writes), so the tile starts without a clear + barrier:
    // five barriers per tile instead of eight
    constexpr bool kLean = LEAN && STAGE && kW <= (uint32_t)TH;
    __shared__ uint32_t s_S[B], s_gbase[B];
    __shared__ uint32_t s_wc[NW][kW];
    __shared__ uint32_t s_scr[NW];
    // STAGE: per-word tile counts, per-bucket tile offsets, the tile in bucket order
    __shared__ uint32_t s_tc[STAGE ? kW : 1], s_tp[STAGE ? B : 1];
    __shared__ uint4 s_stage[STAGE ? TILE : 1];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint64_t lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const int chunk = xcd_chunk((int)blockIdx.x, groups);   // each XCD takes a contiguous run of chunks
    uint64_t b, e;
    chunk_range(n, groups, chunk, kBktTile, b, e);   // chunks as k_bkt_count's
    const uint32_t wbase = w * 64 * kIt;
    uint64_t it[kIt];
    uint32_t pv[kIt], bv[kIt];
    // BID: the count kernel's bucket of every item (bid), loaded with the tile
    auto load = [&](uint64_t tb, uint32_t tn, uint64_t (&ii)[kIt], uint32_t (&pp)[kIt], uint32_t (&bb)[kIt]) {
#pragma unroll
        for (int k = 0; k < kIt; k++) {
            const uint32_t el = wbase + k * 64 + lane;
            ii[k] = el < tn ? in[tb + el] : ~0ull;
            pp[k] = el < tn ? rect[tb + el] : 0u;   // the input is the preprocess order: rect by position
            if (BID) bb[k] = el < tn ? (uint32_t)bid[tb + el] : (uint32_t)B - 1u;
        }
    };
    // the first tile's items and rects, the splitters, the bucket totals and this chunk's
    // histogram row are all loaded in one memory round trip
    load(b, (uint32_t)min((uint64_t)TILE, e - b), it, pv, bv);
    if (!BID) bkt_load_splitters<B, TH>(s_S, splitters);
    {   // this chunk's first slot in every bucket: the bucket's start + the earlier chunks' items
        uint32_t loc[kPer], hrow[kPer], sum = 0;
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            loc[k] = totals[t * kPer + k];
            hrow[k] = hist[(size_t)chunk * B + t * kPer + k];
            sum += loc[k];
        }
        uint32_t tot;
        uint32_t run = block_exclusive_scan<uint32_t, NW>(sum, s_scr, tot);
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const uint32_t d = t * kPer + k;
            if (chunk == 0) bstart[d] = run;
            s_gbase[d] = run + hrow[k];
            run += loc[k];
        }
        if (chunk == 0 && t == 0) bstart[B] = n;
    }
    if (b >= e) return;   // uniform per workgroup, after the scan's barriers
    if (kLean) {
        for (uint32_t j = t; j < NW * kW; j += TH) (&s_wc[0][0])[j] = 0;
        __syncthreads();
    }
    for (uint64_t tb = b; tb < e; tb += TILE) {
        const uint32_t tn = (uint32_t)min((uint64_t)TILE, e - tb);
        const bool more = tb + TILE < e;   // uniform
        uint64_t nit[kIt];
        uint32_t npv[kIt], nbv[kIt];
        if (more) load(tb + TILE, (uint32_t)min((uint64_t)TILE, e - tb - TILE), nit, npv, nbv);
        if (!kLean) {
            for (uint32_t j = t; j < NW * kW; j += TH) (&s_wc[0][0])[j] = 0;
            __syncthreads();
        }
        uint32_t dg[kIt], rk[kIt], keys[kIt];
#pragma unroll
        for (int k = 0; k < kIt; k++) keys[k] = (uint32_t)(it[k] >> 32);
        if (BID) {
#pragma unroll
            for (int k = 0; k < kIt; k++) dg[k] = bv[k];
        } else {
            bkt_of_n<B>(s_S, keys, dg);   // a key 0xFFFFFFFF (culled) counts every splitter: bucket B - 1
        }
        // culled items (the last bucket) rank by ballot against a running wave count, so the
        // live items' returning atomics have no LDS read between them and stay in flight together
        uint32_t dead_run = 0;
        uint32_t old[kIt];
#pragma unroll
        for (int k = 0; k < kIt; k++) {
            const uint32_t el = wbase + k * 64 + lane;
            const bool valid = el < tn;
            const bool dead = keys[k] == 0xffffffffu;
            const uint32_t d = dg[k];
            // a live Gaussian whose key saturated (depth >= ~4295 under a far clip that keeps
            // it) shares the last bucket with the culled items: k_bkt_local's fused row count
            // must then bin that bucket too (rare: a plain vector store of 1)
            if (valid && dead && rect_count(unpack_rect(pv[k]))) bstart[B + 1] = 1u;
            const uint64_t dm = __ballot(valid && dead);
            uint32_t r = dead_run + (uint32_t)__popcll(dm & lt_mask);
            dead_run += (uint32_t)__popcll(dm);
            const uint32_t sh = 16u * (d & 1u);
            if (RA) {
                // every lane adds (0 when it has no live item): no branch, so the eight returning
                // atomics are in flight together; the halves are taken after the loop
                old[k] = atomicAdd(&s_wc[w][d >> 1], valid && !dead ? 1u << sh : 0u);
            } else {
                const uint64_t peers = match_peers<12>(d, valid && !dead, 12);   // every lane takes part
                if (valid && !dead) {
                    r = half16(s_wc[w][d >> 1], d & 1u) + (uint32_t)__popcll(peers & lt_mask);
                    if (lane == (uint32_t)(__ffsll((unsigned long long)peers) - 1))
                        atomicAdd(&s_wc[w][d >> 1], (uint32_t)__popcll(peers) << sh);
                }
            }
            rk[k] = r;
        }
        if (RA) {
#pragma unroll
            for (int k = 0; k < kIt; k++)
                if (keys[k] != 0xffffffffu) rk[k] = half16(old[k], dg[k] & 1u);
        }
        if (lane == 0 && dead_run) atomicAdd(&s_wc[w][(B - 1) >> 1], dead_run << 16);   // B - 1 is odd: high half
        __syncthreads();
        // per word (two buckets): exclusive prefix over the waves in place, tile counts kept
        // (halves <= TILE <= 32,768: no carry between them)
        uint32_t tc[kWPer];
#pragma unroll
        for (int q = 0; q < kWPer; q++) {
            const uint32_t j = t + q * TH;
            tc[q] = 0;
            if (j < kW) {
                uint32_t c[NW];
#pragma unroll
                for (int v = 0; v < NW; v++) c[v] = s_wc[v][j];
                uint32_t run = 0;
#pragma unroll
                for (int v = 0; v < NW; v++) {
                    s_wc[v][j] = run;
                    run += c[v];
                }
                tc[q] = run;
                if (STAGE && !kLean) s_tc[j] = run;
            }
        }
        if (kLean) {
            // the buckets' offsets in the tile: thread t < kW scans word t's two tile counts
            const uint32_t lo = tc[0] & 0xffffu, hi = tc[0] >> 16;
            uint32_t tot;
            const uint32_t ex = block_exclusive_scan_lead<uint32_t, NW>(t < kW ? lo + hi : 0u, s_scr, tot);
            if (t < kW) {
                s_tp[2 * t] = ex;
                s_tp[2 * t + 1] = ex + lo;
            }
            __syncthreads();
        } else {
            __syncthreads();
        }
        if (STAGE && !kLean) {
            // the buckets' offsets in the tile: exclusive scan of their tile counts (thread t
            // owns buckets t * kPer .. + kPer - 1)
            uint32_t c[kPer], sum = 0;
#pragma unroll
            for (int k = 0; k < kPer; k++) {
                const uint32_t d = t * kPer + k;
                c[k] = half16(s_tc[d >> 1], d & 1u);
                sum += c[k];
            }
            uint32_t tot;
            uint32_t run = block_exclusive_scan<uint32_t, NW>(sum, s_scr, tot);
#pragma unroll
            for (int k = 0; k < kPer; k++) {
                s_tp[t * kPer + k] = run;
                run += c[k];
            }
            __syncthreads();
        }
        if (STAGE) {
#pragma unroll
            for (int k = 0; k < kIt; k++) {
                const uint32_t el = wbase + k * 64 + lane;
                if (el < tn) {
                    const uint32_t d = dg[k];
                    const uint32_t p = s_tp[d] + half16(s_wc[w][d >> 1], d & 1u) + rk[k];
                    s_stage[p] = make_uint4((uint32_t)it[k], (uint32_t)(it[k] >> 32), pv[k], d);
                }
            }
            __syncthreads();
            if (kLean)   // the counters' last read is behind: clear them for the next tile
                for (uint32_t j = t; j < NW * kW; j += TH) (&s_wc[0][0])[j] = 0;
            for (uint32_t q = t; q < tn; q += TH) {
                const uint4 r = s_stage[q];
                const uint32_t d = r.w;
                const uint32_t dst = s_gbase[d] + (q - s_tp[d]);
                if (d == (uint32_t)B - 1u) {
                    out[dst] = ((uint64_t)r.y << 32) | r.x;
                    pay_out[dst] = r.z;
                } else {
                    rec_put<R12>(rec, dst, r.x, r.y, r.z);
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < kIt; k++) {
                const uint32_t el = wbase + k * 64 + lane;
                if (el < tn) {
                    const uint32_t d = dg[k];
                    const uint32_t dst = s_gbase[d] + half16(s_wc[w][d >> 1], d & 1u) + rk[k];
                    if (d == (uint32_t)B - 1u) {
                        out[dst] = it[k];
                        pay_out[dst] = pv[k];
                    } else {
                        rec_put<R12>(rec, dst, (uint32_t)it[k], (uint32_t)(it[k] >> 32), pv[k]);
                    }
                }
            }
        }
        if (more) {
#pragma unroll
            for (int k = 0; k < kIt; k++) {
                it[k] = nit[k];
                pv[k] = npv[k];
                if (BID) bv[k] = nbv[k];
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kWPer; q++) {
            const uint32_t j = t + q * TH;
            if (j < kW) {
                s_gbase[2 * j] += tc[q] & 0xffffu;
                s_gbase[2 * j + 1] += tc[q] >> 16;
            }
        }
        // the next tile's counter reset + barrier orders these updates before their use
    }
}

// Next frame's splitters from this bucket's part of the sorted live order: splitter j is
// the key at live position floor((j + 1) * live / (B - 1)), j < B - 2.  key_at(q) reads
// the sorted key at bucket-local position q.
// Where splitter j (j < B - 2) is taken in a sorted live order of `live` items: the open
// first and last live buckets get a quarter of an interior bucket's share, so a moving
// camera's drift past the previous frame's nearest and farthest keys (which lands in
// them) has room under the local capacity (config 2 on a 0.25-deg orbit, the first frames
// after the LSD quantiles: the last bucket held 2,058 items, over the 2,048 capacity, at
// an even split).  pos(j) = floor(N(j) live / D), N(j) = (B - 3) + j (4B - 6),
// D = 4 (B - 3)(B - 1): pos(0) = live / (4 (B - 1)), pos(B - 3) = live (1 - 1 / (4 (B - 1))).
template <int B>
__device__ __forceinline__ uint32_t bkt_split_pos(uint32_t j, uint32_t live) {
    constexpr uint64_t D = 4ull * (uint64_t)(B - 3) * (uint64_t)(B - 1);
    return (uint32_t)(((uint64_t)(B - 3) + (uint64_t)j * (uint64_t)(4 * B - 6)) * live / D);
}
// The smallest j with bkt_split_pos(j, live) >= s (live > 0).
template <int B>
__device__ __forceinline__ uint64_t bkt_split_first(uint64_t s, uint32_t live) {
    constexpr uint64_t D = 4ull * (uint64_t)(B - 3) * (uint64_t)(B - 1);
    const uint64_t c = (s * D + live - 1) / live;   // pos(j) >= s  <=>  N(j) >= c
    return c <= (uint64_t)(B - 3) ? 0ull : (c - (uint64_t)(B - 3) + (uint64_t)(4 * B - 7)) / (uint64_t)(4 * B - 6);
}

template <int B, int TH = kBktThreads, typename KeyAt>
__device__ __forceinline__ void bkt_write_splitters(uint32_t start, uint32_t count, uint32_t live,
                                                    uint32_t* __restrict__ s_out, KeyAt key_at) {
    if (live == 0 || count == 0) return;
    // splitters j in [j0, j1) are taken at positions in [start, start + count)
    const uint64_t j0 = bkt_split_first<B>(start, live);
    const uint64_t j1 = min(bkt_split_first<B>((uint64_t)start + count, live), (uint64_t)B - 2u);
    for (uint64_t j = j0 + threadIdx.x; j < j1; j += TH)
        s_out[j] = key_at(bkt_split_pos<B>((uint32_t)j, live) - start);
}

// Row-pass histograms of one chunk of the depth order (k_bin_rows_count's, for the chunk
// of the bucket this workgroup sorted): per tile row the row items and the pairs of its
// rects, as difference arrays in LDS (per wave), then a prefix over the rows.
// hist[row][g] and hist[256 + row][g], rows < tiles_y.
struct RowHist {
    uint32_t* hist;      // nullptr: not fused (the row pass counts for itself)
    int groups;          // the row pass's chunks: the live buckets (B - 1)
    int tiles_y;
};

__device__ __forceinline__ void row_hist_add(uint32_t (*h_items)[256], uint32_t (*h_pairs)[256], uint32_t w,
                                             uint32_t packed) {
    const uint64_t r = unpack_rect(packed);
    if (rect_count(r)) {
        const uint32_t ty0 = (uint32_t)((r >> 32) & 0xffffu), ty1 = (uint32_t)(r >> 48);
        const uint32_t cols = rect_cols(r);
        atomicAdd(&h_items[w][ty0], 1u);
        atomicAdd(&h_pairs[w][ty0], cols);
        if (ty1 < 255u) {
            atomicSub(&h_items[w][ty1 + 1], 1u);
            atomicSub(&h_pairs[w][ty1 + 1], cols);
        }
    }
}

__device__ __forceinline__ void row_hist_write(const RowHist& rh, uint32_t g, uint32_t (*h_items)[256],
                                               uint32_t (*h_pairs)[256], uint32_t* s_scr) {
    const uint32_t t = threadIdx.x;
    __syncthreads();
    const uint32_t di = h_items[0][t] + h_items[1][t] + h_items[2][t] + h_items[3][t];
    const uint32_t dp = h_pairs[0][t] + h_pairs[1][t] + h_pairs[2][t] + h_pairs[3][t];
    uint32_t ti, tp;
    const uint32_t ci = block_exclusive_scan<uint32_t>(di, s_scr, ti) + di;
    const uint32_t cp = block_exclusive_scan<uint32_t>(dp, s_scr, tp) + dp;
    if (t < (uint32_t)rh.tiles_y) {
        rh.hist[t * (uint32_t)rh.groups + g] = ci;
        rh.hist[(256 + t) * (uint32_t)rh.groups + g] = cp;
    }
}

// One workgroup per live bucket (grid B - 1; B with the fused row count, whose last
// workgroup only counts the last bucket's rows).  bstart: the buckets' first positions
// (k_bkt_scatter); s_in: the splitters this frame was bucketed by, which bound the keys of
// every bucket but the first and the last (their key span sets the passes).  cap: buckets
// above it take the global path (kBktCap; smaller only as a test hook).  over_host
// (host-mapped, nullable): items sorted by the global path, for the diagnostics.
template <int B, bool RA, bool R12 = false>
__global__ __launch_bounds__(kBktThreads) void k_bkt_local(uint64_t* __restrict__ items, uint64_t* __restrict__ scratch,
                                                           uint32_t* __restrict__ pay, uint32_t* __restrict__ pay_scratch,
                                                           uint32_t* __restrict__ bstart,
                                                           const uint32_t* __restrict__ s_in,
                                                           uint32_t* __restrict__ s_next, uint32_t cap,
                                                           unsigned int* over_host, RowHist rh,
                                                           const uint4* __restrict__ rec,
                                                           const uint32_t* __restrict__ only = nullptr) {
    GSR_GEOM_PRIO();
    __shared__ uint64_t s_items[kBktTile];
    __shared__ uint32_t s_pay[kBktTile];
    __shared__ uint32_t s_wc[4][256], s_lbase[256], s_gb[256];
    __shared__ uint32_t s_hp[4][256];   // fused row-pass count: pairs (s_wc holds the items)
    __shared__ uint32_t s_scr[4], s_mm[2];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    auto row_zero = [&]() {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            s_wc[k][t] = 0;
            s_hp[k][t] = 0;
        }
    };
    if (blockIdx.x == (uint32_t)B - 1u) {
        // fused row count only (grid B): the last bucket (key 0xFFFFFFFF, index order, never
        // sorted) is the row pass's last chunk.  It holds culled items only unless the scatter
        // raised bstart[B + 1]; then its rects are counted (every live one binned, as the LSD
        // path and render.cu do), else the chunk is emptied (bstart[B] = its start: the
        // row pass reads nothing there).  Only this workgroup reads bstart[B].
        const uint32_t start = bstart[B - 1], end = bstart[B];
        const bool sat = bstart[B + 1] != 0u;
        row_zero();
        __syncthreads();
        if (sat) {
            for (uint32_t i = start + t; i < end; i += 4u * kBktThreads) {
                uint32_t p[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t j = i + (uint32_t)k * kBktThreads;
                    p[k] = j < end ? pay[j] : pack_rect(kDeadRect);
                }
#pragma unroll
                for (int k = 0; k < 4; k++) row_hist_add(s_wc, s_hp, w, p[k]);
            }
        }
        row_hist_write(rh, (uint32_t)B - 1u, s_wc, s_hp, s_scr);
        if (!sat && t == 0) bstart[B] = start;
        return;
    }
    // XCD-contiguous buckets: the fused row count's histogram lines (16 consecutive
    // buckets of a row) merge in one L2 (12.4 -> 11.95 us at config 2,
    // profiles/r05_kt_xcd_hist.txt)
    const uint32_t bkt = (uint32_t)xcd_chunk((int)blockIdx.x, B - 1);
    if (only && only[bkt] == 0u) return;   // big buckets: only those k_bbk_local left to this kernel
    const uint32_t start = bstart[bkt], count = bstart[bkt + 1] - start, live = bstart[B - 1];
    // keys of bucket b lie in [s_in[b - 1], s_in[b]) for 0 < b < B - 2
    const bool bounded = bkt > 0 && bkt < (uint32_t)B - 2u;
    const uint32_t klo = bounded ? s_in[bkt - 1] : 0u, khi = bounded ? s_in[bkt] : 0u;
    if (bkt == 0 && t == 0) {
        s_next[B - 2] = 0xffffffffu;
        if (live == 0)   // no live quantiles (a camera looking away): keep this frame's splitters
            for (uint32_t j = 0; j < (uint32_t)B - 2u; j++) s_next[j] = s_in[j];
    }
    if (count == 0) {   // uniform; an empty bucket is an empty row-pass chunk
        if (rh.hist) {
            row_zero();
            row_hist_write(rh, bkt, s_wc, s_hp, s_scr);
        }
        return;
    }
    uint64_t* const seg = items + start;
    uint32_t* const pseg = pay + start;
    auto rseg = [&](uint32_t q) { return rec_get<R12>(rec, start + q); };   // the bucket's records, index order
    // ---- fast path: the bucket in registers, stable 8-bit passes through LDS.  IT items per
    // thread: 4 for buckets of up to 1,024 (the usual ~n / B: every wave holds a quarter of
    // the bucket), 8 up to the capacity (at 8, buckets under 1,024 left waves 2 and 3 idle
    // and waves 0 and 1 with twice the slots) ----
    auto fast = [&](auto it_c) {
        constexpr int IT = decltype(it_c)::value;
        const uint32_t wbase = w * 64 * IT;
        uint64_t it[IT];
        uint32_t pv[IT];
#pragma unroll
        for (int k = 0; k < IT; k++) {
            const uint32_t el = wbase + k * 64 + lane;
            const uint4 r = el < count ? rseg(el) : make_uint4(~0u, ~0u, 0u, 0u);
            it[k] = ((uint64_t)r.y << 32) | r.x;
            pv[k] = r.z;
        }
        uint32_t kmin = klo, span = khi - klo - 1u;   // bounded: keys in [klo, khi)
        if (!bounded) {   // the open-ended first and last buckets: their own min and max
            uint32_t mn = 0xffffffffu, mx = 0;
#pragma unroll
            for (int k = 0; k < IT; k++)
                if (wbase + k * 64 + lane < count) {
                    mn = min(mn, (uint32_t)(it[k] >> 32));
                    mx = max(mx, (uint32_t)(it[k] >> 32));
                }
            mn = ~wave_max_u32(~mn);
            mx = wave_max_u32(mx);
            if (t < 2) s_mm[t] = t ? 0u : 0xffffffffu;
            __syncthreads();
            if (lane == 0) {
                atomicMin(&s_mm[0], mn);
                atomicMax(&s_mm[1], mx);
            }
            __syncthreads();
            kmin = s_mm[0];
            span = s_mm[1] - kmin;
        }
        const int bits = span ? 32 - __clz((int)span) : 0;
        for (int shift = 0; shift < bits; shift += 8) {   // uniform
            uint32_t dig[IT], pos[IT];
#pragma unroll
            for (int k = 0; k < IT; k++) dig[k] = (((uint32_t)(it[k] >> 32) - kmin) >> shift) & 0xffu;
            (void)bin_rank_tile<IT, 8, RA>(dig, count, pos, s_wc, s_lbase, s_scr);
#pragma unroll
            for (int k = 0; k < IT; k++) {
                const uint32_t el = wbase + k * 64 + lane;
                if (el < count) {
                    s_items[pos[k]] = it[k];
                    s_pay[pos[k]] = pv[k];
                }
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < IT; k++) {
                const uint32_t el = wbase + k * 64 + lane;
                if (el < count) {
                    it[k] = s_items[el];
                    pv[k] = s_pay[el];
                }
            }
            __syncthreads();
        }
#pragma unroll
        for (int k = 0; k < IT; k++) {
            const uint32_t el = wbase + k * 64 + lane;
            if (el < count) {
                seg[el] = it[k];
                pseg[el] = pv[k];
                s_items[el] = it[k];
            }
        }
        if (rh.hist) {   // the bucket is the row pass's chunk: its row histograms from the rects
            row_zero();
            __syncthreads();
#pragma unroll
            for (int k = 0; k < IT; k++)
                if (wbase + k * 64 + lane < count) row_hist_add(s_wc, s_hp, w, pv[k]);
            row_hist_write(rh, bkt, s_wc, s_hp, s_scr);
        }
        __syncthreads();
        if (bkt < (uint32_t)B - 1u)
            bkt_write_splitters<B>(start, count, live, s_next,
                                   [&](uint32_t q) { return (uint32_t)(s_items[q] >> 32); });
    };
    // (5 and 6 items per thread for the 1,025-1,536-item buckets of scenes above 4M items:
    // at 8 the items of a 1,220-item bucket sat on waves 0-1 and 2-3 idled)
    if (count <= min(cap, (uint32_t)kBktThreads * 4u)) {
        fast(std::integral_constant<int, 4>{});
        return;
    }
    if (count <= min(cap, (uint32_t)kBktThreads * 5u)) {
        fast(std::integral_constant<int, 5>{});
        return;
    }
    if (count <= min(cap, (uint32_t)kBktThreads * 6u)) {
        fast(std::integral_constant<int, 6>{});
        return;
    }
    if (count <= cap) {
        fast(std::integral_constant<int, 8>{});
        return;
    }
    const uint32_t wbase = w * 64 * kBktItems;
    // ---- over capacity: stable 8-bit passes through global memory, one tile at a time ----
    if (over_host && t == 0) atomicAdd_system(over_host, count);
    for (uint32_t i = t; i < count; i += kBktThreads) {   // the records into the item / rect arrays
        const uint4 r = rseg(i);
        seg[i] = ((uint64_t)r.y << 32) | r.x;
        pseg[i] = r.z;
    }
    __threadfence();
    __syncthreads();
    uint32_t kmin = 0xffffffffu, kmax = 0;
    for (uint32_t i = t; i < count; i += kBktThreads) {
        const uint32_t k = (uint32_t)(seg[i] >> 32);
        kmin = min(kmin, k);
        kmax = max(kmax, k);
    }
    kmin = ~wave_max_u32(~kmin);
    kmax = wave_max_u32(kmax);
    if (t < 2) s_mm[t] = t ? 0u : 0xffffffffu;
    __syncthreads();
    if (lane == 0) {
        atomicMin(&s_mm[0], kmin);
        atomicMax(&s_mm[1], kmax);
    }
    __syncthreads();
    kmin = s_mm[0];
    const uint32_t span = s_mm[1] - kmin;
    const int bits = span ? 32 - __clz((int)span) : 0;
    if (over_host && t == 0 && bits) atomicAdd_system(over_host + 1, count * (uint32_t)((bits + 7) / 8));
    uint64_t* src = seg;
    uint64_t* dst = scratch + start;
    uint32_t* psrc = pseg;
    uint32_t* pdst = pay_scratch + start;
    int passes = 0;
    for (int shift = 0; shift < bits; shift += 8, ++passes) {
        auto digit = [&](uint64_t v) { return (((uint32_t)(v >> 32) - kmin) >> shift) & 0xffu; };
        s_gb[t] = 0;
        __syncthreads();
        for (uint32_t i = t; i < count; i += kBktThreads) atomicAdd(&s_gb[digit(src[i])], 1u);
        __syncthreads();
        {
            const uint32_t c = s_gb[t];
            uint32_t tot;
            const uint32_t ex = block_exclusive_scan<uint32_t>(c, s_scr, tot);
            s_gb[t] = ex;   // every read of s_gb[t] (its own count) is done by this thread
        }
        for (uint32_t tb = 0; tb < count; tb += kBktTile) {
            const uint32_t tn = min(kBktTile, count - tb);
            uint64_t it[kBktItems];
            uint32_t pv[kBktItems], dig[kBktItems], pos[kBktItems];
#pragma unroll
            for (int k = 0; k < kBktItems; k++) {
                const uint32_t el = wbase + k * 64 + lane;
                it[k] = el < tn ? src[tb + el] : ~0ull;
                pv[k] = el < tn ? psrc[tb + el] : 0u;
                dig[k] = digit(it[k]);
            }
            const uint32_t tcount = bin_rank_tile<kBktItems, 8, RA>(dig, tn, pos, s_wc, s_lbase, s_scr);
#pragma unroll
            for (int k = 0; k < kBktItems; k++) {
                const uint32_t el = wbase + k * 64 + lane;
                if (el < tn) {
                    s_items[pos[k]] = it[k];
                    s_pay[pos[k]] = pv[k];
                }
            }
            __syncthreads();
            for (uint32_t q = t; q < tn; q += kBktThreads) {
                const uint64_t v = s_items[q];
                const uint32_t d = digit(v);
                const uint32_t o = s_gb[d] + (q - s_lbase[d]);
                dst[o] = v;
                pdst[o] = s_pay[q];
            }
            __syncthreads();
            s_gb[t] += tcount;
            // bin_rank_tile's first barrier orders this before the next tile's reads
        }
        __threadfence();   // the next pass (other waves of this workgroup) reads what this one wrote
        __syncthreads();
        uint64_t* ts = src;
        src = dst;
        dst = ts;
        uint32_t* tp = psrc;
        psrc = pdst;
        pdst = tp;
    }
    if (passes & 1) {   // the result is in the scratch segment: copy it back
        for (uint32_t i = t; i < count; i += kBktThreads) {
            seg[i] = src[i];
            pseg[i] = psrc[i];
        }
        __threadfence();
        __syncthreads();
    }
    if (rh.hist) {
        row_zero();
        __syncthreads();
        for (uint32_t i = t; i < count; i += kBktThreads) row_hist_add(s_wc, s_hp, w, pseg[i]);
        row_hist_write(rh, bkt, s_wc, s_hp, s_scr);
    }
    if (bkt < (uint32_t)B - 1u)
        bkt_write_splitters<B>(start, count, live, s_next, [&](uint32_t q) { return (uint32_t)(seg[q] >> 32); });
}

// ---- big buckets (scenes above 2M Gaussians: 512 buckets of ~n / 512 items) ----
//
// One 1,024-thread workgroup sorts a bucket of up to 16,384 items in LDS: up to 16 per thread
// (blocked per wave, so a wave's items are consecutive positions; the 16 waves share the
// bucket evenly, ceil(count / 1,024) rows of 64 each, so all of them work), stable 8-bit LSD passes
// over key - lo whose exchange carries one u32 per item, slot (original position, 14 bits) |
// (key - lo) << 14, so keys may span 18 bits above lo (config 3's buckets: 12-13).  After
// the last pass each position knows its slot and key; the index (kept in LDS by slot) and
// the rect (pulled through the exchange buffer by slot) join them and the bucket is written
// out coalesced.  Buckets over the capacity or wider than 18 bits are flagged in `left` and
// sorted by k_bkt_local's paths in a second launch.
constexpr int kBbThreads = 1024;
constexpr int kBbItems = 16;                            // capacity TH * 16: 16,384 at 1,024 threads

// TH threads (1,024: capacity 16,384, one workgroup per CU; 512: 8,192 at half the LDS)
template <int B, bool RA, bool R12, int TH = kBbThreads>
__global__ __launch_bounds__(TH) void k_bbk_local(uint64_t* __restrict__ items, uint32_t* __restrict__ pay,
                                                  const uint32_t* __restrict__ bstart,
                                                  const uint32_t* __restrict__ s_in,
                                                  uint32_t* __restrict__ s_next, uint32_t cap,
                                                  const uint4* __restrict__ rec, uint32_t* __restrict__ left) {
    GSR_GEOM_PRIO();
    constexpr int NW = TH / 64;
    constexpr uint32_t kCap = (uint32_t)TH * kBbItems;
    constexpr int kBbSlot = __builtin_ctz(kCap);        // slot bits of the exchange word
    constexpr int kBbKeyBits = 32 - kBbSlot;            // key bits above lo it carries
    __shared__ uint32_t s_buf[kCap];                    // the exchange, then the rect pull, then the keys
    __shared__ uint32_t s_idx[kCap];                    // the indices by slot
    __shared__ uint32_t s_wc[NW][256];                  // per-wave digit counts, then their wave prefixes
    __shared__ uint32_t s_db[256];                      // the digits' first positions
    __shared__ uint32_t s_scr[NW], s_mm[2];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint32_t bkt = blockIdx.x;
    const uint32_t start = bstart[bkt], count = bstart[bkt + 1] - start, live = bstart[B - 1];
    const bool bounded = bkt > 0 && bkt < (uint32_t)B - 2u;
    const uint32_t klo = bounded ? s_in[bkt - 1] : 0u, khi = bounded ? s_in[bkt] : 0u;
    if (bkt == 0 && t == 0) {
        s_next[B - 2] = 0xffffffffu;
        if (live == 0)   // no live quantiles (a camera looking away): keep this frame's splitters
            for (uint32_t j = 0; j < (uint32_t)B - 2u; j++) s_next[j] = s_in[j];
    }
    if (count == 0) {
        if (t == 0) left[bkt] = 0u;
        return;
    }
    if (count > min(cap, kCap)) {
        if (t == 0) left[bkt] = 1u;
        return;
    }
    // the waves split the bucket evenly (kk rows of 64 each) so every wave has work
    const uint32_t kk = (count + NW * 64u - 1u) / (NW * 64u), wbase = w * kk * 64u;
    uint32_t x[kBbItems], rct[kBbItems];
    {
        uint32_t key[kBbItems];
#pragma unroll
        for (int k = 0; k < kBbItems; k++) {
            const uint32_t el = wbase + k * 64 + lane;
            const bool in = k < (int)kk && el < count;
            const uint4 r = in ? rec_get<R12>(rec, start + el) : make_uint4(0u, 0xffffffffu, 0u, 0u);
            if (in) s_idx[el] = r.x;
            key[k] = r.y;
            rct[k] = r.z;
        }
        uint32_t kmin = klo, span = khi - klo - 1u;
        if (!bounded) {   // the open first and last buckets: their own min and max
            uint32_t mn = 0xffffffffu, mx = 0;
#pragma unroll
            for (int k = 0; k < kBbItems; k++)
                if (k < (int)kk && wbase + k * 64 + lane < count) {
                    mn = min(mn, key[k]);
                    mx = max(mx, key[k]);
                }
            mn = ~wave_max_u32(~mn);
            mx = wave_max_u32(mx);
            if (t < 2) s_mm[t] = t ? 0u : 0xffffffffu;
            __syncthreads();
            if (lane == 0) {
                atomicMin(&s_mm[0], mn);
                atomicMax(&s_mm[1], mx);
            }
            __syncthreads();
            kmin = s_mm[0];
            span = s_mm[1] - kmin;
        }
        if (span >> kBbKeyBits) {   // uniform: wider than the exchange word (k_bkt_local sorts it)
            if (t == 0) left[bkt] = 1u;
            return;
        }
        // the exchange word of every position (before the first pass: position = slot)
#pragma unroll
        for (int k = 0; k < kBbItems; k++) x[k] = (wbase + k * 64 + lane) | ((key[k] - kmin) << kBbSlot);
        __syncthreads();   // every thread has read s_mm before it is rewritten
        if (t == 0) {
            left[bkt] = 0u;
            s_mm[0] = kmin;
            s_mm[1] = span;
        }
    }
    __syncthreads();
    const uint32_t kmin = s_mm[0], span = s_mm[1];
    const int bits = span ? 32 - __clz((int)span) : 0;   // the passes: the bits the keys span
    for (int shift = 0; shift < bits; shift += 8) {   // uniform
        auto digit = [&](int k) { return (x[k] >> (kBbSlot + shift)) & 0xffu; };
        for (uint32_t j = t; j < (uint32_t)NW * 256u; j += TH) (&s_wc[0][0])[j] = 0;
        __syncthreads();
        uint32_t rk[kBbItems];
#pragma unroll
        for (int k = 0; k < kBbItems; k++) {
            rk[k] = 0;
            if (k >= (int)kk) continue;   // uniform
            const uint32_t el = wbase + k * 64 + lane;
            const bool valid = el < count;
            const uint32_t dk = digit(k);
            if (RA) {
                rk[k] = atomicAdd(&s_wc[w][dk], valid ? 1u : 0u);
            } else {
                const uint64_t peers = match_peers<8>(dk, valid, 8);
                rk[k] = 0;
                if (valid) {
                    rk[k] = s_wc[w][dk] + (uint32_t)__popcll(peers & (lane ? (~0ull >> (64 - lane)) : 0ull));
                    if (lane == (uint32_t)(__ffsll((unsigned long long)peers) - 1))
                        atomicAdd(&s_wc[w][dk], (uint32_t)__popcll(peers));
                }
            }
        }
        __syncthreads();
        uint32_t dtot = 0;
        if (t < 256u) {
            uint32_t run = 0;
#pragma unroll
            for (int v = 0; v < NW; v++) {
                const uint32_t c = s_wc[v][t];
                s_wc[v][t] = run;
                run += c;
            }
            dtot = run;
        }
        {
            uint32_t tot;
            const uint32_t ex = block_exclusive_scan<uint32_t, NW>(dtot, s_scr, tot);
            if (t < 256u) s_db[t] = ex;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kBbItems; k++) {
            const uint32_t el = wbase + k * 64 + lane;
            if (k < (int)kk && el < count) {
                const uint32_t dk = digit(k);
                s_buf[s_db[dk] + s_wc[w][dk] + rk[k]] = x[k];
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kBbItems; k++) {
            const uint32_t el = wbase + k * 64 + lane;
            if (k < (int)kk && el < count) x[k] = s_buf[el];
        }
        __syncthreads();
    }
    // rect by slot through the buffer (owners write by slot, positions read), then write out
#pragma unroll
    for (int k = 0; k < kBbItems; k++)
        if (k < (int)kk && wbase + k * 64 + lane < count) s_buf[wbase + k * 64 + lane] = rct[k];
    __syncthreads();
    uint64_t* const seg = items + start;
    uint32_t* const pseg = pay + start;
#pragma unroll
    for (int k = 0; k < kBbItems; k++) {
        const uint32_t el = wbase + k * 64 + lane;
        if (k < (int)kk && el < count) {
            const uint32_t slot = x[k] & (kCap - 1u);
            rct[k] = s_buf[slot];
            seg[el] = ((uint64_t)(kmin + (x[k] >> kBbSlot)) << 32) | s_idx[slot];
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kBbItems; k++) {
        const uint32_t el = wbase + k * 64 + lane;
        if (k < (int)kk && el < count) {
            pseg[el] = rct[k];
            s_buf[el] = kmin + (x[k] >> kBbSlot);   // sorted keys, for the next frame's splitters
        }
    }
    __syncthreads();
    if (bkt < (uint32_t)B - 1u)
        bkt_write_splitters<B, TH>(start, count, live, s_next, [&](uint32_t q) { return s_buf[q]; });
}

// Splitters from a depth order the LSD passes sorted (a context's first frame, or the
// first after the bucket count changed): one workgroup.  live (nullable): the visible
// count of a partitioned sort; else the first key 0xFFFFFFFF is found by two rounds of
// 256 probes and a last scan.
template <int B>
__global__ __launch_bounds__(kBktThreads) void k_bkt_splitters(const uint64_t* __restrict__ items0,
                                                               const uint64_t* __restrict__ items1,
                                                               const uint32_t* __restrict__ dstats, uint32_t n,
                                                               const uint32_t* __restrict__ live_dev,
                                                               uint32_t* __restrict__ s_out) {
    GSR_GEOM_PRIO();
    __shared__ uint32_t s_lo, s_hi;
    const uint64_t* sorted = depth_sorted(items0, items1, dstats);
    const uint32_t t = threadIdx.x;
    uint32_t live;
    if (live_dev) {
        live = min(*live_dev, n);
    } else {
        // the first position whose key is 0xFFFFFFFF (n if none): narrow [lo, hi) by probes
        if (t == 0) {
            s_lo = 0;
            s_hi = n;
        }
        __syncthreads();
        for (int round = 0; round < 3; round++) {
            const uint32_t lo = s_lo, hi = s_hi;
            __syncthreads();
            const uint32_t len = hi - lo;
            if (len <= 1) break;   // uniform
            const uint32_t step = (len + kBktThreads - 1) / kBktThreads;
            const uint32_t p = lo + t * step;
            const bool dead = p < hi && (uint32_t)(sorted[p] >> 32) == 0xffffffffu;
            // the last probe that is live, then the first that is dead, bound the answer
            if (p < hi && !dead) atomicMax(&s_lo, p + 1);
            if (dead) atomicMin(&s_hi, p);
            __syncthreads();
        }
        uint32_t lo = s_lo;
        const uint32_t hi = s_hi;
        __syncthreads();
        // at most a few positions left: each thread checks one
        if (t == 0) s_lo = hi;
        __syncthreads();
        for (uint32_t p = lo + t; p < hi; p += kBktThreads)
            if ((uint32_t)(sorted[p] >> 32) == 0xffffffffu) atomicMin(&s_lo, p);
        __syncthreads();
        live = s_lo;
        (void)lo;
    }
    // thread t takes splitters t * kPer .. + kPer - 1 and makes them non-decreasing with a
    // running max (an order the host's pass budget left incomplete — that frame re-renders
    // — must still give sorted splitters: the bucket search assumes them)
    constexpr int kPer = B / kBktThreads;
    __shared__ uint32_t s_wmax[4];
    uint32_t v[kPer], run = 0;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const uint32_t j = t * kPer + k;
        v[k] = live && j < (uint32_t)B - 2u ? (uint32_t)(sorted[bkt_split_pos<B>(j, live)] >> 32) : 0u;
        v[k] = min(v[k], 0xfffffffeu);
        run = max(run, v[k]);
        v[k] = run;
    }
    // inclusive max over the wave's threads, then over earlier waves
    const uint32_t lane = t & 63u, w = t >> 6;
    const uint32_t x = wave_incl_scan(run, OpMax{});
    if (lane == 63) s_wmax[w] = x;
    uint32_t before = wave_shr1(x);
    __syncthreads();
    for (uint32_t k = 0; k < w; k++) before = max(before, s_wmax[k]);
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const uint32_t j = t * kPer + k;
        if (j < (uint32_t)B - 2u) s_out[j] = max(before, v[k]);
    }
    if (t == 0) s_out[B - 2] = 0xffffffffu;
}

// Depth split, phase B: the summed-area table of the tiles phase A left unsaturated
// (a tile counts when any of its four blocks' flags is set; the flags of a tile are
// consecutive bytes), (tiles_y + 1) x (tiles_x + 1) words with a zero first row and
// column.  One workgroup: row prefix sums, then column prefix sums.
__global__ __launch_bounds__(256) void k_split_sat(const uint8_t* __restrict__ bflag, int tiles_x, int tiles_y,
                                                    uint32_t* __restrict__ sat, const uint32_t* __restrict__ gate) {
    GSR_GEOM_PRIO();
    if (*gate == 0u) return;
    const int w = tiles_x + 1;
    const uint32_t* tf = reinterpret_cast<const uint32_t*>(bflag);
    for (int y = (int)threadIdx.x; y <= tiles_y; y += 256) {
        uint32_t* row = sat + (size_t)y * (uint32_t)w;
        uint32_t run = 0;
        row[0] = 0;
        for (int x = 0; x < tiles_x; x++) {
            if (y > 0) run += tf[(size_t)(y - 1) * (uint32_t)tiles_x + (uint32_t)x] != 0u ? 1u : 0u;
            row[x + 1] = run;
        }
    }
    __syncthreads();
    for (int x = (int)threadIdx.x + 1; x <= tiles_x; x += 256) {
        uint32_t run = 0;
        for (int y = 1; y <= tiles_y; y++) {
            run += sat[(size_t)y * (uint32_t)w + (uint32_t)x];
            sat[(size_t)y * (uint32_t)w + (uint32_t)x] = run;
        }
    }
}

// Row pass, count: per workgroup (1024-Gaussian sub-chunks in depth order) the
// number of row items and of pairs per tile row; hist[row][g] and
// hist[256 + row][g].  Reads the rects in depth order (the payloads the depth
// sort carried, depth_sorted_rects).
__global__ __launch_bounds__(256) void k_bin_rows_count(uint32_t n, const uint32_t* __restrict__ pay0,
                                                         const uint32_t* __restrict__ pay1,
                                                         const uint32_t* __restrict__ dstats, int groups,
                                                         int tiles_y, uint32_t* __restrict__ hist, uint32_t base,
                                                         const uint32_t* __restrict__ gate,
                                                         const uint32_t* __restrict__ cut, int cut_mode,
                                                         const uint32_t* __restrict__ cut_n) {
    GSR_GEOM_PRIO();
    if (gate && *gate == 0u) return;   // depth split, phase B: every block saturated in phase A
    row_range(base, n, cut, cut_mode, cut_n);
    __shared__ uint32_t h_items[4][256], h_pairs[4][256];
    const uint32_t t = threadIdx.x, w = t >> 6;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        h_items[k][t] = 0;
        h_pairs[k][t] = 0;
    }
    __syncthreads();
    const uint32_t* srect = depth_sorted_rects(pay0, pay1, dstats) + base;
    const int chunk = (int)blockIdx.x;   // (XCD-contiguous chunks: 16.2 -> 18.7 us at config 3)
    uint64_t b, e;
    chunk_range(n, groups, chunk, kRowSources, b, e);
    for (uint64_t c0 = b; c0 < e; c0 += 1024) {
        uint64_t r[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t j = c0 + t + 256 * k;
            r[k] = j < e ? unpack_rect(srect[j]) : kDeadRect;
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            // difference arrays: +1 / +cols at the first row, -1 / -cols past the last
            if (rect_count(r[k])) {
                const uint32_t ty0 = (uint32_t)((r[k] >> 32) & 0xffffu), ty1 = (uint32_t)(r[k] >> 48);
                const uint32_t cols = rect_cols(r[k]);
                atomicAdd(&h_items[w][ty0], 1u);
                atomicAdd(&h_pairs[w][ty0], cols);
                if (ty1 < 255u) {
                    atomicSub(&h_items[w][ty1 + 1], 1u);
                    atomicSub(&h_pairs[w][ty1 + 1], cols);
                }
            }
        }
    }
    __syncthreads();
    // prefix over rows turns the differences into per-row counts (mod 2^32)
    uint32_t ti, tp;
    const uint32_t di = h_items[0][t] + h_items[1][t] + h_items[2][t] + h_items[3][t];
    const uint32_t dp = h_pairs[0][t] + h_pairs[1][t] + h_pairs[2][t] + h_pairs[3][t];
    __shared__ uint32_t scr[4];
    const uint32_t ci = block_exclusive_scan<uint32_t>(di, scr, ti) + di;
    const uint32_t cp = block_exclusive_scan<uint32_t>(dp, scr, tp) + dp;
    if (t < (uint32_t)tiles_y) {   // rows past the grid hold nothing: no scattered writes for them
        hist[t * (uint32_t)groups + chunk] = ci;
        hist[(256 + t) * (uint32_t)groups + chunk] = cp;
    }
}



// Depth split: the next frame's threshold from this frame's near depth order: the key
// at position na (the host's split point) when the near part holds more than na items,
// else the threshold widened in proportion from the smallest key.  Any threshold gives
// the same image.
__device__ __forceinline__ void split_cut_update(const SplitCut& sc) {
    const uint64_t* sorted = depth_sorted(sc.items0, sc.items1, sc.dstats);
    const uint32_t m = sc.nnear ? min(*sc.nnear, sc.n) : sc.n;
    uint32_t K;
    if (sc.na < m) {
        K = (uint32_t)(sorted[sc.na] >> 32);
    } else {
        const uint32_t k0 = *sc.kcut, kmin = m ? (uint32_t)(sorted[0] >> 32) : 0u;
        if (m == 0 || k0 == 0xffffffffu || k0 <= kmin) {
            K = 0xffffffffu;
        } else {
            const uint64_t span = (uint64_t)(k0 - kmin) * sc.na / m + 1u;
            K = (uint32_t)min((uint64_t)kmin + span, (uint64_t)0xffffffffu);
        }
    }
    *sc.kcut = K;
}

// Row pass, scan: one workgroup per row.  Exclusive scan of the row's item
// counts over the workgroups (in place) and the row's totals.
__global__ __launch_bounds__(256) void k_bin_rows_scan(uint32_t* __restrict__ hist, int groups, int tiles_y,
                                                        uint32_t* __restrict__ row_items,
                                                        unsigned long long* __restrict__ row_pairs,
                                                        uint32_t* __restrict__ gate, int gate_mode) {
    GSR_GEOM_PRIO();
    // depth split: phase A clears the count of unsaturated blocks its blend raises;
    // phase B runs only when that count is not zero
    if (gate_mode == 1 && blockIdx.x == 0 && threadIdx.x == 0) *gate = 0u;
    if (gate_mode == 2 && *gate == 0u) return;
    __shared__ uint32_t scr[4];
    __shared__ unsigned long long scr64[4];
    const uint32_t r = blockIdx.x, t = threadIdx.x;
    if (r >= (uint32_t)tiles_y) {   // all 256 row totals are read downstream
        if (t == 0) {
            row_items[r] = 0;
            row_pairs[r] = 0;
        }
        return;
    }
    uint32_t* hi = hist + (size_t)r * (uint32_t)groups;
    const uint32_t* hp = hist + (size_t)(256 + r) * (uint32_t)groups;
    const int per = (groups + 255) / 256;
    const int b = (int)t * per;
    // all loads of the segment issued together (k_radix_scan)
    constexpr int kPerMax = kMaxSortGroups / 256;
    uint32_t v[kPerMax], local = 0;
    unsigned long long lp = 0;
#pragma unroll
    for (int k = 0; k < kPerMax; k++) {
        const bool in = k < per && b + k < groups;
        v[k] = in ? hi[b + k] : 0u;
        lp += in ? hp[b + k] : 0u;
        local += v[k];
    }
    uint32_t tot;
    uint32_t run = block_exclusive_scan<uint32_t>(local, scr, tot);
    unsigned long long ptot;
    block_exclusive_scan<unsigned long long>(lp, scr64, ptot);
#pragma unroll
    for (int k = 0; k < kPerMax; k++)
        if (k < per && b + k < groups) {
            hi[b + k] = run;
            run += v[k];
        }
    if (t == 0) {
        row_items[r] = tot;
        row_pairs[r] = ptot;
    }
}

// Row pass, scatter: the workgroup's Gaussians, 1024 at a time, expand into
// their row items; tiles of 256*ITEMS items are ranked by row and written in
// row runs to rows_out (positions >= cap are dropped; the frame then overflows
// and the column pass emits nothing).  The sorted tile holds only each item's
// source slot: the payload (index | tx0 << 32 | tx1 << 48) is rebuilt at the write.
template <int ITEMS, int BITS, bool RA>
__global__ __launch_bounds__(256, ITEMS == 4 ? 6 : 1) void k_bin_rows_scatter(const uint64_t* __restrict__ items0,
                                                           const uint64_t* __restrict__ items1,
                                                           const uint32_t* __restrict__ dstats,
                                                           const uint32_t* __restrict__ pay0,
                                                           const uint32_t* __restrict__ pay1, uint32_t n,
                                                           int groups, const uint32_t* __restrict__ hist,
                                                           const uint32_t* __restrict__ row_items,
                                                           const unsigned long long* __restrict__ row_pairs,
                                                           uint32_t cap, int tiles_y, uint64_t* __restrict__ rows_out,
                                                           const uint16_t* __restrict__ spans, uint32_t base,
                                                           const uint32_t* __restrict__ gate,
                                                           const uint32_t* __restrict__ cut, int cut_mode,
                                                           const uint32_t* __restrict__ cut_n,
                                                           const uint32_t* __restrict__ cstart) {
    GSR_GEOM_PRIO();
    if (gate && *gate == 0u) return;
    row_range(base, n, cut, cut_mode, cut_n);
    constexpr uint32_t kTile = 256u * ITEMS;
    // per source: exclusive start << 8 | first tile row; index
    __shared__ uint32_t s_ft[kRowSources], s_idx[kRowSources];
    // per source: packed rect (pack_rect) | tile row spans << 32 (no LDS beyond the
    // 8 B per source it always had: 6 workgroups per CU)
    __shared__ uint64_t s_rect[kRowSources];
    // s_own (source owners, read by the generation) and s_dl (the ranked tile: source
    // slot << 8 | row, written after the ranking) share storage: their lives do not overlap
    __shared__ uint32_t s_dl[kTile];
    uint16_t* const s_own = reinterpret_cast<uint16_t*>(s_dl);
    __shared__ uint32_t s_wmax[4];
    // s_dbase[d]: global position of the tile's first item of row d minus its tile slot
    __shared__ uint32_t s_wc[4][256], s_dbase[256], s_lbase[256], s_scr[4];
    __shared__ unsigned long long s_scr64[4];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    uint64_t b, e;
    const int chunk = (int)blockIdx.x;
    if (cstart) {   // the chunks are the bucket sort's buckets (k_bkt_local counted them)
        b = min(cstart[chunk], n);
        e = min(cstart[chunk + 1], n);
    } else {
        chunk_range(n, groups, chunk, kRowSources, b, e);
    }
    const uint64_t* sorted = depth_sorted(items0, items1, dstats) + base;
    const uint32_t* srect = depth_sorted_rects(pay0, pay1, dstats) + base;
    // thread t owns sources 4t .. 4t+3 of a sub-chunk (source order): packed rect, index
    // and (by index) tile row spans; the first sub-chunk's (usually the only one) are
    // loaded before the base scan, so the dependent spans gather overlaps it (loading
    // every next sub-chunk ahead too holds 86 VGPRs: one wave per SIMD fewer)
    uint32_t prc[4], gix[4], spv[4];
    auto load_sources = [&](uint64_t c0) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint64_t j = c0 + 4 * t + i;
            prc[i] = j < e ? srect[j] : pack_rect(kDeadRect);
            gix[i] = j < e ? (uint32_t)sorted[j] : 0u;
        }
#pragma unroll
        for (int i = 0; i < 4; i++) spv[i] = spans && rect_rows(unpack_rect(prc[i])) ? spans[gix[i]] : 0u;
    };
    load_sources(b);
    uint32_t gb;   // row t's running global position (thread t owns row t)
    {
        uint32_t tot;
        gb = block_exclusive_scan<uint32_t>(row_items[t], s_scr, tot) +
             (t < (uint32_t)tiles_y ? hist[t * (uint32_t)groups + chunk] : 0u);
        unsigned long long ptot;
        block_exclusive_scan<unsigned long long>(row_pairs[t], s_scr64, ptot);
        if (ptot > cap || b >= e) return;   // uniform: overflow frames stop here
    }
    for (uint64_t c0 = b; c0 < e; c0 += kRowSources) {
        if (c0 != b) load_sources(c0);
        uint32_t cnt[4], start[4], ty0v[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            s_idx[4 * t + i] = gix[i];
            cnt[i] = rect_rows(unpack_rect(prc[i]));
            ty0v[i] = (prc[i] >> 16) & 0xffu;
        }
#pragma unroll
        for (int i = 0; i < ITEMS; i++) s_own[t * ITEMS + i] = 0;
        const uint32_t total = bin_source_starts<4>(cnt, start, ty0v, s_ft, s_scr);
#pragma unroll
        for (int i = 0; i < 4; i++)   // read after bin_tile_owners' barriers
            s_rect[4 * t + i] = (uint64_t)prc[i] | ((uint64_t)spv[i] << 32);
        uint32_t carry = 0;
        for (uint32_t tb = 0; tb < total; tb += kTile) {
            const uint32_t tn = min(kTile, total - tb);
            bin_tile_owners<ITEMS, 4>(cnt, start, tb, tn, s_own, carry, s_wmax);
            uint32_t dig[ITEMS], pos[ITEMS], src[ITEMS];
#pragma unroll
            for (int k = 0; k < ITEMS; k++) {
                const uint32_t el = min(w * 64 * ITEMS + k * 64 + lane, tn - 1);
                const uint32_t l = (uint32_t)s_own[el] - 1u;
                src[k] = l;
                const uint32_t ft = s_ft[l];
                dig[k] = (ft & 0xffu) + (tb + el - (ft >> 8));   // ty0 + row
            }
            const uint32_t tcount = bin_rank_tile<ITEMS, BITS, RA>(dig, tn, pos, s_wc, s_lbase, s_scr);
            s_dbase[t] = gb - s_lbase[t];   // this thread's own scan output
#pragma unroll
            for (int k = 0; k < ITEMS; k++) {
                const uint32_t el = w * 64 * ITEMS + k * 64 + lane;
                if (el < tn) s_dl[pos[k]] = (src[k] << 8) | dig[k];
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < ITEMS; k++) {
                const uint32_t q = t + 256 * k;
                const uint32_t qc = min(q, tn - 1);
                const uint32_t x = s_dl[qc];
                const uint32_t d = x & 0xffu, l = x >> 8;
                const uint32_t dst = s_dbase[d] + qc;
                const uint64_t r = s_rect[l];
                uint32_t x0 = (uint32_t)(r & 0xffu), x1 = (uint32_t)((r >> 8) & 0xffu);
                const uint32_t ro = d - (uint32_t)((r >> 16) & 0xffu);   // row within the rect
                if (ro < 4u) {
                    // tile row spans: columns [x0 + left, x1 - right]; an empty row gets the
                    // empty range (1, 0), which the column pass counts and expands to nothing
                    const uint32_t sp = (uint32_t)(r >> (32u + 4u * ro)) & 15u;
                    const int c0 = (int)(x0 + (sp & 3u)), c1 = (int)x1 - (int)(sp >> 2);
                    x0 = c0 <= c1 ? (uint32_t)c0 : 1u;
                    x1 = c0 <= c1 ? (uint32_t)c1 : 0u;
                }
                if (q < tn && dst < cap) rows_out[dst] = (uint64_t)s_idx[l] | ((uint64_t)x0 << 32) | ((uint64_t)x1 << 48);
            }
            __syncthreads();
            gb += tcount;
#pragma unroll
            for (int i = 0; i < ITEMS; i++) s_own[t * ITEMS + i] = 0;   // owners of the next tile start cleared
            __syncthreads();
        }
    }
}

// Row geometry of the column pass, rebuilt by each workgroup from the row
// totals: item base and count per row, first chunk per row (chunks of
// CH items never cross a row), chunk total, pair base per row, P.
// (PB: also the pair base per row — only the column scan needs it.)
template <bool PB>
struct ColPlan {
    uint32_t rbase[256], rcnt[256], chbase[257];
    unsigned long long pbase[PB ? 256 : 1];
};

template <uint32_t CH, bool PB>
__device__ __forceinline__ unsigned long long col_plan(const uint32_t* __restrict__ row_items,
                                                       const unsigned long long* __restrict__ row_pairs,
                                                       ColPlan<PB>& pl, uint32_t* s_scr,
                                                       unsigned long long* s_scr64) {
    const uint32_t t = threadIdx.x;
    const uint32_t cnt = row_items[t];
    uint32_t tot;
    pl.rbase[t] = block_exclusive_scan<uint32_t>(cnt, s_scr, tot);
    pl.rcnt[t] = cnt;
    pl.chbase[t] = block_exclusive_scan<uint32_t>((cnt + CH - 1) / CH, s_scr, tot);
    if (t == 255) pl.chbase[256] = tot;
    unsigned long long ptot;
    const unsigned long long pb = block_exclusive_scan<unsigned long long>(row_pairs[t], s_scr64, ptot);
    if (PB) pl.pbase[t] = pb;
    __syncthreads();
    return ptot;
}

// Row of chunk c: the last row whose first chunk is <= c (empty rows own none).
template <bool PB>
__device__ __forceinline__ uint32_t col_chunk_row(const ColPlan<PB>& pl, uint32_t c) {
    uint32_t l = 0;
#pragma unroll
    for (uint32_t st = 128; st >= 1; st >>= 1)
        if (pl.chbase[l + st] <= c) l += st;
    return l;
}

// Column pass, count: per chunk, pairs per tile column -> cbins[chunk][col].
template <uint32_t CH>
__global__ __launch_bounds__(256) void k_bin_cols_count(const uint64_t* __restrict__ rows_in,
                                                         const uint32_t* __restrict__ row_items,
                                                         const unsigned long long* __restrict__ row_pairs,
                                                         uint32_t cap, int tiles_x, uint32_t* __restrict__ cbins,
                                                         const uint32_t* __restrict__ gate) {
    GSR_GEOM_PRIO();
    if (gate && *gate == 0u) return;
    __shared__ ColPlan<false> pl;
    __shared__ uint32_t h[4][256], s_scr[4];
    __shared__ unsigned long long s_scr64[4];
    const uint32_t t = threadIdx.x, w = t >> 6;
    if (col_plan<CH>(row_items, row_pairs, pl, s_scr, s_scr64) > cap) return;
    const uint32_t nch = pl.chbase[256];
    for (uint32_t c = blockIdx.x; c < nch; c += gridDim.x) {
#pragma unroll
        for (int k = 0; k < 4; k++) h[k][t] = 0;
        __syncthreads();
        const uint32_t r = col_chunk_row(pl, c);
        const uint32_t ib = pl.rbase[r] + (c - pl.chbase[r]) * CH;
        const uint32_t ie = min(ib + CH, pl.rbase[r] + pl.rcnt[r]);
        // difference arrays: +1 at the first column, -1 past the last (all of a thread's
        // loads issued before its first LDS update)
        constexpr int PER = CH / 256;
        uint64_t its[PER];
#pragma unroll
        for (int k = 0; k < PER; k++) its[k] = ib + t + 256 * k < ie ? rows_in[ib + t + 256 * k] : 0ull;
#pragma unroll
        for (int k = 0; k < PER; k++)
            if (ib + t + 256 * k < ie) {
                const uint32_t tx0 = (uint32_t)((its[k] >> 32) & 0xffffu), tx1 = (uint32_t)(its[k] >> 48);
                atomicAdd(&h[w][tx0], 1u);
                if (tx1 < 255u) atomicSub(&h[w][tx1 + 1], 1u);
            }
        __syncthreads();
        const uint32_t dsum = h[0][t] + h[1][t] + h[2][t] + h[3][t];
        uint32_t tot;
        const uint32_t cnt = block_exclusive_scan<uint32_t>(dsum, s_scr, tot) + dsum;   // mod 2^32
        if (t < (uint32_t)tiles_x) cbins[(size_t)c * 256 + t] = cnt;
    }
}

// Column pass, scan: one workgroup per row.  Exclusive scan of each column's
// chunk counts over the row's chunks (in place), then the row's tiles: start =
// row pair base + exclusive scan over columns; ranges = {~start, end} (zero =
// empty).  Overflowed frames (P > cap) get empty ranges.  Workgroup 0 publishes
// the frame's pair statistics.
template <uint32_t CH>
__global__ __launch_bounds__(256) void k_bin_cols_scan(const uint32_t* __restrict__ row_items,
                                                        const unsigned long long* __restrict__ row_pairs,
                                                        uint32_t cap, int tiles_x, uint32_t* __restrict__ cbins,
                                                        uint2* __restrict__ ranges, Stats* __restrict__ st,
                                                        Stats* host_st, const uint32_t* __restrict__ dstats,
                                                        int passes_launched, const uint32_t* __restrict__ gate,
                                                        uint32_t* fstatus) {
    GSR_GEOM_PRIO();
    if (gate && *gate == 0u) return;
    __shared__ ColPlan<true> pl;
    __shared__ uint32_t s_scr[4];
    __shared__ unsigned long long s_scr64[4];
    const uint32_t t = threadIdx.x, r = blockIdx.x;
    const unsigned long long P = col_plan<CH>(row_items, row_pairs, pl, s_scr, s_scr64);
    if (r == 0 && t == 0)
        publish_pair_stats(P, cap, st, host_st, dstats ? (uint32_t)depth_passes_run(dstats) : 0u,
                           (uint32_t)passes_launched, fstatus, gate == nullptr);
    uint32_t run = 0;
    if (P <= cap && t < (uint32_t)tiles_x) {
        // 32 chunks per step: the loads are issued together, not one round trip per chunk
        // (a row of the 5M-Gaussian frame has ~75 chunks: 3 round trips instead of 10)
        const uint32_t c1 = pl.chbase[r + 1];
        for (uint32_t c0 = pl.chbase[r]; c0 < c1; c0 += 32) {
            uint32_t v[32];
#pragma unroll
            for (int k = 0; k < 32; k++) v[k] = c0 + k < c1 ? cbins[(size_t)(c0 + k) * 256 + t] : 0u;
#pragma unroll
            for (int k = 0; k < 32; k++)
                if (c0 + k < c1) {
                    cbins[(size_t)(c0 + k) * 256 + t] = run;
                    run += v[k];
                }
        }
    }
    uint32_t tot;
    const uint32_t excl = block_exclusive_scan<uint32_t>(run, s_scr, tot);
    if (t < (uint32_t)tiles_x) {
        const uint32_t start = (uint32_t)pl.pbase[r] + excl;
        ranges[r * (uint32_t)tiles_x + t] = run ? make_uint2(~start, start + run) : make_uint2(0u, 0u);
    }
}

// Column pass, scatter: per chunk, its row items expand into one value per
// covered column; tiles of 256*ITEMS values are ranked by column and written in
// column runs at tile start + chunk offset.
template <int ITEMS, int BITS, bool RA, uint32_t CH>
__global__ __launch_bounds__(256) void k_bin_cols_scatter(const uint64_t* __restrict__ rows_in,
                                                           const uint32_t* __restrict__ row_items,
                                                           const unsigned long long* __restrict__ row_pairs,
                                                           uint32_t cap, int tiles_x,
                                                           const uint32_t* __restrict__ cbins,
                                                           const uint2* __restrict__ ranges,
                                                           uint32_t* __restrict__ vals,
                                                           const uint32_t* __restrict__ gate) {
    GSR_GEOM_PRIO();
    if (gate && *gate == 0u) return;
    constexpr uint32_t kTile = 256u * ITEMS;
    __shared__ ColPlan<false> pl;
    // per source (row item of the chunk): exclusive start << 8 | first column; index
    __shared__ uint32_t s_ft[CH], s_idx[CH];
    __shared__ uint16_t s_own[kTile];
    __shared__ uint32_t s_dl[kTile];   // the ranked tile: source slot << 8 | column
    __shared__ uint32_t s_wmax[4];
    // s_dbase[d]: global position of the tile's first value of column d minus its tile slot
    __shared__ uint32_t s_wc[4][256], s_dbase[256], s_lbase[256], s_scr[4];
    __shared__ unsigned long long s_scr64[4];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    if (col_plan<CH>(row_items, row_pairs, pl, s_scr, s_scr64) > cap) return;
    const uint32_t nch = pl.chbase[256];
    for (uint32_t c = blockIdx.x; c < nch; c += gridDim.x) {
        const uint32_t r = col_chunk_row(pl, c);
        const uint32_t ib = pl.rbase[r] + (c - pl.chbase[r]) * CH;
        const uint32_t m = min(CH, pl.rbase[r] + pl.rcnt[r] - ib);
        // column t's running global position (thread t owns column t)
        uint32_t gb = t < (uint32_t)tiles_x ? ~ranges[r * (uint32_t)tiles_x + t].x + cbins[(size_t)c * 256 + t] : 0u;
        // thread t owns row items PER*t .. PER*t + PER-1 of the chunk (source order)
        constexpr int PER = CH / 256;
        uint32_t cnt[PER], start[PER], tx0v[PER];
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const uint32_t j = PER * t + i;
            const uint64_t it = j < m ? rows_in[ib + j] : 0ull;
            const uint32_t tx0 = (uint32_t)((it >> 32) & 0xffffu);
            cnt[i] = j < m ? (uint32_t)(it >> 48) - tx0 + 1u : 0u;
            tx0v[i] = tx0 & 0xffu;
            s_idx[j] = (uint32_t)it;
        }
#pragma unroll
        for (int i = 0; i < ITEMS; i++) s_own[t * ITEMS + i] = 0;
        const uint32_t total = bin_source_starts<PER>(cnt, start, tx0v, s_ft, s_scr);
        uint32_t carry = 0;
        for (uint32_t tb = 0; tb < total; tb += kTile) {
            const uint32_t tn = min(kTile, total - tb);
            bin_tile_owners<ITEMS, PER>(cnt, start, tb, tn, s_own, carry, s_wmax);
            uint32_t dig[ITEMS], pos[ITEMS], src[ITEMS];
#pragma unroll
            for (int k = 0; k < ITEMS; k++) {
                const uint32_t el = min(w * 64 * ITEMS + k * 64 + lane, tn - 1);
                const uint32_t l = (uint32_t)s_own[el] - 1u;
                src[k] = l;
                const uint32_t ft = s_ft[l];
                dig[k] = (ft & 0xffu) + (tb + el - (ft >> 8));
            }
            const uint32_t tcount = bin_rank_tile<ITEMS, BITS, RA>(dig, tn, pos, s_wc, s_lbase, s_scr);
            s_dbase[t] = gb - s_lbase[t];   // this thread's own scan output
#pragma unroll
            for (int i = 0; i < ITEMS; i++) s_own[t * ITEMS + i] = 0;   // for the next tile (rank barriers passed)
#pragma unroll
            for (int k = 0; k < ITEMS; k++) {
                const uint32_t el = w * 64 * ITEMS + k * 64 + lane;
                if (el < tn) s_dl[pos[k]] = (src[k] << 8) | dig[k];
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < ITEMS; k++) {
                const uint32_t q = t + 256 * k;
                const uint32_t qc = min(q, tn - 1);
                const uint32_t x = s_dl[qc];
                const uint32_t v = s_idx[x >> 8];
                const uint32_t dst = s_dbase[x & 0xffu] + qc;
                if (q < tn) vals[dst] = v;
            }
            __syncthreads();
            gb += tcount;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ live partition
//
// Stable partition of the preprocess items ahead of the global depth sort
// (GSR_TUNE_DEPTH_COMPACT): visible items (key != 0xFFFFFFFF) first, in index
// order, then the culled ones, in index order.  The full sort puts the culled
// items last in index order anyway (their key is the maximum, ties by index), so
// sorting only the visible prefix (n_dev = the visible count) gives the same
// order.  The visible items' rect payloads go to pay0 (pass 0 reads them there).
// The culled tail is written to `out` only, with the dead rect in both payload
// buffers at the same positions (the passes never touch the tail, and which buffer
// ends depth-ordered is decided on the device); the binning never reads items whose
// rect is dead, and gsr_read_depth_order takes the tail from `out`.  Three launches: per-chunk
// visible counts, their exclusive scan (+ total), the scatter.
__global__ __launch_bounds__(256) void k_part_count(const uint64_t* __restrict__ in, uint32_t n, int groups,
                                                     uint32_t* __restrict__ counts) {
    GSR_GEOM_PRIO();
    __shared__ uint32_t s_scr[4];
    uint64_t b, e;
    chunk_range(n, groups, blockIdx.x, 256, b, e);
    uint32_t c = 0;
    for (uint64_t i = b + threadIdx.x; i < e; i += 256) c += (uint32_t)(in[i] >> 32) != 0xffffffffu ? 1u : 0u;
    uint32_t tot;
    (void)block_exclusive_scan<uint32_t>(c, s_scr, tot);
    if (threadIdx.x == 0) counts[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void k_part_scan(uint32_t* __restrict__ counts, int groups,
                                                    uint32_t* __restrict__ n_live) {
    GSR_GEOM_PRIO();
    __shared__ uint32_t s_scr[4];
    const int per = (groups + 255) / 256;
    const int b = (int)threadIdx.x * per;
    uint32_t local = 0;
    for (int k = 0; k < per; k++)
        if (b + k < groups) local += counts[b + k];
    uint32_t total;
    uint32_t run = block_exclusive_scan<uint32_t>(local, s_scr, total);
    for (int k = 0; k < per; k++)
        if (b + k < groups) {
            const uint32_t v = counts[b + k];
            counts[b + k] = run;
            run += v;
        }
    if (threadIdx.x == 0) *n_live = total;
}

__global__ __launch_bounds__(256) void k_part_scatter(const uint64_t* __restrict__ in, uint32_t n, int groups,
                                                       const uint32_t* __restrict__ offs,
                                                       const uint32_t* __restrict__ n_live,
                                                       uint64_t* __restrict__ out,
                                                       const uint32_t* __restrict__ rect,
                                                       uint32_t* __restrict__ pay0, uint32_t* __restrict__ pay1) {
    GSR_GEOM_PRIO();
    __shared__ uint32_t s_w[4];
    uint64_t b, e;
    chunk_range(n, groups, blockIdx.x, 256, b, e);
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint32_t live_base = offs[blockIdx.x];
    // culled items before this chunk = b - visible items before it
    uint32_t dead_base = *n_live + (uint32_t)(b - live_base);
    for (uint64_t c0 = b; c0 < e; c0 += 256) {
        const uint64_t i = c0 + t;
        const bool valid = i < e;
        const uint64_t v = valid ? in[i] : 0ull;
        const bool live = valid && (uint32_t)(v >> 32) != 0xffffffffu;
        const bool dead = valid && !live;
        const uint64_t bl = __ballot(live), bd = __ballot(dead);
        if (lane == 0) s_w[w] = (uint32_t)__popcll(bl) | ((uint32_t)__popcll(bd) << 16);
        __syncthreads();
        uint32_t lb = 0, db = 0, ltot = 0, dtot = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t x = s_w[k];
            if (k < w) {
                lb += x & 0xffffu;
                db += x >> 16;
            }
            ltot += x & 0xffffu;
            dtot += x >> 16;
        }
        if (live) {
            const uint32_t q = live_base + lb + (uint32_t)__popcll(bl & lt);
            out[q] = v;
            pay0[q] = rect[(uint32_t)v];   // pass 0 reads the payloads from pay0
        }
        if (dead) {
            const uint32_t q = dead_base + db + (uint32_t)__popcll(bd & lt);
            out[q] = v;
            pay0[q] = pack_rect(kDeadRect);   // the sort's result parity is decided on the device
            pay1[q] = pack_rect(kDeadRect);
        }
        live_base += ltot;
        dead_base += dtot;
        __syncthreads();
    }
}

// ------------------------------------------------------------------ blend


// Bijective XCD-aware remap: blocks that share an XCD (b % 8) get one
// contiguous run of tiles, so neighbouring tiles' shared splats hit one L2.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int xcd = b & 7, q = nb >> 3, r = nb & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

typedef float f2 __attribute__((ext_vector_type(2)));

// Packed product with the HIGH half of the second operand broadcast to both lanes,
// in one v_pk_mul_f32 through op_sel (the compiler otherwise copies that half into
// a fresh register pair first: one v_mov per use in the compositing loop).
// Same IEEE products as the plain expressions (multiplication commutes exactly).
__device__ __forceinline__ f2 pk_mul_b_hi(f2 a, f2 b) {   // (a.x * b.y, a.y * b.y)
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// Packed fused multiply-adds with the second factor's LOW / HIGH half broadcast:
// (fma(a.x, b.x, c.x), fma(a.y, b.x, c.y)) and (fma(a.x, b.y, c.x), fma(a.y, b.y, c.y)).
__device__ __forceinline__ f2 pk_fma_b_lo(f2 a, f2 b, f2 c) {
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ f2 pk_fma_b_hi(f2 a, f2 b, f2 c) {
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// gsr_blend_expf on two lanes at once (v_pk_* for every float op that has a packed
// form: 11 packed + 4 single VALU, against 11 + 6 for the Cephes gsr_expf), for
// inputs the caller has PROVEN finite and in [-2e7, 5]: on [-104, 5] the clamp and
// the NaN select do not change the result and every remaining step is the same IEEE
// operation in the same order, so each half is bit-identical to gsr_blend_expf of
// that half.  Below -104 (no clamp here) n <= -150 — for |x log2 e| >= 2^22 the
// shifter no longer rounds to an integer and the remainder r drifts to |r| < 1.5,
// still finite — so ldexp(y, n) rounds to +0, the clamped result
// (gsr_exp_probe counts the halves that differ from the scalar function over every
// float of [-2e7, 5]: none).  Out-of-box lanes are discarded by the caller.
__device__ __forceinline__ f2 gsr_blend_expf_x2(f2 xc) {
    const f2 t = __builtin_elementwise_fma(xc, (f2)1.44269504088896341f, (f2)12582912.0f);
    const f2 n = t - 12582912.0f;
    f2 r = __builtin_elementwise_fma(-n, (f2)0.693359375f, xc);
    r = __builtin_elementwise_fma(-n, (f2)-2.12194440e-4f, r);
    f2 q = __builtin_elementwise_fma((f2)0x1.6b42a4p-10f, r, (f2)0x1.125e6cp-7f);
    q = __builtin_elementwise_fma(q, r, (f2)0x1.5557c2p-5f);
    q = __builtin_elementwise_fma(q, r, (f2)0x1.555452p-3f);
    q = __builtin_elementwise_fma(q, r, (f2)0x1.fffffcp-2f);
    const f2 r2 = r * r;
    const f2 y = __builtin_elementwise_fma(q, r2, r) + 1.0f;
    f2 res;
    res.x = __builtin_amdgcn_ldexpf(y.x, (int)n.x);
    res.y = __builtin_amdgcn_ldexpf(y.y, (int)n.y);
    return res;
}

// The blend's fast exp (GSR_TUNE_BLEND_EXP 1): e^x as the hardware 2^t (v_exp_f32) of
// t = x log2(e), two lanes at once.  Its relative difference from gsr_blend_expf, with the
// alpha product, is bounded on the argument range a composited lane can have
// (kFxEpsMax, kFxEpsBig below; measured exhaustively by gsr_exp_probe); the
// alpha decisions never use it (xs), and the transmittance test is guarded.
__device__ __forceinline__ f2 fast_expf_x2(f2 x) {
    const f2 t = x * 1.44269504088896341f;
    f2 q;
    q.x = __builtin_amdgcn_exp2f(t.x);
    q.y = __builtin_amdgcn_exp2f(t.y);
    return q;
}

// Fast-exp blend: bounds on |alpha_fast / alpha_exact - 1| for a composited lane
// (opacity in [0, 1] and alpha_exact >= 1e-3, so the exp argument x lies in
// [ln(1e-3), 5]; alpha > 0.5 needs x > ln 0.5, alpha > 0.9 needs x > ln 0.9).  Each is
// the exhaustive maximum of |fast_expf / gsr_blend_expf - 1| over every float x of its
// range (gsr_exp_probe; tests/test_gpu_fastexp.py checks these constants stay above
// it) plus 2^-23 for the two roundings of op * e:
//   kFxEps3  all composited lanes (x >= -6.95)
//   kFxEps2  alpha > 0.5            (x >= -0.70)
//   kFxEps1  alpha > 0.9            (x >= -0.11)
// The transmittance of a pixel then differs from the exact chain's by a relative
//   rho <= 207.1 kFxEps1 + 6.9078 max(3.909 kFxEps2, 1.4427 kFxEps3) + 3 2^-24 n
// (n = composited splats, bounded by the wave's splat-iterations) up to and including
// the step where it first drops below 1e-3 ("Fast exp"):
// kFxBand0 and kFxBandStep are those terms with 2 % headroom.  The n term counts the
// roundings per composite: the exact chain's two (1 - alpha, then the product) and the
// fast chain's one (T - T alpha as one fma).
constexpr float kFxEps3 = 6.6e-7f;
constexpr float kFxEps2 = 4.8e-7f;
constexpr float kFxEps1 = 4.8e-7f;
constexpr float kFxBand0 = 1.02f * (207.1f * kFxEps1 + 6.9078f * (3.909f * kFxEps2 > 1.4427f * kFxEps3
                                                                  ? 3.909f * kFxEps2 : 1.4427f * kFxEps3));
constexpr float kFxBandStep = 1.02f * 3.0f * 0x1p-24f;

// Set in the batch's last pair's second box descriptor (bit 30: above the survivor lane
// at bits 24-29; box_mask reads bits 0-21 only).
constexpr uint32_t kLastPair = 0x40000000u;

// n + (lane's bit of ma) + (lane's bit of mb): the wave masks are the carry-ins of two
// v_addc_co_u32 (one VALU each; counting booleans compiles to selects and an add).
__device__ __forceinline__ uint32_t count_lanes2(uint32_t n, uint64_t ma, uint64_t mb) {
    uint64_t c0, c1;
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(n), "=s"(c0) : "v"(n), "s"(ma));
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(n), "=s"(c1) : "v"(n), "s"(mb));
    (void)c0;
    (void)c1;
    return n;
}

// The band for one pixel from what it composited so far: n splats, the largest alpha
// m.  Besides the worst case above (band0 = kFxBand0), the alpha terms obey
//   sum alpha_i / (1 - alpha_i) <= (sum alpha_i) / (1 - m)
//                              <= (ln 1000 + ln(1 / (1 - m))) / (1 - m)
// (alpha <= -ln(1 - alpha), and the exact T stayed >= 1e-3 before the step being
// tested, whose own alpha is <= m), so rho <= kFxEps3 of that, which is far smaller
// unless some alpha came near 0.99.  2 % headroom over the hardware log / rcp.
// band0 < 0 (measurement builds only) turns the guard off.
__device__ __forceinline__ float fx_band(float band0, uint32_t n, float m) {
    const float om = 1.0f - m;                                 // >= 0.01 (alpha <= 0.99)
    const float lnm = -0.693147181f * __builtin_amdgcn_logf(om);   // ln(1 / (1 - m))
    const float byM = 1.02f * kFxEps3 * (6.9078f + lnm) * __builtin_amdgcn_rcpf(om);
    return __builtin_fmaf((float)n, kFxBandStep, band0 < 0.0f || band0 > 0.5f ? band0 : fminf(band0, byM));
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
// exact one-splat path instead (same values, full gsr_blend_expf, plain selects).
//
// Pair slot dwords (h = 0 / 1 for the first / second splat of the pair):
//   [0+h] cx  [2+h] cy  [4+h] a  [6+h] b  [8+h] c  [10+h] e  [12+h] opacity
//   [14+2h] red  [15+2h] green  [18+h] blue  (fast exp only: [20+h] xs)
//   [22+h] box descriptor | survivor lane << 24 (0: no splat)
struct BlendDiag {
    uint64_t loaded = 0, iter = 0, active = 0, taken = 0, slow = 0, zero_taken = 0, no_cand_pairs = 0;
};

// 64-bit pixel mask (bit row * 8 + col) of a box descriptor built in the cull:
// bits 0-7 the column byte, 8-15 = 56 - 8 (y1 - y0), 16-23 = 8 y0.  Uniform input,
// so it compiles to scalar instructions.
__device__ __forceinline__ uint64_t box_mask(uint32_t d) {
    const uint32_t rep = (d & 0xffu) * 0x01010101u;
    const uint64_t rows = (~0ull >> ((d >> 8) & 0xffu)) << ((d >> 16) & 0xffu);
    return rows & (((uint64_t)rep << 32) | rep);
}

// Diagnostics take map: per pixel, the number of splats composited and a sum of
// a mix of their Gaussian indices (the oracle's orc_render_takes computes the same).
__device__ __forceinline__ uint32_t take_mix(uint32_t g) { return (g + 1u) * 2654435761u; }

// One 8x8 pixel block (bx, by) blended by one wave over the tile list
// idx[beg, end), using the wave's private LDS slice wP (32 pair slots).
//
// FX (fast exp, GSR_TUNE_BLEND_EXP 1): alpha from fast_expf_x2; the alpha test is
// the exact one through the record's xs (-md2/2 >= xs, gsr_alpha_take_min_x), so
// only the transmittance can differ from the exact chain, by less than the band
// kFxBand0 + kFxBandStep n.  The wave flags a pixel ("suspect") when a value of T on
// either side of its first drop below 1e-3 lies within the band of 1e-3, or when
// it ends unsaturated within the band; then the exact T could have taken the other
// branch.  The block writes every other pixel and returns the suspect mask; the
// caller blends the suspect pixels again exactly (FX false, `only` = the mask).  A
// batch holding a record without the fast proof aborts the fast pass (all ones, no
// pixel written).  Every pixel therefore composites exactly the splats the exact
// blend composites, in the same order.
//
// SPLIT (depth split, exact blend only): 1 = phase A, which composites the block's
// phase-A list and, when some pixel is still unsaturated at its end, saves every
// pixel's T in tsave (64 floats), sets *flag and counts the block in *gate (else
// clears *flag); 2 = phase B, which resumes such a block from the saved T and the
// colours phase A wrote (and, with DIAG, the take map).  Each pixel composites the
// same splats in the same order as over the whole list (the phase-A list is the
// nearest part of it, the phase-B list the rest), with the same operations.
template <bool DIAG, bool FX, int SPLIT>
__device__ __forceinline__ uint64_t blend_block(const uint32_t* __restrict__ idx, const uint4* __restrict__ rec,
                                                uint32_t beg, uint32_t end, int bx, int by, int lane, int W,
                                                int H, int cover_w, int cover_h, float* __restrict__ out,
                                                float* wP, BlendDiag& dg, uint64_t* __restrict__ tmap,
                                                float band0, uint64_t only, float* __restrict__ tsave = nullptr,
                                                uint8_t* __restrict__ flag = nullptr,
                                                uint32_t* __restrict__ gate = nullptr) {
    static_assert(SPLIT == 0 || !FX, "the depth split runs the exact blend");
    constexpr int kSlot = 24;                               // dwords per pair slot
    const int px = bx + (lane & 7), py = by + (lane >> 3);
    const bool inside = px < cover_w && py < cover_h;
    const float fpx = (float)px, fpy = (float)py;
    // transmittance; a pixel is saturated ("done", render.cu:328) iff T < 1e-3.
    // Pixels outside the covered area start saturated (T = 0) and write 0; so do the
    // pixels outside `only` (the exact re-blend of a fast block's suspect pixels).
    const bool mine = ((only >> lane) & 1ull) != 0ull;
    float T = inside && mine ? 1.0f : 0.0f;
    f2 crg = (f2)0.0f;
    float cb = 0.0f;
    const float4* wP4 = reinterpret_cast<const float4*>(wP);
    uint64_t suspect = 0;      // FX: pixels whose T decisions the band cannot vouch for
    uint32_t ntk = 0;          // FX: splats this pixel composited so far
    float amax = 0.0f;         // FX: largest alpha it composited
    float tprev = 1.0f;        // FX: T before the pixel's latest composite
    uint32_t tcount = 0, thash = 0;   // DIAG take map
    if (SPLIT == 2 && inside) {
        // inside => px < W and py < H (cover_w <= W, cover_h <= H)
        const size_t o = (size_t)py * (size_t)W + (size_t)px, hw = (size_t)W * (size_t)H;
        T = tsave[lane];
        crg.x = out[o];
        crg.y = out[hw + o];
        cb = out[2 * hw + o];
        if (DIAG && tmap) {
            const uint64_t tm = tmap[o];
            tcount = (uint32_t)tm;
            thash = (uint32_t)(tm >> 32);
        }
    }

    uint4 ra = make_uint4(0, 0, 0, 0), rb = ra, rc = ra, rd = ra;
    uint32_t nidx = 0, cidx = 0;
    if (beg + lane < end) {
        cidx = idx[beg + lane];
        const uint4* R = rec + 4 * (uint64_t)cidx;
        ra = R[0];
        rb = R[1];
        rc = R[2];
        rd = R[3];
    }
    if (beg + 64 + lane < end) nidx = idx[beg + 64 + lane];
    bool alive = __ballot(!(T < 1e-3f)) != 0ull;
    for (uint32_t base = beg; base < end && alive; base += 64) {
        const uint32_t cnt = min(64u, end - base);
        // ---- cull + lane masks + compaction (lane = record) ----
        // pixels not yet saturated at the batch start: T only decreases, so a record
        // whose in-box pixels are all saturated here can never be taken in this batch
        const uint64_t live_b = __ballot(!(T < 1e-3f));
        // branch-free over the 64 lanes: nearly every batch has lanes on both sides of each
        // test, so branches would only add exec-mask work (lanes >= cnt hold stale
        // registers: their results are discarded through `valid`)
        bool hit, fast;
        uint32_t dsc;
        {
            const bool valid = (uint32_t)lane < cnt;
            const int xmin = (int)(rc.z & 0xffffu), xmax = (int)(rc.z >> 16);
            const int ymin = (int)(rc.w & 0xffffu), ymax = (int)(rc.w >> 16);
            const bool box_hit = valid & !((xmax < bx) | (xmin > bx + 7) | (ymax < by) | (ymin > by + 7));
            {
                const float cx = __uint_as_float(rc.x), cy = __uint_as_float(rc.y);
                const float a = __uint_as_float(ra.x), b = __uint_as_float(ra.y);
                const float c = __uint_as_float(ra.z), e = __uint_as_float(ra.w);
                const int x0 = max(xmin - bx, 0), x1 = min(xmax - bx, 7);
                const int y0 = max(ymin - by, 0), y1 = min(ymax - by, 7);
                const float dx0 = (float)(bx + x0) - cx, dx1 = (float)(bx + x1) - cx;
                const float dy0 = (float)(by + y0) - cy, dy1 = (float)(by + y1) - cy;
                // the box as a descriptor (box_mask: bit row * 8 + col of the block = pixel
                // inside the AABB), expanded on the scalar unit by the compositing loop:
                // column byte | (56 - 8 (y1 - y0)) << 8 | 8 y0 << 16
                // (shift counts masked to the hardware's: only lanes outside the box can
                // have them out of range, and their results are discarded)
                const uint32_t colb = (0xffu >> ((uint32_t)(7 - (x1 - x0)) & 31u)) << ((uint32_t)x0 & 31u);
                const uint32_t rsh = (uint32_t)(56 - 8 * (y1 - y0)) & 63u, lsh = (uint32_t)(8 * y0) & 63u;
                dsc = colb | (rsh << 8) | (lsh << 16);
                // the same 64-bit mask here, only for the saturation filter below
                const uint64_t rows = (~0ull >> rsh) << lsh;
                const uint32_t rep = __builtin_amdgcn_perm(colb, colb, 0u);   // colb in every byte
                const uint64_t lrows = rows & live_b;
                // cull word (cull_word): per-record parts of the block test and the proof
                const float S = __uint_as_float(rd.w);
                const float M = fmaxf(fmaxf(fabsf(dx0), fabsf(dx1)), fmaxf(fabsf(dy0), fabsf(dy1)));
                const float SMM = S * M * M;
                hit = box_hit & ((((uint32_t)lrows | (uint32_t)(lrows >> 32)) & rep) != 0u) &
                      block_may_reach(a, b, c, e, __uint_as_float(rd.y), __uint_as_float(rd.z), dx0, dx1, dy0,
                                      dy1, SMM, block_cut(__uint_as_float(rd.x)));
                fast = SMM <= 4e7f;   // per-block part of the fast-path proof
                // the fast exp's error bound assumes opacity in [0, 1] (NaN fails)
                if (FX) fast = fast && __uint_as_float(rb.x) <= 1.0f;
            }
        }
        const uint64_t m = __ballot(hit);
        const uint32_t nsurv = (uint32_t)__popcll(m);
        const bool all_fast = __ballot(hit & !fast) == 0ull;
        if (FX && !all_fast) return ~0ull;   // exact re-blend of the whole block
        if (hit) {
            const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            float* S = wP + (k >> 1) * kSlot;
            const int h = (int)(k & 1u);
            S[0 + h] = __uint_as_float(rc.x);
            S[2 + h] = __uint_as_float(rc.y);
            // fast batches store the conic pre-scaled by -0.5 (exact, see coef_ok)
            const float sc = all_fast ? -0.5f : 1.0f;
            S[4 + h] = sc * __uint_as_float(ra.x);
            S[6 + h] = sc * __uint_as_float(ra.y);
            S[8 + h] = sc * __uint_as_float(ra.z);
            S[10 + h] = sc * __uint_as_float(ra.w);
            S[12 + h] = __uint_as_float(rb.x);
            S[14 + 2 * h] = __uint_as_float(rb.y);
            S[15 + 2 * h] = __uint_as_float(rb.z);
            S[18 + h] = __uint_as_float(rb.w);
            if (FX) S[20 + h] = __uint_as_float(rd.x);
            // box descriptor (box_mask) | survivor lane << 24: the compositing loop reads
            // both splats' from the slot instead of walking the survivor mask.  The last
            // pair's second descriptor carries kLastPair (below)
            S[22 + h] = __uint_as_float(dsc | ((uint32_t)lane << 24) | (k + 1u == nsurv && h ? kLastPair : 0u));
        }
        if ((nsurv & 1u) && lane < 11) {
            // odd count: zero the unused second half of the last slot (descriptor 0 = empty
            // box keeps it inert); second-half dwords of a slot: 1 3 5 7 9 11 13 | 16 17 |
            // 19 | 23 (arithmetic, not a table: a table load would stall the wave on memory
            // once per odd batch)
            // (dword 23, the pair's second descriptor: kLastPair alone, an empty box)
            wP[(nsurv >> 1) * kSlot + (lane < 7 ? 2 * lane + 1 : lane < 10 ? lane + 9 + (lane == 9) : 23)] =
                lane == 10 ? __uint_as_float(kLastPair) : 0.0f;
        }
        if (DIAG) dg.loaded += cnt;
        const float xs_l = DIAG ? __uint_as_float(rd.x) : 0.0f;   // diagnostics: xs of record `lane`
        const uint32_t gi_l = cidx;                                // diagnostics: its Gaussian index
        // ---- prefetch: records of batch k+1, indices of batch k+2 ----
        if (base + 64 + lane < end) {
            cidx = nidx;
            const uint4* R = rec + 4 * (uint64_t)nidx;
            ra = R[0];
            rb = R[1];
            rc = R[2];
            rd = R[3];
        }
        if (base + 128 + lane < end) nidx = idx[base + 128 + lane];

        uint64_t mm = m;
        if (all_fast) {
            // lanes not yet saturated; the end-of-iteration ballot of T2 is the next
            // iteration's "!(T < 1e-3)" (render.cu:328), so it is compared once
            uint64_t live = __ballot(!(T < 1e-3f));
            f2 TT;
            TT.x = T;
            TT.y = T;
            const uint32_t npairs = (uint32_t)__builtin_amdgcn_readfirstlane((int)((nsurv + 1u) >> 1));
            // one exit test per pair: after the batch's last pair `live` is 0 (the threshold
            // above; the next batch recomputes it from T), so the loop stops when the block
            // saturates or the batch ends
            if (npairs != 0u) {
#pragma unroll
            for (uint32_t j = 0; j < 32u;) {   // unrolled: the slot offsets are immediates
                const float4 q0 = wP4[j * (kSlot / 4) + 0], q1 = wP4[j * (kSlot / 4) + 1];
                const float4 q2 = wP4[j * (kSlot / 4) + 2], q3 = wP4[j * (kSlot / 4) + 3];
                const float4 q4 = wP4[j * (kSlot / 4) + 4];
                // the pair's box descriptors from the slot (one v_readfirstlane each); the
                // 64-bit lane masks are rebuilt from them by scalar instructions.  The
                // unused half of an odd batch's last slot holds descriptor 0: an empty box.
                // No survivor-mask walk, no "second splat?" selects: the loop's scalar
                // work is a co-bound of the VALU work (round 4).
                uint32_t dd0, dd1;
                float2 xs;
                if (FX) {
                    const float4 q5 = wP4[j * (kSlot / 4) + 5];
                    xs = make_float2(q5.x, q5.y);
                    dd0 = __float_as_uint(q5.z);
                    dd1 = __float_as_uint(q5.w);
                } else {
                    const float2 dd = *reinterpret_cast<const float2*>(wP + j * kSlot + 22);
                    dd0 = __float_as_uint(dd.x);
                    dd1 = __float_as_uint(dd.y);
                }
                const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)dd0);
                const uint32_t d1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)dd1);
                const uint64_t box0 = box_mask(d0), box1 = box_mask(d1);
                const bool has1 = (d1 & 0xffu) != 0u;                        // diagnostics
                const int s0 = (int)(d0 >> 24), s1 = has1 ? (int)((d1 >> 24) & 63u) : s0;
                // render.cu:329-332, same operation order and fused multiply-adds
                // (gsr_blend_md2), both splats at once; the conic is stored pre-scaled
                // by -0.5, so this is -0.5f * md2 exactly
                const f2 dx = (f2)fpx - (f2){q0.x, q0.y};
                const f2 dy = (f2)fpy - (f2){q0.z, q0.w};
                const f2 u = __builtin_elementwise_fma((f2){q1.x, q1.y}, dx, (f2){q1.z, q1.w} * dy);
                const f2 v = __builtin_elementwise_fma((f2){q2.x, q2.y}, dx, (f2){q2.z, q2.w} * dy);
                const f2 mdh = __builtin_elementwise_fma(dx, u, dy * v);
                const f2 ee = FX ? fast_expf_x2(mdh) : gsr_blend_expf_x2(mdh);
                const f2 al = (f2){q3.x, q3.y} * ee;
                const float al0 = fminf(al.x, 0.99f), al1 = fminf(al.y, 0.99f);
                // alpha tests (render.cu:335): on alpha itself, or (FX) on the exp
                // argument against xs — the same decisions
                bool pass0, pass1;
                if (FX) {
                    pass0 = !(mdh.x < xs.x);
                    pass1 = !(mdh.y < xs.y);
                } else {
                    pass0 = !(al0 < 1e-3f);
                    pass1 = !(al1 < 1e-3f);
                }
                // render.cu:333-340: splat 2j, then splat 2j+1 against what 2j left
                const bool in0 = __builtin_amdgcn_inverse_ballot_w64(box0 & live);
                const bool in1 = __builtin_amdgcn_inverse_ballot_w64(box1);
                // (a0, a1) and (T, T1) live in register pairs, written in place, so
                // the packed blue product needs no moves; TT.x carries T across.
                // FX forms the take decisions as wave masks (the composited-splat
                // count below uses them as carry-ins)
                uint64_t t0m = 0, t1m = 0;
                bool take0, take1;
                f2 AA;
                if (FX) {
                    t0m = box0 & live & __builtin_amdgcn_ballot_w64(pass0);
                    take0 = __builtin_amdgcn_inverse_ballot_w64(t0m);
                    tprev = take0 ? TT.x : tprev;
                } else {
                    take0 = in0 & pass0;
                }
                AA.x = take0 ? al0 : 0.0f;
                // T (1 - alpha) (render.cu:339); the fast blend folds it into one fma, T - T alpha
                // with one rounding (kFxBandStep: 3 2^-24 per composite, 1 here and 2 in the
                // exact chain)
                TT.y = FX ? __builtin_fmaf(-TT.x, AA.x, TT.x) : TT.x * (1.0f - AA.x);
                if (FX) {
                    t1m = box1 & __builtin_amdgcn_ballot_w64(!(TT.y < 1e-3f)) & __builtin_amdgcn_ballot_w64(pass1);
                    take1 = __builtin_amdgcn_inverse_ballot_w64(t1m);
                    tprev = take1 ? TT.y : tprev;
                } else {
                    take1 = in1 & !(TT.y < 1e-3f) & pass1;
                }
                AA.y = take1 ? al1 : 0.0f;
                // the three colour products, then rgb += (col * alpha) * T as fused
                // multiply-adds in list order (render.cu:337, the contraction
                // gsr_blend_md2 documents)
                const f2 p0 = (f2){q3.z, q3.w} * AA.x;
                const f2 p1 = pk_mul_b_hi((f2){q4.x, q4.y}, AA);     // col1 * AA.y
                const f2 pb = (f2){q4.z, q4.w} * AA;
                crg = pk_fma_b_lo(p0, TT, crg);                      // + (col0 * AA.x) * TT.x
                crg = pk_fma_b_hi(p1, TT, crg);                      // + (col1 * AA.y) * TT.y
                cb = __builtin_fmaf(pb.y, TT.y, __builtin_fmaf(pb.x, TT.x, cb));
                if (DIAG) {
                    // splat-iterations with no taken lane; pair-iterations in which no live
                    // in-box lane of either splat passes the alpha test's exp argument
                    const float xs0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xs_l), s0));
                    const float xs1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xs_l), s1));
                    const bool cand0 = in0 && !(mdh.x < xs0);
                    const bool cand1 = has1 && in1 && !(TT.x < 1e-3f) && !(mdh.y < xs1);
                    dg.zero_taken += (__ballot(take0) == 0ull ? 1 : 0) + (has1 && __ballot(take1) == 0ull ? 1 : 0);
                    dg.no_cand_pairs += (__ballot(cand0 || cand1) == 0ull) ? 1 : 0;
                    dg.iter += has1 ? 2 : 1;
                    dg.active += (uint64_t)__popcll(__ballot(in0)) +
                                (uint64_t)__popcll(__ballot(in1 & !(TT.y < 1e-3f)));
                    dg.taken += (uint64_t)__popcll(__ballot(take0)) + (uint64_t)__popcll(__ballot(take1));
                    const uint32_t g0 = (uint32_t)__builtin_amdgcn_readlane((int)gi_l, s0);
                    const uint32_t g1 = (uint32_t)__builtin_amdgcn_readlane((int)gi_l, s1);
                    tcount += (take0 ? 1u : 0u) + (take1 ? 1u : 0u);
                    thash += (take0 ? take_mix(g0) : 0u) + (take1 ? take_mix(g1) : 0u);
                }
                TT.x = FX ? __builtin_fmaf(-TT.y, AA.y, TT.y) : TT.y * (1.0f - AA.y);
                // render.cu:328 for the next pair; after the batch's last pair the threshold
                // is ~3.4e35 (1e-3's bits | kLastPair), so the ballot is 0 and the loop ends:
                // the batch-end test costs two scalar instructions, not a compare of j
                const float thr = __uint_as_float(0x3a83126fu | (d1 & kLastPair));
                const uint64_t live_new = __ballot(!(TT.x < thr));
                if (FX) {
                    // n += take0 + take1 as two v_addc (the take masks as carry-in);
                    // alpha >= +0 here, so its float maximum is the u32 maximum
                    ntk = count_lanes2(ntk, t0m, t1m);
                    amax = __uint_as_float(max(max(__float_as_uint(amax), __float_as_uint(AA.x)),
                                               __float_as_uint(AA.y)));
                    // (the band checks of each pixel's T decisions run once, at the block's
                    // end, on the latched T before its last composite: no per-iteration branch)
                }
                ++j;
                live = live_new;
                if (live == 0ull) break;
            }
            }
            alive = __ballot(!(TT.x < 1e-3f)) != 0ull;   // block not yet saturated
            T = TT.x;
        } else {
            // exact one-splat path (render.cu:329-340 with gsr_blend_expf and selects)
            for (uint32_t k = 0; mm && alive; ++k) {
                const int s = __builtin_ctzll(mm);
                mm &= mm - 1;
                const uint64_t box = box_mask((uint32_t)__builtin_amdgcn_readlane((int)dsc, s));
                const float* S = wP + (k >> 1) * kSlot;
                const int h = (int)(k & 1u);
                const float dx = fpx - S[0 + h], dy = fpy - S[2 + h];
                const float md = gsr_blend_md2(dx, dy, S[4 + h], S[6 + h], S[8 + h], S[10 + h]);
                const float ee = gsr_blend_expf(-0.5f * md);
                float alpha = S[12 + h] * ee;
                alpha = fminf(alpha, 0.99f);
                const bool in = __builtin_amdgcn_inverse_ballot_w64(box);
                const bool take = in & !(T < 1e-3f) & !(alpha < 1e-3f);
                const float wr = __builtin_fmaf(S[14 + 2 * h] * alpha, T, crg.x);
                const float wg = __builtin_fmaf(S[15 + 2 * h] * alpha, T, crg.y);
                const float wb = __builtin_fmaf(S[18 + h] * alpha, T, cb);
                const float Tn = T * (1.0f - alpha);
                if (DIAG) {
                    dg.iter += 1;
                    dg.slow += 1;
                    dg.active += (uint64_t)__popcll(__ballot(in & !(T < 1e-3f)));
                    dg.taken += (uint64_t)__popcll(__ballot(take));
                    tcount += take ? 1u : 0u;
                    thash += take ? take_mix((uint32_t)__builtin_amdgcn_readlane((int)gi_l, s)) : 0u;
                }
                crg.x = take ? wr : crg.x;
                crg.y = take ? wg : crg.y;
                cb = take ? wb : cb;
                T = take ? Tn : T;
                alive = __ballot(!(T < 1e-3f)) != 0ull;
            }
        }
    }
    if (FX) {
        // The band checks, once per pixel.  A pixel's n, m and tprev stop changing once
        // its T drops below 1e-3 (nothing is composited after), so at the end:
        //  - saturated: its decisive step took T from tprev (>= 1e-3) to T (< 1e-3); the
        //    exact chain takes the same branches if both lie outside the band (every
        //    earlier T is >= tprev: T never increases);
        //  - unsaturated: T must lie above the band.
        // Pixels that started saturated (outside the cover or `only`) composited nothing.
        const float B = fx_band(band0, ntk, amax);
        const float hi = 1e-3f * (1.0f + B), lo = 1e-3f * (1.0f - B);
        const bool nr = (T < 1e-3f) ? (ntk != 0u) & ((tprev < hi) | !(T < lo)) : (T < hi);
        suspect |= __ballot(nr);
    }
    if (SPLIT == 1) {
        const bool unsat = __ballot(!(T < 1e-3f)) != 0ull;
        if (unsat) tsave[lane] = T;
        if (lane == 0) {
            *flag = unsat ? 1u : 0u;
            if (unsat) atomicAdd(gate, 1u);
        }
        suspect = unsat ? 1ull : 0ull;   // returned: the caller flags a speculative frame
    }
    // FX: every pixel but the suspect ones; exact: the pixels of `only`
    const bool write = FX ? ((suspect >> lane) & 1ull) == 0ull : mine;
    if (write && px < W && py < H) {
        const size_t o = (size_t)py * (size_t)W + (size_t)px;
        const size_t hw = (size_t)W * (size_t)H;
        out[o] = inside ? crg.x : 0.0f;
        out[hw + o] = inside ? crg.y : 0.0f;
        out[2 * hw + o] = inside ? cb : 0.0f;
        if (DIAG && tmap) tmap[o] = (uint64_t)tcount | ((uint64_t)thash << 32);
    }
    return suspect;
}

// One-wave workgroups: workgroup g blends one 8x8 block, so a finished block
// frees its wave slot at once (no waiting for the tile's other three waves).
// Hardware dispatch sends workgroup g to XCD g mod 8.  bands > 1: the blocks
// (tile-major, a tile's four blocks consecutive) are cut into bands of B
// consecutive blocks and band j goes to XCD j mod 8, so each XCD's L2 serves runs
// of neighbouring tiles while heavy and light image regions spread over all XCDs;
// padding workgroups past the last block exit.  bands <= 1: one contiguous run of
// blocks per XCD (xcd_remap).
// FX: fast-exp blend; a block it cannot vouch for is blended again exactly by the
// same wave (counters[8] blocks, counters[9] suspect pixels, with diagnostics).
// STAMPS (timeline diagnostics, no counters): counters[2 * g] = start of the
// s_memrealtime clock (100 MHz), counters[2 * g + 1] = duration (40 bits) |
// placement << 40 (XCC id and HW_ID's SE / SH / CU / SIMD / slot).
// DIAG: counters[0..9], then the take map (one u64 per pixel) from counters + 16.
// SPLIT: the depth split's phase A (1) or B (2), blend_block; phase B's workgroup 0
// publishes the count of blocks phase A left unsaturated (sp.host_st), and every
// workgroup returns at once when that count is 0 or its own block is saturated.
template <bool DIAG, bool STAMPS, bool FX, int SPLIT>
__global__ __launch_bounds__(64, 8) void k_blend_w(const uint32_t* __restrict__ idx,
                                                 const uint2* __restrict__ ranges,
                                                 const uint4* __restrict__ rec, int tiles_x, int tiles_y,
                                                 int W, int H, int cover_w, int cover_h,
                                                 float* __restrict__ out,
                                                 unsigned long long* __restrict__ counters, int bands,
                                                 float band0, BlendSplit sp) {
    __shared__ float4 sP[32 * 24 / 4];
    const int ntiles = tiles_x * tiles_y;
    const int vb = (int)blockIdx.x;
    if (SPLIT == 1 && vb == 0 && threadIdx.x == 0 && sp.cut.kcut) split_cut_update(sp.cut);
    if (SPLIT == 2) {
        const uint32_t g = *sp.gate;   // uniform
        if (vb == 0 && threadIdx.x == 0 && sp.host_st) {
            // a frame whose near part fell short of the split point by more than 1/16 (its
            // threshold was extrapolated from a smaller point, split_cut_update) says
            // nothing about that point: its tag's low half 0xffff matches no split point
            // (<= 1000), so the controller waits for a frame with a measured threshold
            // rather than grow twice on one miss
            const bool short_near = sp.cut.nnear && *sp.cut.nnear < sp.cut.na - sp.cut.na / 16u;
            sp.host_st->split_unsat = g;
            sp.host_st->split_pm = short_near ? (sp.pm | 0xffffu) : sp.pm;
            __threadfence_system();
        }
        if (g == 0u) return;
    }
    int L;
    if (bands > 1) {
        const int nu = 4 * ntiles;
        const int B = (nu + 8 * bands - 1) / (8 * bands);
        const int k = vb >> 3;
        L = ((k / B) * 8 + (vb & 7)) * B + k % B;
        if (L >= nu) return;
    } else {
        if (vb >= ntiles * 4) return;
        L = xcd_remap(vb, ntiles * 4);
    }
    if (SPLIT == 2 && sp.bflag[L] == 0u) return;   // saturated in phase A: its pixels are final
    const int tile = L >> 2, sub = L & 3;
    const int tx = tile % tiles_x, ty = tile / tiles_x;
    const int lane = (int)(threadIdx.x & 63u);
    uint64_t t_start = 0, place = 0;
    if (STAMPS && lane == 0) {
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        place = ((uint64_t)(xcc & 7u) << 16) | (hw & 0xffffu);
        t_start = __builtin_amdgcn_s_memrealtime();
        counters[2 * vb] = t_start;
    }
    const uint2 rr = ranges[tile];                          // {~start, end}, zero = empty
    const uint32_t beg = rr.y ? ~rr.x : 0u;
    const int bx = tx * GSR_TILE_PX + (sub & 1) * 8, by = ty * GSR_TILE_PX + (sub >> 1) * 8;
    uint64_t* tmap = DIAG ? reinterpret_cast<uint64_t*>(counters + 16) : nullptr;
    BlendDiag dg;
    const uint64_t redo = blend_block<DIAG, FX, SPLIT>(idx, rec, beg, rr.y, bx, by, lane, W, H, cover_w, cover_h,
                                                       out, reinterpret_cast<float*>(sP), dg, tmap, band0, ~0ull,
                                                       SPLIT ? sp.tbuf + 64 * (size_t)L : nullptr,
                                                       SPLIT ? sp.bflag + L : nullptr, sp.gate);
    if (SPLIT == 1 && redo && sp.spec_host && lane == 0) {
        sp.spec_host->spec_miss = 1u;   // no phase B queued for this frame: it is incomplete
        if (sp.fstatus) atomicOr(sp.fstatus, 4u);
        __threadfence_system();
    }
    if (FX && redo) {
        if (DIAG && lane == 0) {
            atomicAdd(counters + 8, 1ull);
            atomicAdd(counters + 9, (unsigned long long)__popcll(redo));
        }
        // only the suspect pixels (all of them after an aborted fast pass): the others
        // start saturated, so the cull drops every record that misses the suspects
        // and the wave stops once they saturate
        blend_block<DIAG, false, 0>(idx, rec, beg, rr.y, bx, by, lane, W, H, cover_w, cover_h, out,
                                 reinterpret_cast<float*>(sP), dg, tmap, 0.0f, redo);
    }
    if (STAMPS && lane == 0)
        counters[2 * vb + 1] = ((__builtin_amdgcn_s_memrealtime() - t_start) & ((1ull << 40) - 1)) | (place << 40);
    if (DIAG && lane == 0) {
        if (sub == 0 && dg.loaded) atomicAdd(counters, (unsigned long long)dg.loaded);
        atomicAdd(counters + 1, (unsigned long long)dg.iter);
        atomicAdd(counters + 2, (unsigned long long)dg.active);
        atomicAdd(counters + 3, (unsigned long long)dg.taken);
        atomicAdd(counters + 4, (unsigned long long)dg.slow);
        atomicAdd(counters + 5, (unsigned long long)dg.zero_taken);
        atomicAdd(counters + 7, (unsigned long long)dg.no_cand_pairs);
        atomicAdd(counters + 6, (unsigned long long)(dg.iter * 64));
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

// ------------------------------------------------------------------ rank-order self-check
//
// The RA rank path (match_peers' comment) relies on same-address ds_add_rtn_u32 lanes
// of one wave64 instruction returning the old values in lane order.  The runtime runs
// this check once per process and device before it uses that path: every wave of
// 256-thread workgroups (per-wave counters, as in the sort and binning kernels) ranks
// digits from 24 patterns — 1 to 256 distinct digits; uniform, a third of the lanes on
// one digit, runs of 16 lanes, interleaved; ~1/8 of the lanes idle — by returning
// atomics and by ballot matching, and counts the lanes where the two differ.
__device__ __forceinline__ uint32_t rank_check_hash(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(256) void k_rank_order_check(uint32_t seed, int iters,
                                                           unsigned long long* __restrict__ out) {
    __shared__ uint32_t cnt[4][256];
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
#pragma unroll
    for (int k = 0; k < 4; k++) cnt[k][t] = 0;
    __syncthreads();
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    unsigned long long bad = 0, ops = 0;
    for (int pat = 0; pat < 24; pat++) {
        const int skew = pat / 6;
        constexpr uint32_t kDigits[6] = {1u, 2u, 4u, 16u, 128u, 256u};
        const uint32_t ndig = kDigits[pat % 6];
        for (int it = 0; it < iters; it++) {
            const uint32_t h = rank_check_hash(seed ^ (blockIdx.x * 7919u + (uint32_t)(pat * iters + it) * 104729u +
                                                       lane * 31u + w * 1000003u));
            uint32_t d = h % ndig;
            if (skew == 1) d = (h >> 8) % 3u == 0u ? 0u : d;
            if (skew == 2) d = (lane >> 4) % ndig;
            if (skew == 3) d = ((h >> 4) & 1u) ? (lane * 5u) % ndig : 1u % ndig;
            const bool valid = ((h >> 20) & 7u) != 0u;
            const uint64_t peers = match_peers<8>(d, valid, 8);
            uint32_t before = 0;
            if (valid) before = cnt[w][d];
            __builtin_amdgcn_wave_barrier();
            uint32_t got = 0;
            if (valid) got = atomicAdd(&cnt[w][d], 1u);
            __builtin_amdgcn_wave_barrier();
            if (valid) {
                bad += got != before + (uint32_t)__popcll(peers & lt);
                ops++;
            }
        }
    }
    // wave sums, one device atomic per wave
    for (int o = 32; o >= 1; o >>= 1) {
        bad += __shfl_xor(bad, o, 64);
        ops += __shfl_xor(ops, o, 64);
    }
    if (lane == 0) {
        atomicAdd(&out[0], ops);
        atomicAdd(&out[1], bad);
    }
}

// ------------------------------------------------------------------ math probe

__global__ void k_math_probe(const float* __restrict__ in, int n, float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = in[2 * i], y = in[2 * i + 1];
    float* o = out + 9 * i;
    o[0] = gsr_expf(x);
    o[8] = gsr_blend_expf(x);
    o[1] = gsr_sinf(x);
    o[2] = gsr_cosf(x);
    o[3] = gsr_atan2f(x, y);
    o[4] = sqrtf(x);
    o[5] = x / y;
    o[6] = roundf(x);
    o[7] = __int_as_float(gsr_f2i_sat(x * 1000.0f));
}

// Exhaustive checks behind the blend's exp (gsr_exp_probe).  Over every float key k
// in [key_lo, key_hi): viol[0] counts gsr_blend_expf(x_k) > gsr_blend_expf(x_k+1)
// (monotonicity of the exact exp, which makes the alpha test a threshold on its
// argument); viol[1] counts the x in [-2e7, 5] where a half of gsr_blend_expf_x2 differs
// from gsr_blend_expf (the packed path's unclamped domain); and over the same keys the
// largest |fast_expf / gsr_blend_expf - 1| is kept as float bits, split at x >= x_big:
// errs[0] every key (x in the range), errs[1] x >= x_big.
__global__ __launch_bounds__(256) void k_exp_probe(uint32_t key_lo, uint32_t key_hi, float x_big,
                                                   unsigned long long* __restrict__ viol,
                                                   uint32_t* __restrict__ errs) {
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    uint64_t bad = 0, pk_bad = 0;
    float emax = 0.0f, ebig = 0.0f;
    for (uint64_t k = (uint64_t)key_lo + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < key_hi; k += nthr) {
        const float x = gsr_key_float((uint32_t)k);
        const float e = gsr_blend_expf(x);
        const float en = gsr_blend_expf(gsr_key_float((uint32_t)k + 1u));
        bad += e > en ? 1u : 0u;
        f2 xx;
        xx.x = x;
        xx.y = -x;
        if (x >= -2e7f && x <= 5.0f) {
            const f2 pk = gsr_blend_expf_x2(xx);
            pk_bad += __float_as_uint(pk.x) != __float_as_uint(e) ? 1u : 0u;
            if (-x >= -2e7f && -x <= 5.0f)
                pk_bad += __float_as_uint(pk.y) != __float_as_uint(gsr_blend_expf(-x)) ? 1u : 0u;
        }
        const float f = fast_expf_x2(xx).x;
        const float r = (float)fabs((double)f / (double)e - 1.0);   // rounded up below
        const float ru = __uint_as_float(__float_as_uint(r) + 1u);
        emax = fmaxf(emax, ru);
        if (x >= x_big) ebig = fmaxf(ebig, ru);
    }
    if (bad) atomicAdd(viol, (unsigned long long)bad);
    if (pk_bad) atomicAdd(viol + 1, (unsigned long long)pk_bad);
    atomicMax(errs, __float_as_uint(emax));
    atomicMax(errs + 1, __float_as_uint(ebig));
}

// gsr_alpha_take_min_x on the device, one opacity per thread (tests).
__global__ void k_xs_probe(const float* __restrict__ op, int n, float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = gsr_alpha_take_min_x(op[i]);
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
                             uint4* rec, uint64_t* items, uint64_t* rect, bool packed, bool four_d, bool sh3,
                             float t, hipStream_t s, uint16_t* spans, const RecSplit* rsp) {
    if (n <= 0) return hipSuccess;
    const RecSplit rs = rsp ? *rsp : RecSplit{0, nullptr, nullptr, nullptr};
    if ((rs.mode == 1 && (!rs.kcut || !rs.kcut_frame || spans)) || (rs.mode == 2 && !rs.kcut_frame) || rs.mode < 0 ||
        rs.mode > 2)
        return hipErrorInvalidValue;
    const dim3 g(grid_for(n, 256));
    const int pk = packed ? 1 : 0;
    if (four_d)
        hipLaunchKernelGGL((k_preprocess<true, false>), g, dim3(256), 0, s, arrays, stride, n, fr, rec, items, rect,
                           pk, packed ? spans : nullptr, t, rs);
    else if (sh3)
        hipLaunchKernelGGL((k_preprocess<false, true>), g, dim3(256), 0, s, arrays, stride, n, fr, rec, items, rect,
                           pk, packed ? spans : nullptr, t, rs);
    else
        hipLaunchKernelGGL((k_preprocess<false, false>), g, dim3(256), 0, s, arrays, stride, n, fr, rec, items, rect,
                           pk, packed ? spans : nullptr, t, rs);
    return hipGetLastError();
}

// A filtered pass 0 ranks by the rect payloads it reads at each position (rect_direct).
static bool carry_ok(const uint32_t* pay0, int rect_direct) { return pay0 != nullptr && rect_direct > 0; }

template <int ITEMS, bool RA>
static void radix_pass(const uint64_t* in, uint64_t* out, const uint32_t* n_dev, uint32_t n_host, int shift,
                       int bits, int groups, uint32_t* hist, uint32_t* totals, uint2* ranges, uint32_t* dstats,
                       int pass, const uint32_t* rect, int rect_direct, uint32_t* pay0, uint32_t* pay1,
                       hipStream_t s, SortRange sr) {
    const uint32_t mask = (1u << bits) - 1u;
    if (sr.filter)
        hipLaunchKernelGGL((k_radix_upsweep<ITEMS, true>), dim3(groups), dim3(kSortThreads), 0, s, in, n_dev, n_host,
                           shift, mask, groups, hist, dstats, pass, sr);
    else
        hipLaunchKernelGGL((k_radix_upsweep<ITEMS, false>), dim3(groups), dim3(kSortThreads), 0, s, in, n_dev, n_host,
                           shift, mask, groups, hist, dstats, pass, sr);
    hipLaunchKernelGGL(k_radix_scan, dim3(256), dim3(256), 0, s, hist, groups, totals,
                       static_cast<const uint32_t*>(dstats), pass, sr.gate);
    // rect payloads (binning): pass p reads pay[p & 1] (pass 0: rect, or pay[0] when
    // rect_direct < 0 — the live partition wrote it) and writes pay[(p + 1) & 1]
    const uint32_t* pay_in = pay0 && (pass > 0 || rect_direct < 0) ? ((pass & 1) ? pay1 : pay0) : nullptr;
    uint32_t* pay_out = pay0 ? ((pass & 1) ? pay0 : pay1) : nullptr;
    if (sr.filter)
        hipLaunchKernelGGL((k_radix_downsweep<ITEMS, RA, true>), dim3(groups), dim3(kSortThreads), 0, s, in, out, n_dev,
                           n_host, shift, bits, groups, hist, totals, ranges, static_cast<const uint32_t*>(dstats), pass,
                           rect, rect_direct > 0 ? 1 : 0, pay_in, pay_out, sr);
    else
        hipLaunchKernelGGL((k_radix_downsweep<ITEMS, RA, false>), dim3(groups), dim3(kSortThreads), 0, s, in, out, n_dev,
                           n_host, shift, bits, groups, hist, totals, ranges, static_cast<const uint32_t*>(dstats), pass,
                           rect, rect_direct > 0 ? 1 : 0, pay_in, pay_out, sr);
}

hipError_t launch_radix_pass(const uint64_t* in, uint64_t* out, const uint32_t* n_dev, uint32_t n_host,
                             int shift, int bits, int groups, int items, uint32_t* hist, uint32_t* totals,
                             uint2* ranges, hipStream_t s, uint32_t* dstats, int pass, const uint32_t* rect,
                             int rect_direct, uint32_t* pay0, uint32_t* pay1, bool rank_atomic,
                             const uint32_t* base_dev, const uint32_t* gate, const SortFilter* f) {
    if ((rect == nullptr) != (pay0 == nullptr) || (pay0 == nullptr) != (pay1 == nullptr))
        return hipErrorInvalidValue;
    const int filter = f ? f->mode : 0;
    if (filter < 0 || filter > 2 || (filter && (pass != 0 || !f->kcut || n_dev || (filter == 2) != (base_dev != nullptr))))
        return hipErrorInvalidValue;
    if (base_dev && !filter && (n_dev || rect_direct > 0)) return hipErrorInvalidValue;
    if (filter && !carry_ok(pay0, rect_direct)) return hipErrorInvalidValue;
    const SortRange sr{base_dev, gate, filter ? f->kcut : nullptr, filter, filter ? f->count_out : nullptr,
                       filter == 1 ? f->kcut_copy : nullptr, filter == 2 ? f->sat : nullptr, f ? f->sat_w : 0,
                       filter == 2 && f->sat ? rect : nullptr, f && !filter ? f->count : nullptr};
    // 16 items per thread always rank with ballots, one tile per workgroup
    // (k_radix_downsweep): a grid too small for that sorts 8 per thread
    if (items == 16 && (uint64_t)groups * kSortTile < (uint64_t)n_host) items = 8;
    if (items == 4 && rank_atomic)
        radix_pass<4, true>(in, out, n_dev, n_host, shift, bits, groups, hist, totals, ranges, dstats, pass, rect,
                            rect_direct, pay0, pay1, s, sr);
    else if (items == 4)
        radix_pass<4, false>(in, out, n_dev, n_host, shift, bits, groups, hist, totals, ranges, dstats, pass, rect,
                             rect_direct, pay0, pay1, s, sr);
    else if (items == 8 && rank_atomic)
        radix_pass<8, true>(in, out, n_dev, n_host, shift, bits, groups, hist, totals, ranges, dstats, pass, rect,
                            rect_direct, pay0, pay1, s, sr);
    else if (items == 8)
        radix_pass<8, false>(in, out, n_dev, n_host, shift, bits, groups, hist, totals, ranges, dstats, pass, rect,
                             rect_direct, pay0, pay1, s, sr);
    else
        radix_pass<16, false>(in, out, n_dev, n_host, shift, bits, groups, hist, totals, ranges, dstats, pass, rect,
                              rect_direct, pay0, pay1, s, sr);
    return hipGetLastError();
}

template <int B>
static void bucket_sort_b(const uint64_t* in, uint64_t* items0, uint64_t* items1, uint32_t n, int groups,
                          const uint32_t* s_in, uint32_t* s_out, uint32_t* hist, uint32_t* totals,
                          const uint32_t* rect, uint32_t* pay0, uint32_t* pay1, bool rank_atomic, uint32_t cap,
                          unsigned int* over_host, hipStream_t s, int row_tiles_y, uint4* rec) {
    // fused row-pass count: the row hist overwrites the bucket hist, which only the scatter reads
    // (grid B with it: the last bucket is the row pass's last chunk, k_bkt_local)
    const RowHist rh{row_tiles_y > 0 ? hist : nullptr, B, row_tiles_y};
    const int local_grid = row_tiles_y > 0 ? B : B - 1;
    uint32_t* bstart = totals + B;   // B + 2 words after the totals
    constexpr int kScTh = B >= 512 ? 512 : kBktThreads;   // k_bkt_scatter's workgroup size
    // A/B: GSR_BKT_SCATTER_256=1 runs the 4,096-bucket scatter in 256-thread workgroups (64 KB of
    // LDS instead of 96: two workgroups per CU)
    static const bool sc256 = [] { const char* e = std::getenv("GSR_BKT_SCATTER_256"); return e && e[0] == '1'; }();
    // A/B: GSR_BKT_STAGE_SMALL=1 writes each scatter tile in bucket order here too
    static const bool stage = [] { const char* e = std::getenv("GSR_BKT_STAGE_SMALL"); return e && e[0] == '1'; }();
    // A/B: GSR_BKT_BID=1 hands each item's bucket from the count to the scatter (big buckets' scheme)
    static const bool bids = [] { const char* e = std::getenv("GSR_BKT_BID"); return e && e[0] == '1'; }();
    const bool bid_on = bids && !stage && !(B == 4096 && sc256);
    uint16_t* bid = bid_on ? reinterpret_cast<uint16_t*>(pay1) : nullptr;
    hipLaunchKernelGGL(k_bkt_count<B>, dim3(groups), dim3(kBktThreads), 0, s, in, n, s_in, groups, hist, bid);
    // A/B: GSR_BKT_SCANG=1 scans 16 buckets per workgroup over 64 chunk slices (the big buckets' scan)
    static const bool scang = [] { const char* e = std::getenv("GSR_BKT_SCANG"); return e && e[0] == '1'; }();
    if (scang)
        hipLaunchKernelGGL((k_bkt_scan_g<B, kBktMaxGroups>), dim3(B / 16), dim3(1024), 0, s, hist, groups, totals);
    else
        hipLaunchKernelGGL(k_bkt_scan<B>, dim3(B / 64), dim3(1024), 0, s, hist, groups, totals);
    if (stage) {
        auto run = [&](auto ra) {
            constexpr bool RA = decltype(ra)::value;
            hipLaunchKernelGGL((k_bkt_scatter<B, RA, kScTh, true>), dim3(groups), dim3(kScTh), 0, s, in, items0, n,
                               s_in, groups, hist, static_cast<const uint32_t*>(totals), rect, pay0, bstart, rec,
                               static_cast<const uint16_t*>(nullptr));
            hipLaunchKernelGGL((k_bkt_local<B, RA>), dim3(local_grid), dim3(kBktThreads), 0, s, items0, items1, pay0,
                               pay1, bstart, s_in, s_out, cap, over_host, rh, static_cast<const uint4*>(rec));
        };
        if (rank_atomic) run(std::true_type{});
        else run(std::false_type{});
        return;
    }
    if (B == 4096 && sc256) {
        if (rank_atomic)
            hipLaunchKernelGGL((k_bkt_scatter<B, true, kBktThreads>), dim3(groups), dim3(kBktThreads), 0, s, in, items0,
                               n, s_in, groups, hist, static_cast<const uint32_t*>(totals), rect, pay0, bstart, rec,
                               static_cast<const uint16_t*>(nullptr));
        else
            hipLaunchKernelGGL((k_bkt_scatter<B, false, kBktThreads>), dim3(groups), dim3(kBktThreads), 0, s, in, items0,
                               n, s_in, groups, hist, static_cast<const uint32_t*>(totals), rect, pay0, bstart, rec,
                               static_cast<const uint16_t*>(nullptr));
        if (rank_atomic)
            hipLaunchKernelGGL((k_bkt_local<B, true>), dim3(local_grid), dim3(kBktThreads), 0, s, items0, items1, pay0,
                               pay1, bstart, s_in, s_out, cap, over_host, rh, static_cast<const uint4*>(rec));
        else
            hipLaunchKernelGGL((k_bkt_local<B, false>), dim3(local_grid), dim3(kBktThreads), 0, s, items0, items1, pay0,
                               pay1, bstart, s_in, s_out, cap, over_host, rh, static_cast<const uint4*>(rec));
        return;
    }
    if (bid_on) {
        auto run = [&](auto ra) {
            constexpr bool RA = decltype(ra)::value;
            hipLaunchKernelGGL((k_bkt_scatter<B, RA, kScTh, false, kBktTile, 1, false, false, true>), dim3(groups),
                               dim3(kScTh), 0, s, in, items0, n, s_in, groups, hist,
                               static_cast<const uint32_t*>(totals), rect, pay0, bstart, rec,
                               static_cast<const uint16_t*>(bid));
            hipLaunchKernelGGL((k_bkt_local<B, RA>), dim3(local_grid), dim3(kBktThreads), 0, s, items0, items1, pay0,
                               pay1, bstart, s_in, s_out, cap, over_host, rh, static_cast<const uint4*>(rec));
        };
        if (rank_atomic) run(std::true_type{});
        else run(std::false_type{});
        return;
    }
    if (rank_atomic) {
        hipLaunchKernelGGL((k_bkt_scatter<B, true, kScTh>), dim3(groups), dim3(kScTh), 0, s, in, items0, n, s_in,
                           groups, hist, static_cast<const uint32_t*>(totals), rect, pay0, bstart, rec,
                               static_cast<const uint16_t*>(nullptr));
        hipLaunchKernelGGL((k_bkt_local<B, true>), dim3(local_grid), dim3(kBktThreads), 0, s, items0, items1, pay0,
                           pay1, bstart, s_in, s_out, cap, over_host, rh, static_cast<const uint4*>(rec));
    } else {
        hipLaunchKernelGGL((k_bkt_scatter<B, false, kScTh>), dim3(groups), dim3(kScTh), 0, s, in, items0, n, s_in,
                           groups, hist, static_cast<const uint32_t*>(totals), rect, pay0, bstart, rec,
                               static_cast<const uint16_t*>(nullptr));
        hipLaunchKernelGGL((k_bkt_local<B, false>), dim3(local_grid), dim3(kBktThreads), 0, s, items0, items1, pay0,
                           pay1, bstart, s_in, s_out, cap, over_host, rh, static_cast<const uint4*>(rec));
    }
}

hipError_t launch_bucket_sort(const uint64_t* in, uint64_t* items0, uint64_t* items1, uint32_t n, int buckets,
                              int groups, const uint32_t* s_in, uint32_t* s_out, uint32_t* hist, uint32_t* totals,
                              const uint32_t* rect, uint32_t* pay0, uint32_t* pay1, bool rank_atomic, uint32_t cap,
                              unsigned int* over_host, hipStream_t s, int row_tiles_y, uint4* rec) {
    if (groups < 1 || groups > kBktMaxGroups || (int64_t)groups * buckets > 256 * (int64_t)kMaxSortGroups || cap < 1 ||
        cap > kBktCap ||
        in == items0 || !rect || !pay0 || !pay1 || !rec)   // in may be items1: the scratch is used after the scatter
        return hipErrorInvalidValue;
    if (n == 0 || row_tiles_y > 256 || (int64_t)512 * buckets > 256 * (int64_t)kMaxSortGroups)
        return n == 0 ? hipSuccess : hipErrorInvalidValue;
    switch (buckets) {
    case 256: bucket_sort_b<256>(in, items0, items1, n, groups, s_in, s_out, hist, totals, rect, pay0, pay1, rank_atomic, cap, over_host, s, row_tiles_y, rec); break;
    case 512: bucket_sort_b<512>(in, items0, items1, n, groups, s_in, s_out, hist, totals, rect, pay0, pay1, rank_atomic, cap, over_host, s, row_tiles_y, rec); break;
    case 1024: bucket_sort_b<1024>(in, items0, items1, n, groups, s_in, s_out, hist, totals, rect, pay0, pay1, rank_atomic, cap, over_host, s, row_tiles_y, rec); break;
    case 2048: bucket_sort_b<2048>(in, items0, items1, n, groups, s_in, s_out, hist, totals, rect, pay0, pay1, rank_atomic, cap, over_host, s, row_tiles_y, rec); break;
    case 4096: bucket_sort_b<4096>(in, items0, items1, n, groups, s_in, s_out, hist, totals, rect, pay0, pay1, rank_atomic, cap, over_host, s, row_tiles_y, rec); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// B buckets, sorted by TH-thread workgroups (512 / 1,024 or 1,024 / 512).  The scatter's tile
// is staged (bucket runs written coalesced), barrier-lean (52.0 -> 50.2 us at config 3 orbit)
// and writes 12-B records (16-B: 51.7 -> 50.5 us); the eight-barrier tile, 16-B records and
// the unstaged scatter measured slower (profiles/r06k_big_buckets_c3_orbit.txt, DESIGN.md
// section 3).
template <int B, int TH>
static void bucket_sort_big_b(const uint64_t* in, uint64_t* items0, uint64_t* items1, uint32_t n, int groups,
                              const uint32_t* s_in, uint32_t* s_out, uint32_t* hist, uint32_t* totals,
                              const uint32_t* rect, uint32_t* pay0, uint32_t* pay1, bool rank_atomic, uint32_t cap,
                              unsigned int* over_host, hipStream_t s, uint4* rec) {
    uint32_t* bstart = totals + B;          // B + 2 words after the totals
    uint32_t* left = totals + 2 * B + 2;    // per bucket: k_bbk_local left it to k_bkt_local
    const RowHist none{nullptr, B, 0};
    // the count hands each item's bucket to the scatter (u16 in pay1, free until the second
    // launch), which then skips its own splitter search (GSR_BB_BID=0: it searches, A/B)
    static const bool bids = [] { const char* e = std::getenv("GSR_BB_BID"); return !e || e[0] != '0'; }();
    uint16_t* bid = bids ? reinterpret_cast<uint16_t*>(pay1) : nullptr;
    hipLaunchKernelGGL(k_bkt_count<B>, dim3(groups), dim3(kBktThreads), 0, s, in, n, s_in, groups, hist, bid);
    // chunk scan: 16 buckets per workgroup over 64 chunk slices (5.9 vs 8.5 us for a wave per
    // bucket at config 3, profiles/r06sg_kt_big_bucket_scan.txt); GSR_BB_SCANG=0 for the latter
    static const bool scang = [] { const char* e = std::getenv("GSR_BB_SCANG"); return !e || e[0] != '0'; }();
    if (scang)
        hipLaunchKernelGGL((k_bkt_scan_g<B, kBigBucketGroups>), dim3(B / 16), dim3(1024), 0, s, hist, groups, totals);
    else
        hipLaunchKernelGGL((k_bkt_scan_w<B, kBigBucketGroups>), dim3(B / 4), dim3(256), 0, s, hist, groups, totals);
    auto run = [&](auto ra) {
        constexpr bool RA = decltype(ra)::value;
        if (bids)
            hipLaunchKernelGGL((k_bkt_scatter<B, RA, 512, true, kBktTile, 1, true, true, true>), dim3(groups), dim3(512),
                               0, s, in, items0, n, s_in, groups, hist, static_cast<const uint32_t*>(totals), rect,
                               pay0, bstart, rec, static_cast<const uint16_t*>(bid));
        else
            hipLaunchKernelGGL((k_bkt_scatter<B, RA, 512, true, kBktTile, 1, true, true>), dim3(groups), dim3(512), 0,
                               s, in, items0, n, s_in, groups, hist, static_cast<const uint32_t*>(totals), rect, pay0,
                               bstart, rec, static_cast<const uint16_t*>(nullptr));
        hipLaunchKernelGGL((k_bbk_local<B, RA, true, TH>), dim3(B - 1), dim3(TH), 0, s, items0, pay0,
                           static_cast<const uint32_t*>(bstart), s_in, s_out, cap, static_cast<const uint4*>(rec), left);
        hipLaunchKernelGGL((k_bkt_local<B, RA, true>), dim3(B - 1), dim3(kBktThreads), 0, s, items0, items1, pay0,
                           pay1, bstart, s_in, s_out, min(cap, kBktCap), over_host, none,
                           static_cast<const uint4*>(rec), static_cast<const uint32_t*>(left));
    };
    if (rank_atomic) run(std::true_type{});
    else run(std::false_type{});
}

hipError_t launch_bucket_sort_big(const uint64_t* in, uint64_t* items0, uint64_t* items1, uint32_t n, int buckets,
                                  int groups, const uint32_t* s_in, uint32_t* s_out, uint32_t* hist, uint32_t* totals,
                                  const uint32_t* rect, uint32_t* pay0, uint32_t* pay1, bool rank_atomic, uint32_t cap,
                                  unsigned int* over_host, hipStream_t s, uint4* rec) {
    if ((buckets != 512 && buckets != 1024) || groups < 1 || groups > kBigBucketGroups ||
        (int64_t)groups * buckets > 256 * (int64_t)kMaxSortGroups || cap < 1 || in == items0 || !rect || !pay0 ||
        !pay1 || !rec)
        return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    if (buckets == 512)
        bucket_sort_big_b<512, 1024>(in, items0, items1, n, groups, s_in, s_out, hist, totals, rect, pay0, pay1,
                                     rank_atomic, cap, over_host, s, rec);
    else
        bucket_sort_big_b<1024, 512>(in, items0, items1, n, groups, s_in, s_out, hist, totals, rect, pay0, pay1,
                                     rank_atomic, cap, over_host, s, rec);
    return hipGetLastError();
}

hipError_t launch_bkt_splitters(const uint64_t* items0, const uint64_t* items1, const uint32_t* dstats, uint32_t n,
                                const uint32_t* live_dev, int buckets, uint32_t* s_out, hipStream_t s) {
    switch (buckets) {
    case 256: hipLaunchKernelGGL(k_bkt_splitters<256>, dim3(1), dim3(kBktThreads), 0, s, items0, items1, dstats, n, live_dev, s_out); break;
    case 512: hipLaunchKernelGGL(k_bkt_splitters<512>, dim3(1), dim3(kBktThreads), 0, s, items0, items1, dstats, n, live_dev, s_out); break;
    case 1024: hipLaunchKernelGGL(k_bkt_splitters<1024>, dim3(1), dim3(kBktThreads), 0, s, items0, items1, dstats, n, live_dev, s_out); break;
    case 2048: hipLaunchKernelGGL(k_bkt_splitters<2048>, dim3(1), dim3(kBktThreads), 0, s, items0, items1, dstats, n, live_dev, s_out); break;
    case 4096: hipLaunchKernelGGL(k_bkt_splitters<4096>, dim3(1), dim3(kBktThreads), 0, s, items0, items1, dstats, n, live_dev, s_out); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_emit(const uint64_t* items0, const uint64_t* items1, const uint32_t* dstats, uint32_t n,
                       const uint64_t* rect, int groups, unsigned long long* wg_scratch, Stats* stats,
                       Stats* host_mapped_stats, uint32_t pair_capacity, int tiles_x, int tiles_y, void* keys,
                       bool key16, uint32_t* vals, uint2* ranges, hipStream_t s, uint32_t* fstatus) {
    hipLaunchKernelGGL(k_emit_count, dim3(groups), dim3(256), 0, s, items0, items1, dstats, n, rect, groups,
                       wg_scratch, ranges, tiles_x * tiles_y);
    hipLaunchKernelGGL(k_emit_scan, dim3(1), dim3(256), 0, s, wg_scratch, groups, pair_capacity, stats,
                       host_mapped_stats, fstatus);
    if (key16)
        hipLaunchKernelGGL(k_emit_pairs<uint16_t>, dim3(groups), dim3(256), 0, s, items0, items1, dstats, n, groups,
                           wg_scratch, pair_capacity, tiles_x, static_cast<uint16_t*>(keys), vals);
    else
        hipLaunchKernelGGL(k_emit_pairs<uint32_t>, dim3(groups), dim3(256), 0, s, items0, items1, dstats, n, groups,
                           wg_scratch, pair_capacity, tiles_x, static_cast<uint32_t*>(keys), vals);
    return hipGetLastError();
}

hipError_t launch_partition(const uint64_t* in, uint32_t n, int groups, uint32_t* counts, uint32_t* n_live,
                            uint64_t* out, const uint32_t* rect, uint32_t* pay0, uint32_t* pay1, hipStream_t s) {
    if (groups < 1 || groups > kMaxSortGroups) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_part_count, dim3(groups), dim3(256), 0, s, in, n, groups, counts);
    hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(256), 0, s, counts, groups, n_live);
    hipLaunchKernelGGL(k_part_scatter, dim3(groups), dim3(256), 0, s, in, n, groups, counts, n_live, out, rect,
                       pay0, pay1);
    return hipGetLastError();
}

hipError_t launch_bin_rows(const uint64_t* items0, const uint64_t* items1, const uint32_t* dstats, uint32_t n,
                           const uint32_t* pay0, const uint32_t* pay1, int groups, uint32_t* hist,
                           uint32_t* row_items,
                           unsigned long long* row_pairs, uint32_t pair_capacity, int tiles_y, uint64_t* rows_buf,
                           int items, hipStream_t s, const uint16_t* spans, bool rank_atomic, uint32_t base,
                           uint32_t* gate, int gate_mode, const uint32_t* cut, const RowSplit* rs,
                           const uint32_t* cstart) {
    const int cut_mode = rs ? rs->cut_mode : 0;
    if (tiles_y < 1 || tiles_y > 256 || groups < 1 || groups > kMaxSortGroups / 2 ||
        (items != 4 && items != 8 && items != 16) || (gate_mode != 0 && !gate) || gate_mode < 0 || gate_mode > 2 ||
        (cut_mode != 0 && !cut) || cut_mode < 0 || cut_mode > 2)
        return hipErrorInvalidValue;
    const uint32_t* g = gate_mode == 2 ? gate : nullptr;
    const uint32_t* cut_n = rs ? rs->cut_n : nullptr;
    if (cstart && (cut_mode != 0 || gate_mode != 0 || base != 0)) return hipErrorInvalidValue;
    if (!cstart)   // with bucket chunks the bucket sort's local kernel wrote the counts
        hipLaunchKernelGGL(k_bin_rows_count, dim3(groups), dim3(256), 0, s, n, pay0, pay1, dstats, groups, tiles_y,
                           hist, base, g, cut, cut_mode, cut_n);
    hipLaunchKernelGGL(k_bin_rows_scan, dim3(256), dim3(256), 0, s, hist, groups, tiles_y, row_items, row_pairs,
                       gate, gate_mode);
    auto pick = [&](auto ra) {
        constexpr bool RA = decltype(ra)::value;
        return tiles_y <= 128 ? (items == 4 ? k_bin_rows_scatter<4, 7, RA> : items == 8 ? k_bin_rows_scatter<8, 7, RA>
                                                                                     : k_bin_rows_scatter<16, 7, RA>)
                              : (items == 4 ? k_bin_rows_scatter<4, 8, RA> : items == 8 ? k_bin_rows_scatter<8, 8, RA>
                                                                                     : k_bin_rows_scatter<16, 8, RA>);
    };
    auto scatter = rank_atomic ? pick(std::true_type{}) : pick(std::false_type{});
    hipLaunchKernelGGL(scatter, dim3(groups), dim3(256), 0, s, items0, items1, dstats, pay0, pay1, n, groups, hist,
                       row_items, row_pairs, pair_capacity, tiles_y, rows_buf, spans, base, g, cut, cut_mode, cut_n,
                       cstart);
    return hipGetLastError();
}

hipError_t launch_bin_cols(const uint64_t* rows_buf, const uint32_t* row_items, const unsigned long long* row_pairs,
                           uint32_t* cbins, int col_groups, uint32_t pair_capacity, int tiles_x, int tiles_y,
                           uint32_t* vals, uint2* ranges, Stats* stats, Stats* host_mapped_stats, int items,
                           hipStream_t s, const uint32_t* dstats, int passes_launched, bool rank_atomic,
                           const uint32_t* gate, uint32_t* fstatus, int chunk) {
    if (tiles_x < 1 || tiles_x > 256 || tiles_y < 1 || tiles_y > 256 || col_groups < 1 ||
        (items != 4 && items != 8 && items != 16) || (chunk != (int)kColChunkMin && chunk != (int)kColChunkMax))
        return hipErrorInvalidValue;
    auto run = [&](auto ch) {
        constexpr uint32_t CH = decltype(ch)::value;
        hipLaunchKernelGGL(k_bin_cols_count<CH>, dim3(col_groups), dim3(256), 0, s, rows_buf, row_items, row_pairs,
                           pair_capacity, tiles_x, cbins, gate);
        hipLaunchKernelGGL(k_bin_cols_scan<CH>, dim3(tiles_y), dim3(256), 0, s, row_items, row_pairs, pair_capacity,
                           tiles_x, cbins, ranges, stats, host_mapped_stats, dstats, passes_launched, gate, fstatus);
        auto pick = [&](auto ra) {
            constexpr bool RA = decltype(ra)::value;
            return tiles_x <= 128
                       ? (items == 4   ? k_bin_cols_scatter<4, 7, RA, CH>
                          : items == 8 ? k_bin_cols_scatter<8, 7, RA, CH>
                                       : k_bin_cols_scatter<16, 7, RA, CH>)
                       : (items == 4   ? k_bin_cols_scatter<4, 8, RA, CH>
                          : items == 8 ? k_bin_cols_scatter<8, 8, RA, CH>
                                       : k_bin_cols_scatter<16, 8, RA, CH>);
        };
        auto scatter = rank_atomic ? pick(std::true_type{}) : pick(std::false_type{});
        hipLaunchKernelGGL(scatter, dim3(col_groups), dim3(256), 0, s, rows_buf, row_items, row_pairs, pair_capacity,
                           tiles_x, cbins, ranges, vals, gate);
    };
    if (chunk == (int)kColChunkMin)
        run(std::integral_constant<uint32_t, kColChunkMin>{});
    else
        run(std::integral_constant<uint32_t, kColChunkMax>{});
    return hipGetLastError();
}

// cbins rows for either chunk size: a row's chunks <= its items / chunk + 1, and every row
// item holds at least one pair
uint32_t bin_col_chunks_max(uint32_t pair_capacity, int tiles_y) {
    return pair_capacity / kColChunkMin + (uint32_t)tiles_y + 1u;
}

template <typename K, int ITEMS>
static void kv_pass(const K* kin, const uint32_t* vin, K* kout, uint32_t* vout, const uint32_t* n_dev, int shift,
                    int bits, int groups, uint32_t* hist, uint32_t* totals, uint2* ranges, hipStream_t s) {
    const uint32_t mask = (1u << bits) - 1u;
    hipLaunchKernelGGL((k_kv_upsweep<K, ITEMS>), dim3(groups), dim3(kSortThreads), 0, s, kin, n_dev, shift, mask,
                       groups, hist);
    hipLaunchKernelGGL(k_radix_scan, dim3(256), dim3(256), 0, s, hist, groups, totals,
                       static_cast<const uint32_t*>(nullptr), 0, static_cast<const uint32_t*>(nullptr));
    hipLaunchKernelGGL((k_kv_downsweep<K, ITEMS>), dim3(groups), dim3(kSortThreads), 0, s, kin, vin, kout, vout,
                       n_dev, shift, bits, groups, hist, totals, ranges);
}

hipError_t launch_kv_pass(const void* keys_in, const uint32_t* vals_in, void* keys_out, uint32_t* vals_out,
                          bool key16, const uint32_t* n_dev, int shift, int bits, int groups, int items,
                          uint32_t* hist, uint32_t* totals, uint2* ranges, hipStream_t s) {
    using u16 = uint16_t;
    using u32 = uint32_t;
    const auto* k16 = static_cast<const u16*>(keys_in);
    const auto* k32 = static_cast<const u32*>(keys_in);
    auto* o16 = static_cast<u16*>(keys_out);
    auto* o32 = static_cast<u32*>(keys_out);
    if (key16 && items == 8)
        kv_pass<u16, 8>(k16, vals_in, o16, vals_out, n_dev, shift, bits, groups, hist, totals, ranges, s);
    else if (key16)
        kv_pass<u16, 16>(k16, vals_in, o16, vals_out, n_dev, shift, bits, groups, hist, totals, ranges, s);
    else if (items == 8)
        kv_pass<u32, 8>(k32, vals_in, o32, vals_out, n_dev, shift, bits, groups, hist, totals, ranges, s);
    else
        kv_pass<u32, 16>(k32, vals_in, o32, vals_out, n_dev, shift, bits, groups, hist, totals, ranges, s);
    return hipGetLastError();
}

hipError_t launch_blend(const uint32_t* idx, const uint2* ranges, const uint4* rec, const Frame& fr,
                        float* out, unsigned long long* consumed, bool stamps, int band_tiles, int blend_exp,
                        hipStream_t s, const BlendSplit* split) {
    // blend_exp 2 (test hook): the fast blend with a band of 100 %, so every block in
    // which a pixel saturates (or ends below 2e-3) is blended again exactly
    const bool fast_exp = blend_exp != 0;
    const float band0 = blend_exp == 2 ? 1.0f : kFxBand0;
    const int nt = fr.tiles_x * fr.tiles_y;
    if (nt <= 0) return hipSuccess;
    // bands of band_tiles tiles (4 blocks each) dealt round-robin to the 8 XCDs; the
    // grid is padded to whole rounds of bands.  Images too small for two rounds:
    // one contiguous run per XCD.
    int bands = 1, ng = 4 * nt;
    if (band_tiles > 0 && (nt + 8 * band_tiles - 1) / (8 * band_tiles) > 1) {
        bands = (nt + 8 * band_tiles - 1) / (8 * band_tiles);          // bands per XCD
        ng = 8 * bands * ((4 * nt + 8 * bands - 1) / (8 * bands));
    }
    const int phase = split ? split->phase : 0;
    if (phase < 0 || phase > 2 || (phase && (fast_exp || stamps || !split->tbuf || !split->bflag || !split->gate)))
        return hipErrorInvalidValue;
    const BlendSplit sp = split ? *split : BlendSplit{0, nullptr, nullptr, nullptr, nullptr, nullptr, {}, 0u, nullptr};
#define GSR_BLEND_S(D, ST, FX, SP)                                                                          \
    hipLaunchKernelGGL((k_blend_w<D, ST, FX, SP>), dim3(ng), dim3(64), 0, s, idx, ranges, rec, fr.tiles_x,  \
                       fr.tiles_y, fr.W, fr.H, fr.cover_w, fr.cover_h, out, consumed, bands, band0, sp)
#define GSR_BLEND(D, ST, FX) GSR_BLEND_S(D, ST, FX, 0)
    if (phase) {
        if (consumed) {
            if (phase == 1) GSR_BLEND_S(true, false, false, 1);
            else GSR_BLEND_S(true, false, false, 2);
        } else {
            if (phase == 1) GSR_BLEND_S(false, false, false, 1);
            else GSR_BLEND_S(false, false, false, 2);
        }
    } else if (stamps && consumed) {
        if (fast_exp) GSR_BLEND(false, true, true);
        else GSR_BLEND(false, true, false);
    } else if (consumed) {
        if (fast_exp) GSR_BLEND(true, false, true);
        else GSR_BLEND(true, false, false);
    } else {
        if (fast_exp) GSR_BLEND(false, false, true);
        else GSR_BLEND(false, false, false);
    }
#undef GSR_BLEND
#undef GSR_BLEND_S
    return hipGetLastError();
}

hipError_t launch_split_sat(const uint8_t* bflag, int tiles_x, int tiles_y, uint32_t* sat, const uint32_t* gate,
                            hipStream_t s) {
    if (tiles_x < 1 || tiles_x > 256 || tiles_y < 1 || tiles_y > 256 || !gate) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_split_sat, dim3(1), dim3(256), 0, s, bflag, tiles_x, tiles_y, sat, gate);
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

hipError_t rank_order_check(unsigned long long* lane_ops, unsigned long long* mismatches) {
    unsigned long long* d = nullptr;
    unsigned long long h[2] = {0, 0};
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&d), sizeof h);
    if (e != hipSuccess) return e;
    e = hipMemset(d, 0, sizeof h);
    // 1,024 workgroups (4 per CU) x 24 patterns x 8 iterations: ~44M lane-operations, well under 1 ms
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_rank_order_check, dim3(1024), dim3(256), 0, nullptr, 0x9E3779B9u, 8, d);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    *lane_ops = h[0];
    *mismatches = h[1];
    return e;
}

hipError_t launch_math_probe(const float* in, int n, float* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_math_probe, dim3(grid_for(n, 256)), dim3(256), 0, s, in, n, out);
    return hipGetLastError();
}

hipError_t launch_exp_probe(uint32_t key_lo, uint32_t key_hi, float x_big, unsigned long long* viol, uint32_t* errs,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_exp_probe, dim3(8192), dim3(256), 0, s, key_lo, key_hi, x_big, viol, errs);
    return hipGetLastError();
}

hipError_t launch_xs_probe(const float* op, int n, float* out, hipStream_t s) {
    if (n > 0) hipLaunchKernelGGL(k_xs_probe, dim3(grid_for(n, 256)), dim3(256), 0, s, op, n, out);
    return hipGetLastError();
}

}  // namespace gsr
