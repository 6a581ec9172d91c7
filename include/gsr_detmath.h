/*
 * gsr_detmath.h — deterministic single-precision elementary functions, compiled
 * IDENTICALLY for the gfx950 kernels (hipcc) and for host code (gcc / clang).
 *
 * Why this exists
 * ---------------
 * The reference renderer (src/core/cuda/render.cu) calls CUDA's libdevice
 * `expf` (render.cu:333, per pixel-splat), `atan2f` (render.cu:719), `cosf`/
 * `sinf` (render.cu:724-725) and `tanf` (render.cu:620).  Their results feed
 * integer quantisers (floorf/ceilf of the AABB, render.cu:748-751) and the
 * alpha / transmittance thresholds of the blend (render.cu:328,335), so a
 * one-ulp difference between the GPU and the CPU oracle can move a pixel by
 * ~1e-3 — ten times the 1e-4 L-inf parity gate.  Both sides therefore use the
 * functions below, which are built only from IEEE-exact primitives
 * (+ - * / with round-to-nearest, fmaf, rintf, fabsf, bit casts) and so give
 * bit-identical results on x86-64 SSE and on CDNA4 VALU, provided the
 * translation unit is compiled with -ffp-contract=off (no implicit FMA) and
 * without fast-math.
 *
 * Accuracy (checked by tests/test_detmath.py against double precision over
 * dense sweeps): expf <= 2 ulp, sin/cos <= 2 ulp on |x| <= pi, atan2f <= 3 ulp,
 * i.e. within the error bounds CUDA documents for the libdevice functions the
 * reference calls (CUDA C Programming Guide, "Mathematical Functions":
 * expf 2 ulp, sinf/cosf 2 ulp, atan2f 3 ulp).  The polynomial coefficients are
 * the published Cephes single-precision minimax sets (S. Moshier), evaluated
 * here with explicit fmaf Horner steps.
 *
 * tanf is NOT restated here: fx/fy (render.cu:620-621) are computed once per
 * frame on the host as a correctly rounded float tan (see gsr_camera_intrinsics
 * in gsr_runtime.cpp) and passed to the kernels, so both sides share them.
 */
#ifndef GSR_DETMATH_H
#define GSR_DETMATH_H

#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define GSR_HD __host__ __device__ __forceinline__
#else
#define GSR_HD static inline
#endif

GSR_HD float gsr_bits_to_float(uint32_t u) {
    union { uint32_t u; float f; } c;
    c.u = u;
    return c.f;
}

GSR_HD uint32_t gsr_float_to_bits(float f) {
    union { uint32_t u; float f; } c;
    c.f = f;
    return c.u;
}

/* float -> int32 with CUDA cvt.rzi.s32.f32 semantics (truncate, saturate,
 * NaN -> 0).  The reference casts with static_cast<int> (render.cu:748-754),
 * which on the GPU saturates; C leaves out-of-range casts undefined, so both
 * sides spell the saturation out. */
GSR_HD int32_t gsr_f2i_sat(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return (-2147483647 - 1);
    return (int32_t)f;
}

/* float -> uint32 with cvt.rzi.u32.f32 semantics: the depth key
 * static_cast<uint32_t>(-Z * 1e6f) (render.cu:850). */
GSR_HD uint32_t gsr_f2u_sat(float f) {
    if (!(f > 0.0f)) return 0u;                 /* NaN, zero, negative */
    if (f >= 4294967296.0f) return 0xffffffffu;
    return (uint32_t)f;
}

/* 2^e as a float for e in [-126, 127] (normal range), built from bits. */
GSR_HD float gsr_pow2i(int e) {
    return gsr_bits_to_float((uint32_t)(e + 127) << 23);
}

/*
 * expf(x): Cody-Waite reduction x = n*ln2 + r, |r| <= ln2/2, then
 * e^r = 1 + r + r^2 * P(r) (Cephes expf coefficients), scaled by 2^n as two
 * exact power-of-two multiplies so the whole finite range (including
 * subnormal results) is covered with IEEE rounding only.
 */
GSR_HD float gsr_expf(float x) {
    /* Branch-free: evaluate on x clamped into [-104, 88.75].  The clamp alone
     * yields the right special results: 2^-150 * e^(-104 + 150 ln2) rounds to
     * +0 for every x <= -104, and 2^128 * e^(88.75 - 128 ln2) overflows to +inf
     * for every x >= 88.75 (ln FLT_MAX = 88.7228); only NaN needs a select. */
    const float xc = fminf(fmaxf(x, -104.0f), 88.75f);   /* NaN -> -104 (replaced below) */
    const float t = xc * 1.44269504088896341f;            /* log2(e) */
    const float n = rintf(t);
    float r = __builtin_fmaf(-n, 0.693359375f, xc);       /* ln2 hi part (exact product) */
    r = __builtin_fmaf(-n, -2.12194440e-4f, r);           /* ln2 lo part */
    float p = 1.9875691500e-4f;
    p = __builtin_fmaf(p, r, 1.3981999507e-3f);
    p = __builtin_fmaf(p, r, 8.3334519073e-3f);
    p = __builtin_fmaf(p, r, 4.1665795894e-2f);
    p = __builtin_fmaf(p, r, 1.6666665459e-1f);
    p = __builtin_fmaf(p, r, 5.0000001201e-1f);
    const float r2 = r * r;
    const float y = __builtin_fmaf(p, r2, r) + 1.0f;
    const int ni = (int)n;                                /* n in [-150, 128] */
#if defined(__HIP_DEVICE_COMPILE__)
    /* v_ldexp_f32: one correctly rounded y * 2^ni — the same value as the two
     * multiplies below (y * 2^e1 is exact and normal, so the second product
     * is the only rounding); gfx950 keeps f32 denormals. */
    const float res = __builtin_amdgcn_ldexpf(y, ni);
#else
    const int e1 = ni / 2;
    const int e2 = ni - e1;
    const float res = (y * gsr_pow2i(e1)) * gsr_pow2i(e2);
#endif
    return (x != x) ? x + x : res;                        /* NaN */
}

/*
 * The blend's expf (render.cu:333, one per pixel-splat pair: the renderer's hottest
 * function).  Same domain handling as gsr_expf (clamp to [-104, 88.75], NaN kept) and
 * the same accuracy class (<= 1.006 ulp against exp over every float, 0.9991 ulp on
 * [-7, 0], monotone non-decreasing on every float: tests/test_detmath.py sweeps it
 * exhaustively), but two instructions cheaper per packed pair on gfx950:
 *   - n = rint(x log2 e) by the 1.5 * 2^23 shifter inside one fma (the rounding of the
 *     exact product, ties to even) instead of a product and two v_rndne_f32;
 *   - a degree-6 minimax e^r = 1 + r + r^2 Q(r) on |r| <= ln2/2 (Q of degree 4, fitted
 *     for relative error 5.5e-9 with float coefficients) instead of Cephes' degree 7.
 * The reference's own expf is CUDA libdevice's, which cannot run here; gsr_expf was
 * the previous stand-in.  Against it this one differs on 0.24 % of all floats, by
 * one ulp; the rendered effect is measured in profiles/r04_blend_exp_parity.txt.
 */
GSR_HD float gsr_blend_expf(float x) {
    const float xc = fminf(fmaxf(x, -104.0f), 88.75f);   /* NaN -> -104 (replaced below) */
    const float t = __builtin_fmaf(xc, 1.44269504088896341f, 12582912.0f);
    const float n = t - 12582912.0f;                      /* rint(xc log2 e), exact */
    float r = __builtin_fmaf(-n, 0.693359375f, xc);
    r = __builtin_fmaf(-n, -2.12194440e-4f, r);
    float q = 0x1.6b42a4p-10f;                            /* 1.38572813e-3 */
    q = __builtin_fmaf(q, r, 0x1.125e6cp-7f);              /* 8.37307237e-3 */
    q = __builtin_fmaf(q, r, 0x1.5557c2p-5f);              /* 4.16678227e-2 */
    q = __builtin_fmaf(q, r, 0x1.555452p-3f);              /* 1.66664734e-1 */
    q = __builtin_fmaf(q, r, 0x1.fffffcp-2f);              /* 4.99999940e-1 */
    const float r2 = r * r;
    const float y = __builtin_fmaf(q, r2, r) + 1.0f;
    const int ni = (int)n;                                /* n in [-150, 128] */
#if defined(__HIP_DEVICE_COMPILE__)
    const float res = __builtin_amdgcn_ldexpf(y, ni);
#else
    const int e1 = ni / 2;
    const int e2 = ni - e1;
    const float res = (y * gsr_pow2i(e1)) * gsr_pow2i(e2);
#endif
    return (x != x) ? x + x : res;
}

/* md2 of renderGaussians (render.cu:331),
 *   dx * (ic0 * dx + ic1 * dy) + dy * (ic2 * dx + ic3 * dy),
 * with the fused multiply-adds the reference's compiler forms: nvcc contracts
 * a * b + c into an FMA by default (--fmad=true) and, like LLVM's combiner, fuses
 * the product that is the sum's FIRST operand.  The blend's accumulation
 * rgb += color * alpha * T (render.cu:337) contracts the same way, to
 * fmaf(color * alpha, T, rgb).  Which product nvcc fuses cannot be observed here
 * (the CUDA path cannot be built); the oracle and the kernels make this one choice
 * together, so they agree bit for bit.  The other choices, measured against this one
 * (profiles/r04_contraction_parity.txt): within 8.7e-5 except the
 * second-product fusion, which moves one config-2 pixel by 1.6e-4. */
GSR_HD float gsr_blend_md2(float dx, float dy, float ic0, float ic1, float ic2, float ic3) {
    return __builtin_fmaf(dx, __builtin_fmaf(ic0, dx, ic1 * dy), dy * __builtin_fmaf(ic2, dx, ic3 * dy));
}

/* Total order of floats as unsigned keys (-inf < ... < -0 < +0 < ... < +inf). */
GSR_HD uint32_t gsr_float_key(float f) {
    const uint32_t b = gsr_float_to_bits(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
GSR_HD float gsr_key_float(uint32_t k) {
    return gsr_bits_to_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

/* The blend's alpha test (render.cu:333-335) as a predicate of the exp argument
 * x = -md2 / 2: is fminf(op * expf(x), 0.99f) >= 1e-3f? */
GSR_HD int gsr_alpha_taken(float op, float x) {
    return !(fminf(op * gsr_blend_expf(x), 0.99f) < 1e-3f);
}

/*
 * Smallest float x with gsr_alpha_taken(op, x): a splat is composited on a pixel
 * (alpha test passed) iff its exp argument -md2/2 >= this value, because
 * gsr_blend_expf is monotone non-decreasing on every float (checked exhaustively on
 * [-104, 88.75], tests/test_gpu_fastexp.py; constant outside) and so is the
 * rounded product op * y for op > 0.  NaN op: alpha = fminf(NaN, 0.99) passes for
 * every x (-inf); op <= 0 never passes (+inf); op = +inf always passes (-inf).
 * For finite op > 0 the answer lies in (-104, 88.75]: gsr_blend_expf(-104) = +0
 * fails and gsr_blend_expf(88.75) = +inf passes.  A few steps from the log estimate find it
 * (the estimate is within a few ulp), with bisection on the float order as the
 * bound.  Host and device give the same value: the estimate only picks where the
 * search starts.
 */
GSR_HD float gsr_alpha_take_min_x(float op) {
    if (op != op) return -INFINITY;
    if (!(op > 0.0f)) return INFINITY;
    if (op == INFINITY) return -INFINITY;
    uint32_t lo = gsr_float_key(-104.0f), hi = gsr_float_key(88.75f);   /* fails / passes */
#if defined(__HIP_DEVICE_COMPILE__)
    float e = __logf(1e-3f / op);
#else
    float e = logf(1e-3f / op);
#endif
    e = fminf(fmaxf(e, -103.0f), 88.0f);
    uint32_t k = gsr_float_key(e);
    for (int s = 0; s < 6 && hi - lo > 1u; s++) {
        if (gsr_alpha_taken(op, gsr_key_float(k))) {
            hi = k;
            k = k - 1u;
        } else {
            lo = k;
            k = k + 1u;
        }
        if (k <= lo || k >= hi) break;
    }
    while (hi - lo > 1u) {
        const uint32_t mid = lo + (hi - lo) / 2u;
        if (gsr_alpha_taken(op, gsr_key_float(mid))) hi = mid;
        else lo = mid;
    }
    return gsr_key_float(hi);
}

/* Polynomial cores on |r| <= pi/4 (Cephes sinf / cosf). */
GSR_HD float gsr_sin_core(float r) {
    const float z = r * r;
    float p = -1.9515295891e-4f;
    p = __builtin_fmaf(p, z, 8.3321608736e-3f);
    p = __builtin_fmaf(p, z, -1.6666654611e-1f);
    return __builtin_fmaf(p * z, r, r);
}

GSR_HD float gsr_cos_core(float r) {
    const float z = r * r;
    float p = 2.443315711809948e-5f;
    p = __builtin_fmaf(p, z, -1.388731625493765e-3f);
    p = __builtin_fmaf(p, z, 4.166664568298827e-2f);
    return __builtin_fmaf(p * z, z, __builtin_fmaf(-0.5f, z, 1.0f));
}

/* Quadrant reduction x = j*pi/2 + r with a three-part pi/2 (Cody-Waite).
 * Accurate for |x| up to ~1e4; the renderer only needs |x| <= pi/2
 * (theta = atan2/2, render.cu:719). Non-finite x gives NaN. */
GSR_HD float gsr_reduce_pio2(float x, int* quadrant) {
    const float j = rintf(x * 0.636619772367581343f);    /* 2/pi */
    float r = __builtin_fmaf(-j, 1.5703125f, x);
    r = __builtin_fmaf(-j, 4.837512969970703125e-4f, r);
    r = __builtin_fmaf(-j, 7.54978995489188216e-8f, r);
    *quadrant = ((int)j) & 3;
    return r;
}

GSR_HD float gsr_sinf(float x) {
    if (!(fabsf(x) < 16384.0f)) return (x - x) / (x - x) ;  /* NaN for inf/NaN/huge */
    int q;
    const float r = gsr_reduce_pio2(x, &q);
    const float s = gsr_sin_core(r);
    const float c = gsr_cos_core(r);
    return (q == 0) ? s : (q == 1) ? c : (q == 2) ? -s : -c;
}

GSR_HD float gsr_cosf(float x) {
    if (!(fabsf(x) < 16384.0f)) return (x - x) / (x - x);
    int q;
    const float r = gsr_reduce_pio2(x, &q);
    const float s = gsr_sin_core(r);
    const float c = gsr_cos_core(r);
    return (q == 0) ? c : (q == 1) ? -s : (q == 2) ? -c : s;
}

/* atan on t >= 0 (Cephes atanf range reduction + minimax polynomial). */
GSR_HD float gsr_atan_pos(float t) {
    float base = 0.0f, base_lo = 0.0f;        /* base = hi + lo (two-part pi/2, pi/4) */
    float u = t;
    if (t > 2.414213562373095f) {             /* tan(3pi/8) */
        base = 1.57079632679489662f;
        base_lo = -4.37113900018624283e-8f;
        u = -1.0f / t;
    } else if (t > 0.4142135623730950f) {     /* tan(pi/8) */
        base = 0.785398163397448310f;
        base_lo = -2.18556950009312141e-8f;
        u = (t - 1.0f) / (t + 1.0f);
    }
    const float z = u * u;
    float p = 8.05374449538e-2f;
    p = __builtin_fmaf(p, z, -1.38776856032e-1f);
    p = __builtin_fmaf(p, z, 1.99777106478e-1f);
    p = __builtin_fmaf(p, z, -3.33329491539e-1f);
    return base + (__builtin_fmaf(p * z, u, u) + base_lo);
}

/* atan2f(y, x) with the C99 Annex F special cases. */
GSR_HD float gsr_atan2f(float y, float x) {
    const float PI = 3.14159265358979323846f;
    const float PI_2 = 1.57079632679489662f;
    const float PI_4 = 0.785398163397448310f;
    const float PI_LO = -8.74227800037248566e-8f;               /* pi - (float)pi */
    if (x != x || y != y) return x + y;                        /* NaN */
    const int ysign = (gsr_float_to_bits(y) >> 31) != 0;
    const int xsign = (gsr_float_to_bits(x) >> 31) != 0;
    const float ay = fabsf(y);
    const float ax = fabsf(x);
    float res;
    if (ay == 0.0f) {
        res = xsign ? PI : 0.0f;                               /* atan2(+-0, x) */
    } else if (ax == 0.0f) {
        res = PI_2;
    } else if (ax == __builtin_inff() && ay == __builtin_inff()) {
        res = xsign ? 3.0f * PI_4 : PI_4;
    } else if (ax == __builtin_inff()) {
        res = xsign ? PI : 0.0f;
    } else if (ay == __builtin_inff()) {
        res = PI_2;
    } else {
        const float a = gsr_atan_pos(ay / ax);
        res = xsign ? ((PI - a) + PI_LO) : a;
    }
    return ysign ? -res : res;
}

#endif /* GSR_DETMATH_H */
