// Bit-exact restatement of the three libm functions the reference hot path calls
// (maths.cpp:37-38 cosf/sinf, parallel.cpp:116 cosf/sin(float), maths.h:126 powf).
//
// The reference delegates these to the C library. On the reference's platform here
// (Ubuntu 22.04, glibc 2.35, x86-64 with FMA: ifunc picks __sinf_fma/__cosf_fma/
// __powf_fma) glibc implements them with the published ARM optimized-routines
// algorithms (sincosf.h / powf.c, MIT/Apache-2.0):
//   sinf/cosf: y -> double; |y| < pi/4 direct polynomial, else x - n*pi/2 reduction
//              with n = ((int32)(x * 2^24*2/pi) + 2^23) >> 24, then an even (cos) or
//              odd (sin) polynomial in double, one final rounding to float.
//   powf:      log2(x) via a 16-entry (invc, logc) table + degree-5 polynomial in double,
//              y*log2(x), then exp2 via a 32-entry table + degree-3 polynomial.
// The FMA build contracts every a*b+c of those sources; the restatement below writes
// each contraction as an explicit fma(), and everything else as separate IEEE double
// operations, so host and device produce the glibc bits.
//
// Verified exhaustively against glibc 2.35 (tests/test_libm.py): sinf/cosf on every
// float of +/-[0, 120) (2.2e9 inputs, 0 mismatches), powf(x, 5) on every float of
// [0, 1] (1.07e9 inputs, 0 mismatches); the path only ever calls sinf/cosf on
// fl(kPI * k * 2^-23), k < 2^24, and powf on 1 - cosine with cosine in [0, 1].
//
// Table values are those of glibc 2.35's __sincosf_table, __powf_log2_data and
// __exp2f_data (identical to optimized-routines' sincosf_data.c, powf_log2_data.c,
// exp2f_data.c; Copyright (c) Arm Limited, MIT licence -- see THIRD_PARTY_NOTICES.md).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define LRT_HD __host__ __device__ __forceinline__
#else
#define LRT_HD static inline
#endif
// Tables: __constant__ in the device pass, plain static const in the host pass
// (each compilation pass sees exactly one definition).
#if defined(__HIP_DEVICE_COMPILE__)
#define LRT_CONST __constant__
#else
#define LRT_CONST static const
#endif

namespace lrt {
namespace libm {

LRT_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
LRT_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
LRT_HD uint64_t d2u(double d) { return __builtin_bit_cast(uint64_t, d); }
LRT_HD double u2d(uint64_t u) { return __builtin_bit_cast(double, u); }
LRT_HD int f2u_i(float f) { return __builtin_bit_cast(int, f); }
LRT_HD uint32_t abstop12(float x) { return (f2u(x) >> 20) & 0x7ff; }

// __sincosf_table[0] and [1] in glibc's field order {c0, c1, s1, c2, s2, c3, s3, c4};
// table [1] (used in quadrants 2 and 3) holds the negated cosine coefficients.
struct SinCosPoly { double c0, c1, s1, c2, s2, c3, s3, c4; };

LRT_HD SinCosPoly sincos_poly(int which) {
    SinCosPoly p;
    if (which == 0) {
        p.c0 = 0x1p0;                   p.c1 = -0x1.ffffffd0c621cp-2;
        p.s1 = -0x1.555545995a603p-3;   p.c2 = 0x1.55553e1068f19p-5;
        p.s2 = 0x1.1107605230bc4p-7;    p.c3 = -0x1.6c087e89a359dp-10;
        p.s3 = -0x1.994eb3774cf24p-13;  p.c4 = 0x1.99343027bf8c3p-16;
    } else {
        p.c0 = -0x1p0;                  p.c1 = 0x1.ffffffd0c621cp-2;
        p.s1 = -0x1.555545995a603p-3;   p.c2 = -0x1.55553e1068f19p-5;
        p.s2 = 0x1.1107605230bc4p-7;    p.c3 = 0x1.6c087e89a359dp-10;
        p.s3 = -0x1.994eb3774cf24p-13;  p.c4 = -0x1.99343027bf8c3p-16;
    }
    return p;
}

constexpr double kHpiInv = 0x1.45f306dc9c883p+23;  // 2/pi * 2^24
constexpr double kHpi = 0x1.921fb54442d18p+0;      // pi/2

// sinf_poly of sincosf.h with the FMA build's contractions.
LRT_HD float sinf_poly(double x, double x2, const SinCosPoly& p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = __builtin_fma(x2, p.s3, p.s2);
        double x7 = x3 * x2;
        double s = __builtin_fma(x3, p.s1, x);
        return (float)__builtin_fma(x7, s1, s);
    }
    double x4 = x2 * x2;
    double c2 = __builtin_fma(x2, p.c4, p.c3);
    double c1 = __builtin_fma(x2, p.c1, p.c0);
    double x6 = x4 * x2;
    double c = __builtin_fma(x4, p.c2, c1);
    return (float)__builtin_fma(x6, c2, c);
}

// reduce_fast of sincosf.h (no TOINT intrinsics on x86-64).
LRT_HD double reduce_fast(double x, int* np) {
    double r = x * kHpiInv;
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return __builtin_fma(-(double)n, kHpi, x);
}

// Valid for |y| < 120 (the only range the path uses: [0, 2*pi)).
LRT_HD float sinf(float y) {
    double x = y;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        if (abstop12(y) < abstop12(0x1p-12f)) return y;
        return sinf_poly(x, x * x, sincos_poly(0), 0);
    }
    int n;
    x = reduce_fast(x, &n);
    double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;   // sign[4] = {1,-1,-1,1}
    return sinf_poly(x * s, x * x, sincos_poly((n & 2) ? 1 : 0), n);
}

LRT_HD float cosf(float y) {
    double x = y;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
        return sinf_poly(x, x * x, sincos_poly(0), 1);
    }
    int n;
    x = reduce_fast(x, &n);
    double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
    return sinf_poly(x * s, x * x, sincos_poly((n & 2) ? 1 : 0), n ^ 1);
}

// sinf and cosf of the same argument with one shared reduction (glibc's sincosf computes
// both like this, and each result has the bits of the single call), in a branch-free form
// with the same double operations, so each result has the same bits:
//  * |y| < 0.75 (abstop12 below pi/4's: glibc's direct branch, table 0, n = 0) needs no
//    branch of its own: there reduce_fast gives n = 0 (|y| 2/pi 2^24 < 2^23) and
//    fma(-0, pi/2, x) = x, s = 1, table 0 -- the general path's very operations;
//  * table 1 is table 0 with the cosine coefficients negated and the sine ones equal, and
//    round-to-nearest is symmetric (fma(-a, b, -c) = -fma(a, b, c), (float)-d = -(float)d),
//    so its cosine polynomial is exactly the negated table-0 one: one evaluation, a sign;
//  * the sine and cosine polynomials are each evaluated once and swapped for odd n (glibc's
//    sinf_poly picks by n & 1), instead of both per output.
// Checked against glibc over the path's whole domain and beyond (tests/test_libm.py, kinds 6
// and 7) and on the device (tests/test_gpu_parity.py).
LRT_HD void sincosf(float y, float* sinp, float* cosp) {
    int n;
    const double x = reduce_fast((double)y, &n);
    const double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
    const SinCosPoly p = sincos_poly(0);
    const double xs = x * s, x2 = x * x;
    const float S = sinf_poly(xs, x2, p, 0);   // odd polynomial (sin coefficients: both tables)
    float C = sinf_poly(xs, x2, p, 1);         // even polynomial, table 0
    if (n & 2) C = -C;                         // table 1
    const bool odd = (n & 1) != 0;
    float sn = odd ? C : S, cs = odd ? S : C;
    if (abstop12(y) < abstop12(0x1p-12f)) {    // glibc's tiny-argument results
        sn = y;
        cs = 1.0f;
    }
    *sinp = sn;
    *cosp = cs;
}

// ---- powf: powf_log2_data.c (POWF_LOG2_TABLE_BITS 4, POWF_SCALE_BITS 0) ----
LRT_CONST double kPowLog2InvC[16] = {
    0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010b0p+0, 0x1.3c995b0b80385p+0,
    0x1.30d190c8864a5p+0, 0x1.25e227b0b8ea0p+0, 0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0,
    0x1.0953f419900a7p+0, 0x1.0p+0,               0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aa0p-1,
    0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1, 0x1.767dcf5534862p-1};
LRT_CONST double kPowLog2LogC[16] = {
    -0x1.efec65b963019p-2, -0x1.b0b6832d4fca4p-2, -0x1.7418b0a1fb77bp-2, -0x1.39de91a6dcf7bp-2,
    -0x1.01d9bf3f2b631p-2, -0x1.97c1d1b3b7af0p-3, -0x1.2f9e393af3c9fp-3, -0x1.960cbbf788d5cp-4,
    -0x1.a6f9db6475fcep-5, 0x0.0p+0,               0x1.338ca9f24f53dp-4, 0x1.476a9543891bap-3,
    0x1.e840b4ac4e4d2p-3, 0x1.40645f0c6651cp-2,  0x1.88e9c2c1b9ff8p-2, 0x1.ce0a44eb17bccp-2};
// exp2f_data.c (EXP2F_TABLE_BITS 5): tab[i] = bits(2^(i/32)) - (i << 47)
LRT_CONST uint64_t kExp2Tab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};

// The three powf tables, by pointer so a kernel can stage them in LDS (a per-lane table
// gather from global memory is a VMEM op; trace_kernel copies them to LDS).
struct PowTables {
    const double* invc;     // kPowLog2InvC
    const double* logc;     // kPowLog2LogC
    const uint64_t* exp2;   // kExp2Tab
};
LRT_HD PowTables pow_tables() {
    PowTables t;
    t.invc = kPowLog2InvC;
    t.logc = kPowLog2LogC;
    t.exp2 = kExp2Tab;
    return t;
}

LRT_HD double powf_log2_inline(uint32_t ix, const PowTables& T) {
    const double A0 = 0x1.27616c9496e0bp-2, A1 = -0x1.71969a075c67ap-2, A2 = 0x1.ec70a6ca7baddp-2,
                 A3 = -0x1.7154748bef6c8p-1, A4 = 0x1.71547652ab82bp+0;
    uint32_t tmp = ix - 0x3f330000u;
    int i = (int)((tmp >> 19) % 16);
    uint32_t top = tmp & 0xff800000u;
    uint32_t iz = ix - top;
    int k = (int32_t)top >> 23;
    double invc = T.invc[i];
    double logc = T.logc[i];
    double z = (double)u2f(iz);
    double r = __builtin_fma(z, invc, -1.0);
    double y0 = logc + (double)k;
    double r2 = r * r;
    double y = __builtin_fma(A0, r, A1);
    double p = __builtin_fma(A2, r, A3);
    double r4 = r2 * r2;
    double q = __builtin_fma(A4, r, y0);
    q = __builtin_fma(p, r2, q);
    y = __builtin_fma(y, r4, q);
    return y;
}

LRT_HD float powf_exp2_inline(double xd, uint32_t sign_bias, const PowTables& T) {
    const double C0 = 0x1.c6af84b912394p-5, C1 = 0x1.ebfce50fac4f3p-3, C2 = 0x1.62e42ff0c52d6p-1;
    const double kShift = 0x1.8p+47;   // 0x1.8p52 / 32
    double kd = xd + kShift;
    uint64_t ki = d2u(kd);
    kd -= kShift;
    double r = xd - kd;
    uint64_t t = T.exp2[ki % 32];
    uint64_t ski = ki + sign_bias;
    t += ski << (52 - 5);
    double s = u2d(t);
    double z = __builtin_fma(C0, r, C1);
    double r2 = r * r;
    double y = __builtin_fma(C2, r, 1.0);
    y = __builtin_fma(z, r2, y);
    y = y * s;
    return (float)y;
}

// checkint of powf.c: 0 = not an integer, 1 = odd integer, 2 = even integer.
LRT_HD int checkint(uint32_t iy) {
    int e = (int)(iy >> 23 & 0xff);
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}
LRT_HD bool zeroinfnan(uint32_t ix) { return 2u * ix - 1u >= 2u * 0x7f800000u - 1u; }

// powf(x, y) exactly as glibc 2.35's __powf (powf.c), signalling-NaN subtleties aside.
// The path calls it as powf(1 - cosine, 5) (maths.h:126) and the present step as
// powf(x, 0.416666667f) (main.cpp:112).
LRT_HD float powf(float x, float y, const PowTables& T) {
    const uint32_t kSignBias = 1u << (5 + 11);
    uint32_t sign_bias = 0;
    uint32_t ix = f2u(x), iy = f2u(y);
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u || zeroinfnan(iy)) {
        if (zeroinfnan(iy)) {
            if (2u * iy == 0) return 1.0f;
            if (ix == 0x3f800000u) return 1.0f;
            if (2u * ix > 2u * 0x7f800000u || 2u * iy > 2u * 0x7f800000u) return x + y;
            if (2u * ix == 2u * 0x3f800000u) return 1.0f;
            if ((2u * ix < 2u * 0x3f800000u) == !(iy & 0x80000000u)) return 0.0f;
            return y * y;
        }
        if (zeroinfnan(ix)) {
            float x2 = x * x;
            if ((ix & 0x80000000u) && checkint(iy) == 1) x2 = -x2;
            return (iy & 0x80000000u) ? 1.0f / x2 : x2;
        }
        if (ix & 0x80000000u) {
            int yint = checkint(iy);
            if (yint == 0) return (x - x) / (x - x);   // __math_invalidf
            if (yint == 1) sign_bias = kSignBias;
            ix &= 0x7fffffffu;
        }
        if (ix < 0x00800000u) {
            ix = f2u(u2f(ix) * 0x1p23f);
            ix &= 0x7fffffffu;
            ix -= 23u << 23;
        }
    }
    double logx = powf_log2_inline(ix, T);
    double ylogx = (double)y * logx;
    if (((d2u(ylogx) >> 47) & 0xffff) >= (d2u(126.0) >> 47)) {
        if (ylogx > 0x1.fffffffd1d571p+6) {   // __math_oflowf
            float o = 0x1p97f;
            return (sign_bias ? -o : o) * o;
        }
        if (ylogx <= -150.0) {                 // __math_uflowf
            float o = 0x1p-95f;
            return (sign_bias ? -o : o) * o;
        }
    }
    return powf_exp2_inline(ylogx, sign_bias, T);
}

LRT_HD float powf(float x, float y) { return powf(x, y, pow_tables()); }
// powf(x, 5) for the path's 1 - cosine (maths.h:126), with a fast path that returns glibc's
// bits without its log2/exp2 evaluation. For x in [2^-14, 1], x^5 in double (x*x exact, then two
// roundings: relative error < 2^-51.9) is so close to the true x^5 that the float both round to
// is certain unless the true value lies near a rounding boundary (a midpoint between floats):
// when the double lies farther than kPow5Gap (relative) from both midpoints around its float,
// that float is the correctly rounded x^5, and glibc's own double approximation rounds to it
// too. Otherwise -- and outside [2^-14, 1] -- glibc's algorithm (powf above). glibc is not
// correctly rounded: on 79,748 of the domain's 117,440,513 floats it returns the other
// neighbour, all with the double x^5 within 2^-33.06 (relative) of a midpoint; kPow5Gap = 2^-32
// keeps those (and 0.57 % of the domain in all) on glibc's algorithm. Checked on every float of
// [2^-14, 1] against glibc (tests/test_libm.py test_powf5_fast_path_domain, host and device): 0
// mismatches. (A timing-only build that took
// x^5 in float for every lane priced the exact powf at ~2 % of config 2, profiles/r6_ac.)
constexpr double kPow5Gap = 0x1p-32;
#ifdef LRT_EXP_POWF_TIMING   // timing-only builds (wrong bits): what the exact powf costs
LRT_HD float powf5(float x, const PowTables& T) { (void)T; const float x2 = x * x; return x2 * x2 * x; }
#else
LRT_HD float powf5(float x, const PowTables& T) {
    const uint32_t ix = f2u(x);
    if (ix - 0x38800000u <= 0x3f800000u - 0x38800000u) {   // x in [2^-14, 1]
        const double xd = x, x2 = xd * xd, x4 = x2 * x2, x5 = x4 * xd;
        const float r = (float)x5;
        const uint32_t ir = f2u(r);   // r is normal (>= 2^-70): its neighbours are ir -+ 1
        const double rd = r, lo = u2f(ir - 1u), hi = u2f(ir + 1u);
        const double mlo = 0.5 * (rd + lo), mhi = 0.5 * (rd + hi);   // exact in double
        const double gap = (x5 - mlo < mhi - x5 ? x5 - mlo : mhi - x5);
        if (gap > x5 * kPow5Gap) return r;
    }
    return powf(x, 5.0f, T);
}
#endif
LRT_HD float powf5(float x) { return powf(x, 5.0f, pow_tables()); }

}  // namespace libm
}  // namespace lrt
