// Diagnostic (not product): exhaustive checks of cheaper sqrt / reciprocal / division
// sequences against the correctly rounded IEEE results the build uses today
// (__builtin_sqrtf and '/', which LLVM expands into the full correction sequences).
//
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o tools/fpexact tools/fpexact.hip
//   tools/fpexact            # all 2^31 non-negative floats for the unary functions,
//                            # 2^32 random pairs per range for the divisions
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../learnraytracing_amd/csrc/lrt_trace.h"   // the product's sqrt_rn / rcp_rn

__device__ __forceinline__ float sqrt_fix(float x) {   // v_sqrt + two-sided 1-ulp correction
    float s = __builtin_amdgcn_sqrtf(x);
    float sd = __int_as_float(__float_as_int(s) - 1);
    float su = __int_as_float(__float_as_int(s) + 1);
    float rd = __builtin_fmaf(-sd, s, x);
    float ru = __builtin_fmaf(-su, s, x);
    s = rd <= 0.0f ? sd : s;
    s = ru > 0.0f ? su : s;
    return s;
}
__device__ __forceinline__ float rcp_nr(float x) {   // v_rcp + one Newton step
    float r = __builtin_amdgcn_rcpf(x);
    float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ float div_mk(float a, float b) {   // Markstein: y = RN(1/b), q = a*y, one correction
    float y = rcp_nr(b);
    float q = a * y;
    float r = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(r, y, q);
}
__device__ __forceinline__ float div_mk2(float a, float b) {   // two corrections
    float y = rcp_nr(b);
    float q = a * y;
    float r = __builtin_fmaf(-b, q, a);
    q = __builtin_fmaf(r, y, q);
    r = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(r, y, q);
}

__device__ __forceinline__ float rcp_nr2(float x) {   // v_rcp + two Newton steps
    float r = __builtin_amdgcn_rcpf(x);
    float e = __builtin_fmaf(-x, r, 1.0f);
    r = __builtin_fmaf(e, r, r);
    e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ bool same(float a, float b) {
    return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}
// the product functions over every 32-bit pattern (signs, zeros, denormals, inf, NaN)
__global__ void prod_kernel(uint32_t base, unsigned long long* cnt) {
    const uint32_t u = base + blockIdx.x * blockDim.x + threadIdx.x;
    const float x = __uint_as_float(u);
    if (!same(lrt::sqrt_rn(x), __builtin_sqrtf(x))) atomicAdd(&cnt[0], 1ull);
    if (!same(lrt::rcp_rn(x), 1.0f / x)) atomicAdd(&cnt[1], 1ull);
    const uint32_t a = u & 0x7fffffffu;
    if (a >= 0x01000000u && a < 0x7f000000u && rcp_nr2(x) != 1.0f / x) atomicAdd(&cnt[2 + ((a >> 23) & 0xff)], 1ull);
}

// per biased exponent (0..255) mismatch counts for each unary test
enum { kSqrtRaw, kSqrtFix, kRcpRaw, kRcpNr, kSqrtRawLo, kSqrtRawHi, kNUnary };
__global__ void unary_kernel(uint32_t base, unsigned long long* cnt) {
    const uint32_t u = base + blockIdx.x * blockDim.x + threadIdx.x;   // non-negative floats only
    if (u >= 0x7f800000u) return;
    const float x = __uint_as_float(u);
    const int e = (int)(u >> 23);
    const float s_ref = __builtin_sqrtf(x);
    const float s_raw = __builtin_amdgcn_sqrtf(x);
    if (s_raw != s_ref) {
        atomicAdd(&cnt[kSqrtRaw * 256 + e], 1ull);
        if (s_raw < s_ref) atomicAdd(&cnt[kSqrtRawLo * 256 + e], 1ull);
        else atomicAdd(&cnt[kSqrtRawHi * 256 + e], 1ull);
    }
    if (sqrt_fix(x) != s_ref) atomicAdd(&cnt[kSqrtFix * 256 + e], 1ull);
    if (u != 0) {
        const float r_ref = 1.0f / x;
        if (__builtin_amdgcn_rcpf(x) != r_ref) atomicAdd(&cnt[kRcpRaw * 256 + e], 1ull);
        if (rcp_nr(x) != r_ref) atomicAdd(&cnt[kRcpNr * 256 + e], 1ull);
    }
}

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
// random (a, b) with exponents in [emin, emax], any mantissa, random signs
__global__ void div_kernel(uint32_t seed, int emin, int emax, unsigned long long* cnt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t h1 = hash(i * 2u + seed * 0x9E3779B9u), h2 = hash(i * 2u + 1u + seed * 0x85EBCA6Bu);
    const uint32_t h3 = hash(h1 ^ h2);
    const int span = emax - emin + 1;
    const uint32_t ea = (uint32_t)(emin + (int)(h3 % (uint32_t)span)) + 127u;
    const uint32_t eb = (uint32_t)(emin + (int)((h3 >> 16) % (uint32_t)span)) + 127u;
    const float a = __uint_as_float((h1 & 0x807fffffu) | (ea << 23));
    const float b = __uint_as_float((h2 & 0x807fffffu) | (eb << 23));
    const float ref = a / b;
    if (div_mk(a, b) != ref) atomicAdd(&cnt[0], 1ull);
    if (div_mk2(a, b) != ref) atomicAdd(&cnt[1], 1ull);
    if (a * rcp_nr(b) != ref) atomicAdd(&cnt[2], 1ull);
}

int main() {
    unsigned long long* d;
    const size_t n = kNUnary * 256 + 8;
    hipMalloc(&d, n * 8);
    hipMemset(d, 0, n * 8);
    for (uint64_t base = 0; base < 0x80000000ull; base += 1ull << 28)
        unary_kernel<<<(1u << 28) / 256, 256>>>((uint32_t)base, d);
    unsigned long long h[kNUnary * 256];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[kNUnary] = {"sqrt_raw", "sqrt_fix", "rcp_raw", "rcp_nr", "sqrt_raw<ref", "sqrt_raw>ref"};
    for (int k = 0; k < kNUnary; ++k) {
        unsigned long long tot = 0;
        int lo = -1, hi = -1;
        for (int e = 0; e < 256; ++e) {
            tot += h[k * 256 + e];
            if (h[k * 256 + e]) { if (lo < 0) lo = e; hi = e; }
        }
        printf("%-14s mismatches %12llu  (biased exponents %d..%d)\n", names[k], tot, lo, hi);
        for (int e = 0; e < 256; ++e)
            if (h[k * 256 + e] && (e < 40 || e > 215))
                printf("    e=%3d: %llu\n", e, h[k * 256 + e]);
    }
    {
        unsigned long long* c = d;
        hipMemset(c, 0, (2 + 256) * 8);
        for (uint64_t base = 0; base < 0x100000000ull; base += 1ull << 28)
            prod_kernel<<<(1u << 28) / 256, 256>>>((uint32_t)base, c);
        unsigned long long hc[2 + 256];
        hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        printf("product sqrt_rn vs sqrtf over all 2^32 patterns: %llu mismatches\n", hc[0]);
        printf("product rcp_rn vs 1/x over all 2^32 patterns: %llu mismatches\n", hc[1]);
        unsigned long long t = 0;
        int lo = -1, hi = -1;
        for (int e = 0; e < 256; ++e) if (hc[2 + e]) { t += hc[2 + e]; if (lo < 0) lo = e; hi = e; }
        printf("rcp_nr2 (|x| in [2^-126, 2^127)) mismatches %llu (biased exponents %d..%d)\n", t, lo, hi);
    }
    const int ranges[][2] = {{-20, 20}, {-60, 60}, {-1, 1}, {-126, 127}};
    for (auto& r : ranges) {
        unsigned long long* c = d + kNUnary * 256;
        hipMemset(c, 0, 64);
        for (uint32_t seed = 0; seed < 16; ++seed) div_kernel<<<(1u << 28) / 256, 256>>>(seed, r[0], r[1], c);
        unsigned long long hc[3];
        hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        printf("div exponents [%d, %d], 2^32 pairs: markstein1 %llu  markstein2 %llu  a*rcp_nr %llu mismatches\n",
               r[0], r[1], hc[0], hc[1], hc[2]);
    }
    hipFree(d);
    return 0;
}
