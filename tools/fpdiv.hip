// Diagnostic (not product): the correctly rounded division a / b from the path's correctly
// rounded reciprocal y = rcp_rn(b) and one FMA correction (Markstein: q = RN(a y),
// r = a - b q exactly, RN(q + r y)), against the IEEE division LLVM expands '/' into.
//
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o tools/fpdiv tools/fpdiv.hip
//   tools/fpdiv
// Random pairs per exponent range (2^32 each), and every a of the path's ranges against the b the
// path divides by: the member normalize()'s lengths near 1 (maths.h:19; l.length() of a unit
// light sample), len * len near the light's distance squared, kPI.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../learnraytracing_amd/csrc/lrt_trace.h"   // the product's rcp_rn

__device__ __forceinline__ float div_rn(float a, float b) {
    const float y = lrt::rcp_rn(b);
    const float q = a * y;
    const float r = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(r, y, q);
}
__device__ __forceinline__ bool same(float a, float b) {
    return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
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
    if (!same(div_rn(a, b), a / b)) atomicAdd(&cnt[0], 1ull);
}
// every float a with |a| in [2^-40, 2^2) (both signs) against one b
__global__ void sweep_kernel(uint32_t base, float b, unsigned long long* cnt) {
    const uint32_t u = base + blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lo = (127u - 40u) << 23, hi = (127u + 2u) << 23;
    const uint32_t m = lo + (u >> 1) % (hi - lo);
    const float a = __uint_as_float(m | ((u & 1u) << 31));
    if (!same(div_rn(a, b), a / b)) atomicAdd(&cnt[0], 1ull);
}

int main() {
    unsigned long long* d;
    hipMalloc(&d, 64);
    const int ranges[][2] = {{-1, 1}, {-20, 20}, {-60, 60}, {-100, 100}, {0, 0}, {-1, 0}};
    for (auto& r : ranges) {
        hipMemset(d, 0, 8);
        for (uint32_t seed = 0; seed < 16; ++seed) div_kernel<<<(1u << 28) / 256, 256>>>(seed, r[0], r[1], d);
        unsigned long long h = 0;
        hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
        printf("div_rn, exponents [%d, %d], 2^32 random pairs: %llu mismatches\n", r[0], r[1], h);
        fflush(stdout);
    }
    // b: the 4096 floats either side of 1 (member normalize's lengths), and kPI
    unsigned long long tot = 0, nb = 0;
    const uint32_t span = 2u * ((2u + 40u) << 23);   // the a sweep: both signs of [2^-40, 4)
    auto sweep = [&](float b) {
        hipMemset(d, 0, 8);
        for (uint64_t base = 0; base < span; base += 1ull << 28)
            sweep_kernel<<<(1u << 28) / 256, 256>>>((uint32_t)base, b, d);
        unsigned long long h = 0;
        hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
        tot += h;
        ++nb;
    };
    for (int k = -4096; k <= 4096; k += 64) {   // (every 64th: the sweep per b is 2^30 values)
        const uint32_t one = 0x3f800000u;
        const uint32_t u = (uint32_t)((int)one + k);
        float b;
        memcpy(&b, &u, 4);
        sweep(b);
    }
    sweep(3.1415926f);
    printf("div_rn, every a in +-[2^-40, 4) against %llu values of b near 1 and kPI: %llu mismatches\n", nb, tot);
    hipFree(d);
    return 0;
}
