// Shader clock probe (round 6, profiles/r6_e): one wave per CU spins ~200k shader cycles and
// records the shader-clock (s_memtime) and constant 100-MHz (s_memrealtime) deltas, so that
// the caller can read the running shader clock between renders.
#include <hip/hip_runtime.h>
extern "C" __global__ void clock_spin(unsigned long long* out) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long t = t0;
    float acc = (float)threadIdx.x;
    while (t - t0 < 200000ull) {
        for (int i = 0; i < 64; ++i) acc = acc * 1.0000001f + 0.5f;
        t = __builtin_amdgcn_s_memtime();
    }
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = t - t0;
        out[2 * blockIdx.x + 1] = (r1 - r0) + (acc == 0.0f ? 1ull : 0ull);
    }
}
extern "C" int clock_probe_mhz(void* stream, unsigned long long* d_out, int blocks, double* mhz) {
    hipStream_t s = (hipStream_t)stream;
    clock_spin<<<blocks, 64, 0, s>>>(d_out);
    unsigned long long h[2 * 1024];
    if (hipMemcpyAsync(h, d_out, sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
    if (hipStreamSynchronize(s) != hipSuccess) return -1;
    double c = 0, r = 0;
    for (int b = 0; b < blocks; ++b) { c += (double)h[2 * b]; r += (double)h[2 * b + 1]; }
    *mhz = c / (r / 100.0);   // s_memrealtime ticks at 100 MHz
    return 0;
}
