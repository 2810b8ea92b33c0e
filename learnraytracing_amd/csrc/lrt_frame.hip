// Frame assembly after a gather (unshard, the RGB-only exchange) and the present step
// (LinearToSRGB + BGRA8, main.cpp:109-141).
#include "lrt_internal.h"

namespace lrt {

// Frame assembly: shard g's local row ly -> global row (as lrt_render_desc's map).
__global__ void unshard_kernel(const float4* __restrict__ src, float4* __restrict__ dst, int width, int height,
                               int rb, int period, int maxRows) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= width || y >= height) return;
    const int blk = y / rb;
    const int g = blk % period;
    const int ly = (blk / period) * rb + y % rb;
    dst[(size_t)y * width + x] = src[((size_t)g * maxRows + ly) * width + x];
}

// The multi-GPU exchange carries RGB only: the shard's alpha is never written by the render
// (parallel.cpp:283-285) and the frame's own alpha stays where it is, so 12 of the 16 bytes
// per pixel cross xGMI (precision unchanged).
__global__ void pack_rgb_kernel(const float4* __restrict__ src, float* __restrict__ dst, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 v = src[i];
    dst[3 * i + 0] = v.x;
    dst[3 * i + 1] = v.y;
    dst[3 * i + 2] = v.z;
}
__global__ void unshard_rgb_kernel(const float* __restrict__ src, float4* __restrict__ dst, int width, int height,
                                   int rb, int period, int maxRows) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= width || y >= height) return;
    const int blk = y / rb;
    const int g = blk % period;
    const int ly = (blk / period) * rb + y % rb;
    const float* sp = src + 3 * (((size_t)g * maxRows + ly) * width + x);
    float* d = reinterpret_cast<float*>(dst + (size_t)y * width + x);   // alpha untouched
    d[0] = sp[0];
    d[1] = sp[1];
    d[2] = sp[2];
}

// LinearToSRGB + pack (main.cpp:109-141): b | g << 8 | r << 16 per pixel.
LRT_DEV uint32_t linear_to_srgb(float x) {   // main.cpp:109-115
    x = (x < 0.0f) ? 0.0f : x;                                   // std::max(x, 0.0f)
    x = 1.055f * libm::powf(x, 0.416666667f) - 0.055f;
    x = (x < 0.0f) ? 0.0f : x;                                   // std::max(..., 0.0f)
    uint32_t u = (uint32_t)(x * 255.9f);
    return u < 255u ? u : 255u;                                  // std::min(u, 255u)
}
__global__ void present_kernel(const float4* __restrict__ src, uint32_t* __restrict__ dst, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float4 c = src[i];
    dst[i] = linear_to_srgb(c.z) | (linear_to_srgb(c.y) << 8) | (linear_to_srgb(c.x) << 16);
}

hipError_t launch_unshard(const float4* src, float4* dst, int width, int height, int rb, int period, int maxRows,
                          hipStream_t s) {
    dim3 grid((unsigned)((width + 255) / 256), (unsigned)height);
    unshard_kernel<<<grid, 256, 0, s>>>(src, dst, width, height, rb, period, maxRows);
    return hipGetLastError();
}

hipError_t launch_pack_rgb(const float4* src, float* dst, size_t n, hipStream_t s) {
    pack_rgb_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(src, dst, n);
    return hipGetLastError();
}

hipError_t launch_unshard_rgb(const float* src, float4* dst, int width, int height, int rb, int period, int maxRows,
                              hipStream_t s) {
    dim3 grid((unsigned)((width + 255) / 256), (unsigned)height);
    unshard_rgb_kernel<<<grid, 256, 0, s>>>(src, dst, width, height, rb, period, maxRows);
    return hipGetLastError();
}

}  // namespace lrt

using namespace lrt;

extern "C" {

int lrt_shard_rows(int height, int row_block, int period, int phase) {
    if (height < 0 || row_block < 1 || period < 1 || phase < 0 || phase >= period)
        return fail(LRT_E_INVALID, "invalid shard geometry");
    int blocks = (height + row_block - 1) / row_block;
    int rows = 0;
    for (int b = phase; b < blocks; b += period) {
        int top = (b + 1) * row_block;
        rows += (top > height ? height : top) - b * row_block;
    }
    return rows;
}

int lrt_unshard_rows(const float* d_src, float* d_dst, int width, int height, int row_block, int period,
                     void* stream) {
    if (!d_src || !d_dst || width < 1 || height < 1 || row_block < 1 || period < 1)
        return fail(LRT_E_INVALID, "invalid unshard arguments");
    int maxRows = lrt_shard_rows(height, row_block, period, 0);
    hipStream_t s = (hipStream_t)stream;
    dim3 grid((width + 255) / 256, height);
    unshard_kernel<<<grid, 256, 0, s>>>(reinterpret_cast<const float4*>(d_src), reinterpret_cast<float4*>(d_dst),
                                        width, height, row_block, period, maxRows);
    LRT_HIP(hipGetLastError());
    return LRT_OK;
}

int lrt_pack_rgb(const float* d_rgba, float* d_rgb, long long npix, void* stream) {
    RoctxRange rr_("lrt_pack_rgb");
    if (!d_rgba || !d_rgb || npix < 0) return fail(LRT_E_INVALID, "invalid pack arguments");
    if (npix == 0) return LRT_OK;
    pack_rgb_kernel<<<(unsigned)((npix + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        reinterpret_cast<const float4*>(d_rgba), d_rgb, (size_t)npix);
    LRT_HIP(hipGetLastError());
    return LRT_OK;
}

int lrt_unshard_rows_rgb(const float* d_src_rgb, float* d_dst, int width, int height, int row_block, int period,
                         void* stream) {
    RoctxRange rr_("lrt_unshard_rows_rgb");
    if (!d_src_rgb || !d_dst || width < 1 || height < 1 || row_block < 1 || period < 1)
        return fail(LRT_E_INVALID, "invalid unshard arguments");
    const int maxRows = lrt_shard_rows(height, row_block, period, 0);
    dim3 grid((width + 255) / 256, height);
    unshard_rgb_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(d_src_rgb, reinterpret_cast<float4*>(d_dst), width,
                                                             height, row_block, period, maxRows);
    LRT_HIP(hipGetLastError());
    return LRT_OK;
}

int lrt_present_bgra8(const float* d_rgba, uint32_t* d_bgra, int width, int height, void* stream) {
    RoctxRange rr_("lrt_present_bgra8");
    if (!d_rgba || !d_bgra || width < 1 || height < 1) return fail(LRT_E_INVALID, "invalid present arguments");
    int n = width * height;
    hipStream_t s = (hipStream_t)stream;
    present_kernel<<<(n + 255) / 256, 256, 0, s>>>(reinterpret_cast<const float4*>(d_rgba), d_bgra, n);
    LRT_HIP(hipGetLastError());
    return LRT_OK;
}

}  // extern "C"
