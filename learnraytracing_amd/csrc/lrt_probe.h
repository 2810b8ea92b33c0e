// The pool kernel's tile-cost probe (lrt_order.hip): the first launch of a view takes its
// tiles in the probe's heaviest-first order.
#pragma once
#include "lrt_internal.h"

namespace lrt {

// ---- first launch of a view: a cost probe instead of queue order ------------------------
// The heaviest-first order (tile_order) needs each tile's cost. Until a launch of the render
// signature has measured them, a probe estimates them: kProbe camera rays per tile (a 4x4
// grid over the tile, the launch's first frame, the real camera and seeds), each weighted by
// what its first hit costs a path on average -- the sky ends the path at once, a Lambert
// surface scatters and samples its lights, metal reflects, glass refracts into long chains.
// One closest hit per probe ray, 4 tiles per wave: ~1/16 of a 64-px, 4-spp tile's camera
// rays and none of its bounces. probe_order_kernel then counting-sorts the tiles by
// descending key in one workgroup. Only the order in which the render takes its tiles
// changes, never a pixel; the render still records its measured costs for later launches.
constexpr int kProbe = 16;
constexpr unsigned kProbeW[4] = {1u, 3u, 4u, 8u};   // sky, Lambert, Metal, Dielectric
constexpr unsigned kProbeKeyMax = kProbe * 8u;
template <int kAcc>
__global__ __launch_bounds__(64) void probe_kernel(const KernelArgs a, unsigned* key, int ntiles, int TX, int TY) {
    extern __shared__ float4 smem[];
    const int lane = threadIdx.x;
    SceneView sc;
    sc.rnlut = nullptr;
    sc.sph = a.sph;
    sc.mats = a.mats;
    sc.lights = a.lights;
    sc.count = a.count;
    sc.nlights = a.nlights;
    sc.bv = a.bv;
    sc.gv = a.gv;
    sc.bstk = reinterpret_cast<unsigned short*>(smem) + lane;
    sc.bstride = 64;
    const int tile = blockIdx.x * (64 / kProbe) + lane / kProbe, k = lane % kProbe;
    const int tilesX = (a.xc + TX - 1) / TX;
    const int lx = (tile % tilesX) * TX + (k % 4) * TX / 4 + TX / 8;
    const int ly = (tile / tilesX) * TY + (k / 4) * TY / 4 + TY / 8;
    unsigned w = 0;
    if (tile < ntiles && lx < a.xc && ly < a.rows) {
        const int x = a.x0 + lx, y = GlobalRow(a, ly);
        uint32_t rng = PixelSeed((uint32_t)x, (uint32_t)y, (uint32_t)a.frame0);
        const float u = ((float)x + RandomFloat01(rng)) * (1.0f / (float)a.width);
        const float v = ((float)y + RandomFloat01(rng)) * (1.0f / (float)a.height);
        const Ray r = GetRay(a.cam, u, v, rng, nullptr);
        float t;
        const int id = ClosestHitSV<kAcc, 0>(r, kMinT, kMaxT, sc, t);
        const int type = id < 0 ? -1 : libm::f2u_i(a.mats[3 * id].w);
        w = kProbeW[type < 0 ? 0 : type > 2 ? 3 : type + 1];
    }
    for (int off = 1; off < kProbe; off <<= 1) w += __shfl_xor(w, off, 64);
    if (tile < ntiles && k == 0) key[tile] = w;
}
// One workgroup: per-wave histograms of the keys in LDS (16 copies, so the few distinct keys
// do not serialise every atomic on one address), bucket starts in descending key order
// across the copies, then every tile to its wave's share of its bucket (order within a
// bucket is whatever the LDS atomics give).
__global__ __launch_bounds__(1024) void probe_order_kernel(const unsigned* key, int* perm, int n) {
    constexpr int kB = kProbeKeyMax + 1, kW = 16;
    __shared__ unsigned hist[kW][kB];
    const int w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < kW * kB; i += 1024) (&hist[0][0])[i] = 0;
    __syncthreads();
    // 16 independent loads in flight per thread and pass (one at a time, the passes were
    // load-latency bound: 22 us for 14,400 tiles)
    for (int base = 0; base < n; base += 16 * 1024) {
        unsigned k[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int i = base + j * 1024 + (int)threadIdx.x;
            k[j] = i < n ? min(key[i], kProbeKeyMax) : kB;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if (k[j] < (unsigned)kB) atomicAdd(&hist[w][k[j]], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 64) {   // one wave: bucket b's totals, descending exclusive scan
        unsigned run = 0;
        for (int b0 = kB - 1; b0 >= 0; b0 -= 64) {
            const int b = b0 - (int)threadIdx.x;
            unsigned tot = 0;
            if (b >= 0)
                for (int c = 0; c < kW; ++c) tot += hist[c][b];
            unsigned inc = tot;   // inclusive scan over the lanes (descending b)
            for (int off = 1; off < 64; off <<= 1) {
                const unsigned o = __shfl_up(inc, off, 64);
                if ((int)threadIdx.x >= off) inc += o;
            }
            unsigned base = run + inc - tot;
            if (b >= 0)
                for (int c = 0; c < kW; ++c) {
                    const unsigned v = hist[c][b];
                    hist[c][b] = base;
                    base += v;
                }
            run += __shfl(inc, 63, 64);
        }
    }
    __syncthreads();
    for (int base = 0; base < n; base += 16 * 1024) {
        unsigned k[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int i = base + j * 1024 + (int)threadIdx.x;
            k[j] = i < n ? min(key[i], kProbeKeyMax) : kB;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if (k[j] < (unsigned)kB) perm[atomicAdd(&hist[w][k[j]], 1u)] = base + j * 1024 + (int)threadIdx.x;
    }
}


}  // namespace lrt
