// liblrt_hip.so — the MI355X path tracer behind the C-ABI of include/lrt.h.
//
// v0 (trace_kernel, the default): TraceRowJob's per-pixel body (parallel.cpp:270-286)
// with a pixel's S samples spread over up to 16 adjacent lanes and lerped in frame order
// (so the progressive sequence of S DrawTest calls is reproduced bit for bit from the
// buffer's prev value); persistent single-wave workgroups fed from 16 tile queues; the
// scene, the powf tables and the recursion stack in LDS; one read and one 16-byte write
// of each pixel per call; rays counted per lane, reduced per wave, folded per queue.
// v5 (pool_kernel, lrt_pool.h) adds sample-pool regeneration; v4 wavefront (lrt_wavefront.h)
// is opt-in. Host side: scene upload + BVH build, launch policy, multi-device split with the
// RCCL gather, the C-ABI.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#ifndef LRT_ROCTX   // roctx ranges (tracing only): the Makefile sets it when the header exists
#define LRT_ROCTX 0
#endif
#if LRT_ROCTX
#include <rocprofiler-sdk-roctx/roctx.h>
#endif
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <climits>
#include <functional>
#include <type_traits>
#include <cmath>
#include <mutex>
#include <string>
#include <vector>

#include "lrt.h"
#include "lrt_trace.h"

#define LRT_VERSION_STRING "lrt-mi355x 0.2.0 gfx950"

namespace lrt {

#ifndef LRT_V0_BLOCK
#define LRT_V0_BLOCK 64
#endif
// v0 workgroup: one wave by default. A wave finished early in a multi-wave block keeps
// its slot (and the block's LDS) until the slowest wave ends; with path lengths as
// uneven as these, single-wave blocks keep ~1 more wave resident per SIMD.
constexpr int kBlock = LRT_V0_BLOCK;
static_assert(kBlock == 64 || kBlock == 256, "v0 block: 1 or 4 waves");
constexpr int kBlockWavesX = kBlock == 256 ? 2 : 1;           // waves per block in x
constexpr int kBlockWavesY = kBlock / 64 / kBlockWavesX;       // and in y
// a wave's pixels: 64 / kSplit of them, 8 wide (kSplit <= 8) or a single row
constexpr int WaveCols(int split) { return split <= 8 ? 8 : 64 / split; }
#ifndef LRT_V0_DYNAMIC
#define LRT_V0_DYNAMIC 1
#endif
// Work counters: same-address device-scope atomics serialise at ~12 ns each (measured
// ~80/us chip-wide), so v0's tile queue and ray count are split over kV0Queues
// counters, each on its own 512-B line; block b serves queue b % kV0Queues, which owns
// tiles q, q + kV0Queues, ...
#ifndef LRT_V0_QUEUES
#define LRT_V0_QUEUES 16
#endif
constexpr int kV0Queues = LRT_V0_QUEUES;
constexpr int kCtrStride = 64;   // u64s between counters
static_assert(!LRT_V0_DYNAMIC || kBlock == 64, "dynamic v0 tiles are fetched per wave: one wave per block");

constexpr int kMaxDepthSupported = 64;

struct KernelArgs {
    CameraDev cam;
    const float4* sph;
    const float4* mats;
    const int* lights;
    int count, nlights;
    int width, height;
    int x0, xc, y0, rows;
    int rb, rp, rph;
    int frame0, frames, maxDepth;
    float4* out;
    unsigned long long* rays;
    BvhView bv;
    int bvh_stack_offset;   // bytes into dynamic LDS
    float4* ovf;            // recursion stack levels >= kTraceLdsLevels (null when maxDepth fits)
    unsigned long long* wtrace;   // LRT_EXP_WAVETRACE builds only: per-wave start/end/ids
    unsigned long long* tiles;    // this launch's counters: [q] tile queue, [kV0Queues + q] finished
                                  // blocks (bits 48-63) and ray total (bits 0-47) of queue q
    int ndl;                      // LRT_F_NO_DOUBLE_LIGHT
    // lrt_features (kFeat launches): normal, world_pos, albedo, color_std, normal_std,
    // world_pos_std (any may be null) and the last frame they are updated for (< 0: all)
    float4* feat[6];
    int featMax;
    int regenMin;                 // v5: waiting lanes that trigger a refill
    const float* lerp;            // lerpFac = (float)f / (float)(f + 1) for f < kLerpTable (parallel.cpp:262)
    float4* samp;                 // sample mode: frames planes of xc * rows colours
    float4* colbuf;               // v5 (pool): poolSlots colour slots per block
    int poolSlots;
    const int* perm;              // v5: queue position -> tile, heaviest measured tiles first (null: identity)
    unsigned* tcost;              // v5: per-tile cost recording (100 MHz ticks of the tile's wave), or null
    int sampOnly;                 // colours only (the pipelined host path): samp is the caller's
    float4* frame;                // lrt_render_device_to_frame: the whole width x height frame (any
                                  // device, IPC/peer-mapped) that each finished pixel is also stored
                                  // to at its global row -- the multi-GPU exchange fused into the
                                  // render's last store; null otherwise
};

// Global position of local row ly (lrt_render_desc's row map).
LRT_DEV int GlobalRow(const KernelArgs& a, int ly) { return a.y0 + (ly / a.rb) * a.rb * a.rp + a.rph * a.rb + ly % a.rb; }
constexpr int kLerpTable = 1 << 16;
constexpr int kFixedSpheres = 9;   // the reference's kSphereCount (parallel.cpp:27)

// AdaptiveStdvar (fragmentShader.fs.glsl:494-497) per channel, pow(x, 2) as x * x.
LRT_DEV float adaptive_std(float lastStd, float lastMean, int n, float newVal, float newMean) {
    const float nf = (float)n;
    const float dm = lastMean - newMean, dv = newVal - newMean;
    return __builtin_sqrtf((nf * (lastStd * lastStd) + nf * (dm * dm) + dv * dv) / (float)(n + 1));
}
LRT_DEV float4 adaptive_std3(float4 sd, float4 lastMean, F3 v, float4 newMean, int n) {
    sd.x = adaptive_std(sd.x, lastMean.x, n, v.x, newMean.x);
    sd.y = adaptive_std(sd.y, lastMean.y, n, v.y, newMean.y);
    sd.z = adaptive_std(sd.z, lastMean.z, n, v.z, newMean.z);
    return sd;
}
LRT_DEV float4 lerp_feature(float4 m, F3 v, float lerpFac) {   // parallel.cpp:282's lerp
    F3 c = f3(m.x, m.y, m.z) * lerpFac + v * (1.0f - lerpFac);
    m.x = c.x;
    m.y = c.y;
    m.z = c.z;
    return m;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// A block's last act (one thread): ONE atomic on queue q's 64-bit word that carries the
// count of finished blocks in bits 48-63 and the queue's ray total in bits 0-47 (< 2.8e14
// rays per queue and launch). The block that takes the count to bq -- every fetch on q
// has returned by then -- folds the total into the caller's counter and re-arms q's
// counters for the slot's next launch. No fence is needed (a device-scope fence writes
// back the XCD's L2 on gfx950: measured +28 us per launch), and no collect kernel.
constexpr int kDoneShift = 48;
__device__ void block_epilogue(unsigned long long* tiles, unsigned long long* rays, int q, int bq,
                               unsigned long long total) {
    unsigned long long* const word = tiles + (kV0Queues + q) * kCtrStride;
    const unsigned long long inc = (1ull << kDoneShift) + total;
    const unsigned long long old = atomicAdd(word, inc);
    if ((old >> kDoneShift) == (unsigned long long)(bq - 1)) {
        const unsigned long long v = (old + inc) & ((1ull << kDoneShift) - 1ull);
        atomicExch(word, 0ull);
        atomicExch(tiles + q * kCtrStride, 0ull);
        if (v) atomicAdd(rays, v);
    }
}

// 4 waves per SIMD: caps VGPRs at 128. The MAXD 20/64 and BVH instances otherwise
// take 129-144 and drop to 3 waves (config 3: 4.44 -> 4.15 ms, config 4: 587 -> 538 ms
// with the cap; the BVH instances spill 28-40 B/lane to scratch, which costs less).
#ifndef LRT_V0_WAVES_PER_EU
#define LRT_V0_WAVES_PER_EU 4
#endif
// v0: the reference's per-pixel loop (parallel.cpp:255-289) with each pixel's frames
// spread over kSplit adjacent lanes. Lane `sub` traces frames frame0 + sub, + sub +
// kSplit, ...; after each round of kSplit frames every lane of the pixel gathers the
// round's colours and applies the reference's running lerp (:262, :282) in frame order,
// so the accumulated value is bit-identical to the serial loop. Splitting multiplies the
// number of independent wave tasks by kSplit (config 2: 57,600 instead of 14,400 for
// 1,024 SIMDs) and shortens them, which evens out the tail.
// The grid is persistent (as many blocks as fit, grid-stride over tiles): short wave
// tasks dispatched one per workgroup are limited by the workgroup dispatch rate
// (~80 waves/us chip-wide measured), which left SIMDs at ~2 of 4 resident waves.
//
// kSamp (sample mode, several rounds per pixel and few pixels -- one GPU's row shard of a
// multi-GPU frame): a wave task is ONE round of one tile, so tasks stay as short as at
// one round per pixel; each lane stores its sample colour in a.samp (frame-major planes)
// and merge_samples_kernel applies the lerp chain in frame order afterwards.
// kNS > 0: compile-time sphere count (kDefaultSpheres for the reference's scene): the
// closest-hit scans unroll fully (config 2: 0.359 -> 0.335 ms, config 3: 3.07 -> 2.84 ms).
template <int MAXD, bool kLds, bool kBvh, int kSplit, bool kFeat = false, bool kSamp = false, int kNS = 0>
__global__ __launch_bounds__(kBlock, LRT_V0_WAVES_PER_EU) void trace_kernel(const KernelArgs a) {
    static_assert(kNS == 0 || (kLds && !kBvh), "a fixed sphere count is for the LDS linear scan");
    static_assert(!kFeat || kSplit == 1, "feature launches keep a pixel's frames on one lane");
    static_assert(!(kFeat && kSamp), "sample mode has no features");
    // LDS: [recursion stack kTraceLdsLevels x kBlock][powf tables][spheres][materials][lights][bvh stack]
    extern __shared__ float4 smem[];
    const int tid = threadIdx.x;
    // powf tables (Dielectric's schlick): a per-lane gather from global memory costs a
    // VMEM round trip per lookup, and vmcnt retires in order behind the tile fetch
    double* s_pow = reinterpret_cast<double*>(smem + kTraceLdsLevels * kBlock);
    {
        const libm::PowTables g = libm::pow_tables();
        for (int i = tid; i < 16; i += kBlock) {
            s_pow[i] = g.invc[i];
            s_pow[16 + i] = g.logc[i];
        }
        for (int i = tid; i < 32; i += kBlock) reinterpret_cast<uint64_t*>(s_pow + 32)[i] = g.exp2[i];
    }
    // renormalize() table after the powf tables (not in BVH launches: their 16 waves/CU
    // have no LDS to spare)
    constexpr int kLutBytes = kBvh ? 0 : kRenormBytes;
    float* s_lut = kBvh ? nullptr : reinterpret_cast<float*>(s_pow + 64);
    if (!kBvh) renorm_lut_fill(s_lut, tid, kBlock);
    float4* s_sph = smem + kTraceLdsLevels * kBlock + (kPowTableBytes + kLutBytes) / 16;
    float4* s_mat = s_sph + a.count;
    int* s_lights = reinterpret_cast<int*>(s_mat + 3 * a.count);
    if (kLds) {
        for (int i = tid; i < a.count; i += kBlock) s_sph[i] = a.sph[i];
        for (int i = tid; i < 3 * a.count; i += kBlock) s_mat[i] = a.mats[i];
        for (int i = tid; i < a.nlights; i += kBlock) s_lights[i] = a.lights[i];
    }
    __syncthreads();
    SceneView sc;
    sc.pow.invc = s_pow;
    sc.pow.logc = s_pow + 16;
    sc.pow.exp2 = reinterpret_cast<const uint64_t*>(s_pow + 32);
    sc.rnlut = s_lut;
    sc.sph = kLds ? s_sph : a.sph;
    sc.mats = kLds ? s_mat : a.mats;
    sc.lights = kLds ? s_lights : a.lights;
    sc.count = a.count;
    sc.nlights = a.nlights;
    sc.bv = a.bv;
    sc.bstk = reinterpret_cast<unsigned short*>(reinterpret_cast<char*>(smem) + a.bvh_stack_offset) + tid;
    sc.bstride = kBlock;
#ifdef LRT_EXP_SECSTATS
    __shared__ unsigned long long s_sectime[kBlock / 64][2 + 3 * kSecN];
    sc.secstats = a.wtrace;
    sc.sectime = s_sectime[tid >> 6];
    if ((tid & 63) == 0) {
        for (int k = 0; k < 2 + 3 * kSecN; ++k) sc.sectime[k] = 0;
        sc.sectime[0] = kSecOther;
        sc.sectime[1] = __builtin_amdgcn_s_memtime();
    }
#endif
#ifdef LRT_EXP_WAVETRACE
    const unsigned long long wt0 = __builtin_amdgcn_s_memrealtime();
#endif
    const size_t gtid = (size_t)blockIdx.x * kBlock + tid;
    const size_t gthreads = (size_t)gridDim.x * kBlock;

    // wave = kWaveCols x kWaveRows pixels x kSplit frame lanes; block = kBlockWavesX x kBlockWavesY waves
    const int wave = tid >> 6, lane = tid & 63;
    const int sub = lane % kSplit, p = lane / kSplit;
    constexpr int kWaveCols = WaveCols(kSplit);
    constexpr int kWaveRows = 64 / kSplit / kWaveCols;
    constexpr int kTileRows = kBlockWavesY * kWaveRows;
    constexpr int kTileX = kWaveCols * kBlockWavesX;
    const int tilesX = (a.xc + kTileX - 1) / kTileX;
    const int rounds = kSamp ? (a.frames + kSplit - 1) / kSplit : 1;   // tasks per tile
    const int ntiles = tilesX * ((a.rows + kTileRows - 1) / kTileRows) * rounds;
    const float invWidth = 1.0f / (float)a.width;     // parallel.cpp:260
    const float invHeight = 1.0f / (float)a.height;   // parallel.cpp:261
    const int fend = a.frame0 + a.frames;
    int rays = 0;
    const int q = blockIdx.x % kV0Queues;
    const int bq = ((int)gridDim.x - q + kV0Queues - 1) / kV0Queues;   // blocks serving queue q
    const int nq = (ntiles - q + kV0Queues - 1) / kV0Queues;            // tiles owned by queue q
    unsigned long long* ctr = a.tiles + q * kCtrStride;
    for (int i = blockIdx.x / kV0Queues; i < nq;) {
        // Block b starts on its queue's tile b / kV0Queues; later tiles come from the
        // queue's counter (re-armed by the queue's last block, block_epilogue). The fetch is
        // issued after this tile's loads (vmcnt retires in order, so a load issued behind
        // the atomic would wait for it) and consumed after the trace, which hides it.
        // (Prefetching the next tile's pixels as well costs VGPRs beyond the 128 cap.)
        const int task = q + kV0Queues * i;
        const int tile = kSamp ? task / rounds : task;
        const int lx = (tile % tilesX) * kTileX + (wave % kBlockWavesX) * kWaveCols + (p % kWaveCols);
        const int ly = (tile / tilesX) * kTileRows + (wave / kBlockWavesX) * kWaveRows + (p / kWaveCols);
        const bool valid = lx < a.xc && ly < a.rows;
        const int x = a.x0 + lx;
        const int y = valid ? a.y0 + (ly / a.rb) * a.rb * a.rp + a.rph * a.rb + ly % a.rb : 0;
        float4* px = a.out + (size_t)ly * a.xc + lx;
        float4 acc = (valid && !kSamp) ? *px : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        float4 fb[6];   // feature running values (kFeat)
        const size_t pix = (size_t)ly * a.xc + lx;
        if constexpr (kFeat) {
#pragma unroll
            for (int k = 0; k < 6; ++k)
                fb[k] = (valid && a.feat[k]) ? a.feat[k][pix] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
        unsigned long long fetched = 0;
        if (LRT_V0_DYNAMIC && lane == 0) fetched = atomicAdd(ctr, 1ull);
        const int fbeg = kSamp ? a.frame0 + (task % rounds) * kSplit : a.frame0;
        const int fstop = kSamp ? fbeg + kSplit : fend;
        for (int f0 = fbeg; f0 < fstop; f0 += kSplit) {
            const int f = f0 + sub;
            F3 col = f3(0.0f, 0.0f, 0.0f);
            F3 feat[3] = {f3(0.0f, 0.0f, 0.0f), f3(0.0f, 0.0f, 0.0f), f3(0.0f, 0.0f, 0.0f)};
            if (valid && f < fend) {
                uint32_t rng = PixelSeed((uint32_t)x, (uint32_t)y, (uint32_t)f);
                sec_count(sc, kSecCamera);
                float u = ((float)x + RandomFloat01(rng)) * invWidth;              // :272
                float v = ((float)y + RandomFloat01(rng)) * invHeight;             // :273
                Ray r = GetRay(a.cam, u, v, rng, sc.rnlut);
                col = Trace<MAXD, kBvh, kFeat, kTraceLdsLevels, kNS>(r, a.maxDepth, rays, rng, sc, smem + tid, kBlock, a.ovf + gtid,
                                               gthreads, a.ndl, feat);
            }
            if constexpr (kSamp) {   // the merge kernel lerps the planes in frame order
                if (valid && f < fend)
                    a.samp[(size_t)(f - a.frame0) * ((size_t)a.xc * a.rows) + pix] = make_float4(col.x, col.y, col.z, 0.0f);
                continue;
            }
            // the group's colours go through this lane's (now free) stack level 0 in LDS:
            // one write, then one read per frame, instead of three shuffles per frame
            if (kSplit > 1) {
                smem[tid] = make_float4(col.x, col.y, col.z, 0.0f);
                __builtin_amdgcn_wave_barrier();
            }
#pragma unroll
            for (int j = 0; j < kSplit; ++j) {
                F3 c = col;
                if (kSplit > 1) {
                    const float4 cj = smem[tid - sub + j];
                    c = f3(cj.x, cj.y, cj.z);
                }
                const int fj = f0 + j;   // wave-uniform: the factor is a scalar load
                if (fj < fend) {
                    const float lerpFac = fj < kLerpTable ? a.lerp[fj] : (float)fj / (float)(fj + 1);   // :262
                    const float4 last = acc;
                    F3 prev = f3(acc.x, acc.y, acc.z);
                    const F3 sample = c;
                    c = prev * lerpFac + c * (1.0f - lerpFac);                     // :282
                    acc.x = c.x;
                    acc.y = c.y;
                    acc.z = c.z;
                    if constexpr (kFeat) {   // fragmentShader.fs.glsl:536-568
                        if (a.featMax < 0 || fj <= a.featMax) {
                            fb[3] = adaptive_std3(fb[3], last, sample, acc, fj);
                            const float4 lastN = fb[0], lastP = fb[1];
                            fb[0] = lerp_feature(fb[0], feat[0], lerpFac);
                            fb[1] = lerp_feature(fb[1], feat[1], lerpFac);
                            fb[2] = lerp_feature(fb[2], feat[2], lerpFac);
                            fb[4] = adaptive_std3(fb[4], lastN, feat[0], fb[0], fj);
                            fb[5] = adaptive_std3(fb[5], lastP, feat[1], fb[1], fj);
                        }
                    }
                }
            }
            if (kSplit > 1) __builtin_amdgcn_wave_barrier();
        }
        if (!kSamp && valid && sub == 0) {
            *px = acc;
            if (a.frame) a.frame[(size_t)y * a.width + x] = acc;   // the frame exchange, fused
        }
        if constexpr (kFeat) {
#pragma unroll
            for (int k = 0; k < 6; ++k)
                if (valid && a.feat[k]) a.feat[k][pix] = fb[k];
        }
        if (LRT_V0_DYNAMIC) {
            const unsigned long long n = __shfl(fetched, 0, 64) + (unsigned long long)bq;
            i = n < (unsigned long long)nq ? (int)n : nq;
        } else {
            i += bq;
        }
    }
    // one ray-count atomic per block: same-address atomics serialise in one L2 channel
    __shared__ unsigned long long s_rays[kBlock / 64];
    unsigned long long total = wave_sum((unsigned long long)rays);
    if (lane == 0) s_rays[wave] = total;
    __syncthreads();
#ifdef LRT_EXP_SECSTATS
    sec_enter(sc, kSecOther, false);
    if (lane == 0)
        for (int k = 0; k < kSecN; ++k) {
            unsigned long long* g = sc.secstats + 3 * (k + kSecN * (blockIdx.x & 15));
            atomicAdd(g, sc.sectime[2 + kSecN + k]);
            atomicAdd(g + 1, sc.sectime[2 + 2 * kSecN + k]);
            atomicAdd(g + 2, sc.sectime[2 + k]);
        }
#endif
#ifdef LRT_EXP_WAVETRACE
    if (lane == 0) {
        const size_t w = gtid >> 6;
        a.wtrace[4 * w + 0] = wt0;
        a.wtrace[4 * w + 1] = __builtin_amdgcn_s_memrealtime();
        a.wtrace[4 * w + 2] = __builtin_amdgcn_s_getreg((31 << 11) | 4);           // HW_ID
        a.wtrace[4 * w + 3] = __builtin_amdgcn_s_getreg((15 << 11) | 20);          // XCC_ID
    }
#endif
    if (tid == 0) {
        unsigned long long t = 0;
#ifndef LRT_EXP_NO_RAYCOUNT
        for (int w = 0; w < kBlock / 64; ++w) t += s_rays[w];
#endif
        block_epilogue(a.tiles, a.rays, q, bq, t);
    }
}

}  // namespace lrt
#include "lrt_pool.h"
namespace lrt {
// (lrt_wavefront.h follows merge_samples_kernel)


// Sample mode's second half: TraceRowJob's progressive lerp (parallel.cpp:262,280-286)
// over the frame planes in order, one thread per pixel (coalesced plane reads). `a` supplies
// the window's row map and the fused-exchange frame (a.frame); pixel i is the window's
// pixel pix0 + i.
__global__ void merge_samples_kernel(const float4* __restrict__ samp, float4* __restrict__ out, const float* lerp,
                                     int npix, int frame0, int frames, size_t stride, const KernelArgs a, int pix0) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npix) return;
    const float4 o = out[i];
    F3 acc = f3(o.x, o.y, o.z);
    for (int k = 0; k < frames; ++k) {
        const float4 c = samp[(size_t)k * stride + i];
        const int f = frame0 + k;
        const float lerpFac = f < kLerpTable ? lerp[f] : (float)f / (float)(f + 1);
        acc = acc * lerpFac + f3(c.x, c.y, c.z) * (1.0f - lerpFac);
    }
    float* d = reinterpret_cast<float*>(out + i);   // alpha untouched
    d[0] = acc.x;
    d[1] = acc.y;
    d[2] = acc.z;
    if (a.frame) {   // the frame exchange, fused
        const int p = pix0 + i, lx = p % a.xc, ly = p / a.xc;
        a.frame[(size_t)GlobalRow(a, ly) * a.width + a.x0 + lx] = make_float4(acc.x, acc.y, acc.z, o.w);
    }
}

// The pipelined host path's lerp (render_host_pipelined): prev from device memory (copied
// there by DMA while the colours were rendered), the result written straight into the
// caller's page-locked pixels over PCIe (posted writes; no D2H copy command).
__global__ __launch_bounds__(256) void merge_to_host_kernel(const float4* __restrict__ samp,
                                                            const float4* __restrict__ prev, float4* host,
                                                            const float* lerp, int npix, int frame0, int frames,
                                                            size_t stride) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < npix; i += gridDim.x * blockDim.x) {
        const float4 o = prev[i];
        F3 acc = f3(o.x, o.y, o.z);
        for (int k = 0; k < frames; ++k) {   // parallel.cpp:262,282 in frame order
            const float4 c = samp[(size_t)k * stride + i];
            const int f = frame0 + k;
            const float lerpFac = f < kLerpTable ? lerp[f] : (float)f / (float)(f + 1);
            acc = acc * lerpFac + f3(c.x, c.y, c.z) * (1.0f - lerpFac);
        }
        host[i] = make_float4(acc.x, acc.y, acc.z, o.w);   // alpha as read
    }
}

}  // namespace lrt
#include "lrt_wavefront.h"
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

LRT_HD float libm_eval(int kind, float x) {
    if (kind == 6 || kind == 7) {   // the path's sincosf (one reduction, both results)
        float sn, cs;
        libm::sincosf(x, &sn, &cs);
        return kind == 6 ? sn : cs;
    }
    return kind == 0   ? libm::sinf(x)
           : kind == 1 ? libm::cosf(x)
           : kind == 2 ? libm::powf5(x)
           : kind == 3 ? libm::powf(x, 0.416666667f)
           : kind == 4 ? sqrt_rn(x)    // the path's correctly rounded sqrt (fast sequence on the device)
                       : rcp_rn(x);    // and reciprocal
}

__global__ void libm_kernel(int kind, const float* __restrict__ in, float* __restrict__ out, long long n) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x = in[i];
    out[i] = libm_eval(kind, x);
}

// ---------------------------------------------------------------------------------
// host side
constexpr int kQueueSlots = 64;
constexpr size_t kTileSetU64 = 2 * kV0Queues * kCtrStride;   // one v0 launch's counters

struct Context {
    bool ready = false;
    int device = 0;
    int num_cus = 0;
    // render streams created by lrt_stream_create: CU-masked, and the CUs they may use
    std::vector<std::pair<hipStream_t, int>> masked_streams;
    unsigned long long* d_tiles = nullptr;   // kQueueSlots x v0 counter sets (trace_kernel)
    float* d_lerp = nullptr;                 // kLerpTable lerp factors (host IEEE division)
    struct Wavefront {                       // v4 path state, grown on demand
        void* buf = nullptr;
        size_t bytes = 0;
        unsigned long long* rayp = nullptr;  // 16 ray-count partials
    } wf;
    unsigned tiles_next = 0;
    unsigned scene_version = 0;   // bumped by every scene upload (tile-order signatures)
    // The pool kernel's tile orders, one per recent render signature (tile_order()): per-tile
    // costs recorded by one launch, then a heaviest-first permutation for the later ones.
    struct TileOrder {
        uint64_t sig = 0;              // the render signature (geometry, camera, scene)
        uint64_t gkey = 0;             // its geometry only: views that can share an order
        long long ntiles = 0, cap = 0;
        int state = 0;                 // 0: free, 2: permutation ready once ev_rec has passed
        void* d_base = nullptr;        // one allocation: cost, sorted keys, tile ids, perm, sort scratch
        unsigned* d_cost = nullptr;    // written by the recording launch
        unsigned* d_keys = nullptr;
        int* d_ids = nullptr;          // 0..cap-1
        int* d_perm = nullptr;         // written once (by the sort), read by every later launch
        void* d_tmp = nullptr;
        size_t tmp_bytes = 0;
        hipEvent_t ev_rec = nullptr;   // after the recording launch and the sort behind it
        int donor = -1;                // the entry whose order the recording launch borrowed
        // the streams whose launches read d_perm / wrote d_cost, each with an event after its
        // last such launch: the entry is reused only once all of them have passed it
        std::vector<std::pair<hipStream_t, hipEvent_t>> uses;
        unsigned long long tick = 0;   // least recently used goes first
    };
    static constexpr int kOrderSlots = 8;
    TileOrder order[kOrderSlots];
    unsigned long long order_tick = 0;
    hipStream_t stream = nullptr;
    int count = 0, nlights = 0;
    float4* d_sph = nullptr;
    float4* d_mats = nullptr;
    int* d_lights = nullptr;
    std::vector<lrt_sphere> spheres;
    std::vector<lrt_material> mats;
    // BVH (scenes with more than kBvhMinSpheres spheres)
    float4* d_bvh_nodes = nullptr;
    float4* d_bvh_lsph = nullptr;
    int* d_bvh_lid = nullptr;
    float bvh_margin = 0.0f;
    int bvh_nodes = 0;
    int bvh_on = 0, bvh_big0 = 0, bvh_nbig = 0;
    int bvh_stack_levels = kBvhStackLevels;   // this scene's traversal depth (<= kBvhStackLevels)

    float* d_frame = nullptr;   // lrt_draw_test / lrt_render_host staging
    float4* d_col = nullptr;    // the pipelined host path's sample colours
    size_t col_bytes = 0;
    hipStream_t s_in = nullptr;   // its H2D copy stream
    static constexpr int kHostChunks = 8;
    hipEvent_t ev_in[kHostChunks] = {};
    hipEvent_t ev_ret = nullptr;  // the pipelined call's own work done (the look-ahead may follow)
    // lrt_draw_test's look-ahead (render_host_pipelined): the colours of the frame after the
    // last one, rendered on `stream` behind that call's work, for the call that asks for it
    struct Lookahead {
        bool on = false;
        lrt_render_desc d;            // the render they are (memcmp: descs are zero-filled)
        unsigned scene_version = 0;
        int cur = 0;                  // the buffer pair holding them (the other is free)
        float4* col[2] = {};
        size_t bytes[2] = {};
        unsigned long long* d_rays = nullptr;   // 2 counters
        hipStream_t stream = nullptr;  // CU-masked: leaves CUs for the lerps it runs beside
        hipEvent_t ev = nullptr;       // recorded after the look-ahead render
        hipEvent_t ev_render = nullptr;
    } ahead;
    float* d_feat[6] = {};      // lrt_render_host_ex feature staging
    size_t feat_bytes[6] = {};
    size_t frame_bytes = 0;
    unsigned long long* d_rays = nullptr;
    // multi-device renders (lrt_initialize_devices): this device's row shard, packed for
    // the exchange, and (device 0) the gathered shards
    float* d_shard = nullptr;
    size_t shard_bytes = 0;
    float* d_gath = nullptr;
    size_t gath_bytes = 0;
    hipEvent_t ev_done = nullptr;   // this device's part of a multi-device render is enqueued
};

// One context per device in use: lrt_initialize binds the caller's current device (context
// 0); lrt_initialize_devices binds a list, and host renders are split over all of them.
constexpr int kMaxDevices = 16;
Context g_devs[kMaxDevices];
int g_ndev = 0;   // contexts in use
int g_cur = 0;    // the context the functions below act on (set under g_mu)
Context& ctx() { return g_devs[g_cur]; }

// Multi-device state (lrt_initialize_devices).
struct Multi {
    bool on = false;          // host renders are split over the g_ndev contexts
    bool rccl = false;        // the shards are gathered by RCCL (distinct devices); else peer copies
    int row_block = 8;        // rows per block of the row-block-cyclic split (LRT_ROW_BLOCK)
    ncclComm_t comms[kMaxDevices] = {};
};
Multi g_multi;

std::mutex g_mu;
char g_last_launch[256] = "";   // lrt_last_launch(): the kernel instance of the last render call
thread_local std::string t_err;
thread_local std::string t_launch;   // lrt_last_launch()'s copy for the calling thread

int fail(int code, const std::string& msg) {
    t_err = msg;
    return code;
}
int hip_fail(hipError_t e, const char* what) {
    return fail(LRT_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
#define LRT_HIP(call)                                            \
    do {                                                         \
        hipError_t _e = (call);                                  \
        if (_e != hipSuccess) return hip_fail(_e, #call);        \
    } while (0)

// parallel.cpp:15-51
const lrt_sphere kDefaultSpheres[9] = {
    {{0, -100.5f, -1}, 100.0f}, {{2, 1, -1}, 0.5f},  {{0, 0, -1}, 0.5f},
    {{-2, 0, -1}, 0.5f},        {{2, 0, 1}, 0.5f},   {{0, 0, 1}, 0.5f},
    {{-2, 0, 1}, 0.5f},         {{0.5f, 1, 0.5f}, 0.5f}, {{-1.5f, 1.5f, 0.f}, 0.3f},
};
const lrt_material kDefaultMats[9] = {
    {LRT_LAMBERT, {0.8f, 0.8f, 0.8f}, {0, 0, 0}, 0, 0},
    {LRT_LAMBERT, {0.8f, 0.4f, 0.4f}, {0, 0, 0}, 0, 0},
    {LRT_LAMBERT, {0.4f, 0.8f, 0.4f}, {0, 0, 0}, 0, 0},
    {LRT_METAL, {0.4f, 0.4f, 0.8f}, {0, 0, 0}, 0, 0},
    {LRT_METAL, {0.4f, 0.8f, 0.4f}, {0, 0, 0}, 0, 0},
    {LRT_METAL, {0.4f, 0.8f, 0.4f}, {0, 0, 0}, 0.2f, 0},
    {LRT_METAL, {0.4f, 0.8f, 0.4f}, {0, 0, 0}, 0.6f, 0},
    {LRT_DIELECTRIC, {0.4f, 0.4f, 0.4f}, {0, 0, 0}, 0, 1.5f},
    {LRT_LAMBERT, {0.8f, 0.6f, 0.2f}, {30, 25, 15}, 0, 0},
};

constexpr int kBvhMinSpheres = 16;
constexpr int kBvhLeaf = 6;   // leaf size (LRT_BVH_LEAF overrides, 1..16; config 4: 4 -> 350 ms, 6 -> 335, 8 -> 336)
constexpr int kBvhMaxBuildDepth = 22;   // < kBvhStackLevels
constexpr int kBvhSahMaxDepth = 12;     // SAH splits above this depth, median splits below (LRT_BVH_SAH_DEPTH)

// ---- BVH build (host): SAH splits, median splits on the longest centroid axis deeper down
struct BvhPrim {
    float lo[3], hi[3], c[3];
    int id;
};
struct BvhBuilder {
    std::vector<BvhPrim> P;
    std::vector<float4> nodes, lsph;
    std::vector<int> lid;
    const std::vector<float4>* sph = nullptr;
    int max_depth = 0;   // deepest internal node (root = 0)
    bool sah = true;     // SAH splits (LRT_BVH_SPLIT=median: median of the longest centroid axis)
    int leaf = kBvhLeaf;
    int sahDepth = kBvhSahMaxDepth;

    void sort_axis(int b, int e, int k) {
        std::sort(P.begin() + b, P.begin() + e, [k](const BvhPrim& x, const BvhPrim& y) {
            return x.c[k] < y.c[k] || (x.c[k] == y.c[k] && x.id < y.id);
        });
    }
    static void grow(const BvhPrim& p, float lo[3], float hi[3]) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], p.lo[k]);
            hi[k] = std::max(hi[k], p.hi[k]);
        }
    }
    static float half_area(const float lo[3], const float hi[3]) {
        const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return dx * dy + dy * dz + dz * dx;
    }

    static void bounds(const BvhPrim* p, int n, float lo[3], float hi[3]) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = INFINITY;
            hi[k] = -INFINITY;
        }
        for (int i = 0; i < n; ++i)
            for (int k = 0; k < 3; ++k) {
                lo[k] = std::min(lo[k], p[i].lo[k]);
                hi[k] = std::max(hi[k], p[i].hi[k]);
            }
    }
    int node(int begin, int end, int depth) {
        max_depth = std::max(max_depth, depth);
        const int idx = (int)(nodes.size() / 4);
        nodes.resize(nodes.size() + 4);
        const int n = end - begin;
        float cl[3] = {INFINITY, INFINITY, INFINITY}, ch[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = begin; i < end; ++i)
            for (int k = 0; k < 3; ++k) {
                cl[k] = std::min(cl[k], P[i].c[k]);
                ch[k] = std::max(ch[k], P[i].c[k]);
            }
        int axis = 0;
        for (int k = 1; k < 3; ++k)
            if (ch[k] - cl[k] > ch[axis] - cl[axis]) axis = k;
        int mid = begin + n / 2;
        if (sah && depth < sahDepth) {
            // surface-area heuristic over every split of the centroid order on each axis
            // (full sweep: scenes are at most a few thousand spheres); only above
            // kBvhSahMaxDepth, so the depth bound of the median split still holds
            float best = INFINITY;
            int bestAxis = axis, bestSplit = n / 2;
            std::vector<float> leftArea(n);
            for (int k = 0; k < 3; ++k) {
                sort_axis(begin, end, k);
                float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
                for (int i = 0; i < n - 1; ++i) {
                    grow(P[begin + i], lo, hi);
                    leftArea[i + 1] = half_area(lo, hi);
                }
                for (int q = 0; q < 3; ++q) {
                    lo[q] = INFINITY;
                    hi[q] = -INFINITY;
                }
                for (int i = n - 1; i >= 1; --i) {
                    grow(P[begin + i], lo, hi);
                    const float cost = leftArea[i] * (float)i + half_area(lo, hi) * (float)(n - i);
                    if (cost < best) {
                        best = cost;
                        bestAxis = k;
                        bestSplit = i;
                    }
                }
            }
            axis = bestAxis;
            mid = begin + bestSplit;
        }
        std::nth_element(P.begin() + begin, P.begin() + mid, P.begin() + end, [axis](const BvhPrim& x, const BvhPrim& y) {
            return x.c[axis] < y.c[axis] || (x.c[axis] == y.c[axis] && x.id < y.id);
        });
        float4 child[2][2];
        const int rng[2][2] = {{begin, mid}, {mid, end}};
        for (int h = 0; h < 2; ++h) {
            const int b = rng[h][0], e = rng[h][1], cnt = e - b;
            float lo[3], hi[3];
            bounds(P.data() + b, cnt, lo, hi);
            int ref, code;
            if (cnt <= leaf || depth + 1 >= kBvhMaxBuildDepth) {
                ref = (int)lsph.size();
                for (int i = b; i < e; ++i) {
                    lsph.push_back((*sph)[P[i].id]);
                    lid.push_back(P[i].id);
                }
                code = cnt;                      // leaf
            } else {
                ref = node(b, e, depth + 1);     // internal
                code = 0;
            }
            float fr, fc;
            memcpy(&fr, &ref, 4);
            memcpy(&fc, &code, 4);
            child[h][0] = make_float4(lo[0], lo[1], lo[2], fr);
            child[h][1] = make_float4(hi[0], hi[1], hi[2], fc);
        }
        nodes[4 * idx + 0] = child[0][0];
        nodes[4 * idx + 1] = child[0][1];
        nodes[4 * idx + 2] = child[1][0];
        nodes[4 * idx + 3] = child[1][1];
        return idx;
    }
};

struct BvhHost {
    std::vector<float4> nodes, lsph;
    std::vector<int> lid;
    int big0 = 0, nbig = 0;
    float margin = 0.0f;
    int stack_levels = 1;   // traversal stack entries needed: one deferred sibling per level
};

// Spheres far larger than the typical one (the ground, r = 100) stay out of the tree and
// are tested first; the rest get a BVH2 with leaves of <= kBvhLeaf spheres.
void build_bvh_host(const lrt_sphere* s, int n, const std::vector<float4>& sph, BvhHost& out) {
    std::vector<float> radii(n);
    for (int i = 0; i < n; ++i) radii[i] = std::fabs(s[i].radius);
    std::vector<float> sorted;
    for (float r : radii)
        if (std::isfinite(r)) sorted.push_back(r);
    float big_r = INFINITY;
    if (!sorted.empty()) {
        const size_t m = sorted.size() / 2;
        std::nth_element(sorted.begin(), sorted.begin() + m, sorted.end());
        big_r = 8.0f * sorted[m];
    }
    std::vector<int> big;
    BvhBuilder B;
    B.sph = &sph;
    {
        const char* e = getenv("LRT_BVH_SPLIT");
        B.sah = !(e && strcmp(e, "median") == 0);
        const char* l = getenv("LRT_BVH_LEAF");
        if (l) B.leaf = std::min(16, std::max(1, atoi(l)));
        const char* sd = getenv("LRT_BVH_SAH_DEPTH");
        if (sd) B.sahDepth = std::min(kBvhMaxBuildDepth, std::max(0, atoi(sd)));
    }
    float extent = 1.0f;
    for (int i = 0; i < n; ++i) {
        const bool finite = std::isfinite(s[i].center.x) && std::isfinite(s[i].center.y) &&
                            std::isfinite(s[i].center.z) && std::isfinite(radii[i]);
        // non-finite spheres have no box (and would break the split's ordering): like the
        // ground they are tested in index order by every ray, as in the reference's scan
        if (!finite || (radii[i] > big_r && big.size() < 16)) {
            big.push_back(i);
            continue;
        }
        BvhPrim p;
        const float r = radii[i];
        const float c3[3] = {s[i].center.x, s[i].center.y, s[i].center.z};
        for (int k = 0; k < 3; ++k) {
            // conservative box: c +/- |r|, padded well beyond float rounding
            const float pad = 1e-5f * (std::fabs(c3[k]) + r) + 1e-6f;
            p.lo[k] = c3[k] - r - pad;
            p.hi[k] = c3[k] + r + pad;
            p.c[k] = c3[k];
            extent = std::max(extent, std::max(std::fabs(p.lo[k]), std::fabs(p.hi[k])));
        }
        p.id = i;
        B.P.push_back(p);
    }
    if (B.P.size() >= 2) B.node(0, (int)B.P.size(), 0);
    else
        for (const BvhPrim& p : B.P) big.push_back(p.id);
    out.big0 = (int)B.lsph.size();
    for (int i : big) {
        B.lsph.push_back(sph[i]);
        B.lid.push_back(i);
    }
    out.nbig = (int)big.size();
    out.stack_levels = 1;
    if (!B.nodes.empty()) {   // collapse the BVH2 into 4-wide nodes (grandchildren of each node)
        auto ival = [](float f) { int v; memcpy(&v, &f, 4); return v; };
        auto fval = [](int v) { float f; memcpy(&f, &v, 4); return f; };
        std::vector<float4> n4;
        int depth4 = 0;
        std::function<int(int, int)> collapse = [&](int n2, int dep) -> int {
            depth4 = std::max(depth4, dep);
            const int idx = (int)(n4.size() / 8);
            n4.resize(n4.size() + 8);
            float4 kids[4][2];
            int k = 0;
            for (int c = 0; c < 2; ++c) {
                const float4 lo = B.nodes[4 * n2 + 2 * c], hi = B.nodes[4 * n2 + 2 * c + 1];
                if (ival(hi.w) == 0) {   // internal child: take its two children
                    const int m = ival(lo.w);
                    for (int g = 0; g < 2; ++g) {
                        kids[k][0] = B.nodes[4 * m + 2 * g];
                        kids[k][1] = B.nodes[4 * m + 2 * g + 1];
                        ++k;
                    }
                } else {                 // leaf or empty child stays
                    kids[k][0] = lo;
                    kids[k][1] = hi;
                    ++k;
                }
            }
            for (int c = 0; c < k; ++c)
                if (ival(kids[c][1].w) == 0) kids[c][0].w = fval(collapse(ival(kids[c][0].w), dep + 1));
            for (int c = 0; c < 4; ++c) {
                if (c < k) {
                    n4[8 * idx + 2 * c] = kids[c][0];
                    n4[8 * idx + 2 * c + 1] = kids[c][1];
                } else {   // empty slot
                    n4[8 * idx + 2 * c] = make_float4(INFINITY, INFINITY, INFINITY, fval(0));
                    n4[8 * idx + 2 * c + 1] = make_float4(-INFINITY, -INFINITY, -INFINITY, fval(-1));
                }
            }
            return idx;
        };
        collapse(0, 0);
        B.nodes.swap(n4);
        // a traversal holds at most one (node, child mask) entry per level above its node
        // (StackPush, lrt_bvh.h): depth4 entries; one spare
        out.stack_levels = depth4 + 1;
    }
    out.nodes.swap(B.nodes);
    out.lsph.swap(B.lsph);
    out.lid.swap(B.lid);
    out.margin = 1e-5f * extent + 1e-4f;
}

void free_scene(Context& c) {
    if (c.d_bvh_nodes) (void)hipFree(c.d_bvh_nodes);
    if (c.d_bvh_lsph) (void)hipFree(c.d_bvh_lsph);
    if (c.d_bvh_lid) (void)hipFree(c.d_bvh_lid);
    c.d_bvh_nodes = nullptr;
    c.d_bvh_lsph = nullptr;
    c.d_bvh_lid = nullptr;
    c.bvh_nodes = 0;
    c.bvh_on = 0;
    if (c.d_sph) (void)hipFree(c.d_sph);
    if (c.d_mats) (void)hipFree(c.d_mats);
    if (c.d_lights) (void)hipFree(c.d_lights);
    c.d_sph = nullptr;
    c.d_mats = nullptr;
    c.d_lights = nullptr;
}

// The device layout of a scene: float4(center, r^2), three material rows,
// emissive ids in index order.
int pack_scene(const lrt_sphere* s, const lrt_material* m, int n, std::vector<float4>& sph,
               std::vector<float4>& mats, std::vector<int>& lights) {
    if (!s || !m || n < 1 || n > LRT_MAX_SPHERES) return fail(LRT_E_INVALID, "scene: need 1..LRT_MAX_SPHERES spheres");
    sph.assign(n, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    mats.assign(3 * (size_t)n, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    lights.clear();
    for (int i = 0; i < n; ++i) {
        if (m[i].type < 0 || m[i].type > 2) return fail(LRT_E_INVALID, "scene: material type must be 0..2");
        const float r = s[i].radius;
        sph[i] = make_float4(s[i].center.x, s[i].center.y, s[i].center.z, r * r);
        const bool diel = m[i].type == LRT_DIELECTRIC;
        int type = m[i].type;
        float typef;
        memcpy(&typef, &type, 4);
        mats[3 * i + 0] = make_float4(m[i].albedo.x, m[i].albedo.y, m[i].albedo.z, typef);
        mats[3 * i + 1] = make_float4(m[i].emissive.x, m[i].emissive.y, m[i].emissive.z, m[i].roughness);
        mats[3 * i + 2] = diel ? make_float4(1.0f, 1.0f, 1.0f, m[i].ri)
                               : make_float4(m[i].albedo.x, m[i].albedo.y, m[i].albedo.z, m[i].ri);
        // parallel.cpp:96: skip only if every channel <= 0
        if (!(m[i].emissive.x <= 0 && m[i].emissive.y <= 0 && m[i].emissive.z <= 0)) lights.push_back(i);
    }
    return LRT_OK;
}

int upload_scene(Context& c, const lrt_sphere* s, const lrt_material* m, int n) {
    std::vector<float4> sph, mats;
    std::vector<int> lights;
    if (const int e = pack_scene(s, m, n, sph, mats, lights)) return e;
    free_scene(c);
    LRT_HIP(hipMalloc(&c.d_sph, sizeof(float4) * n));
    LRT_HIP(hipMalloc(&c.d_mats, sizeof(float4) * 3 * n));
    LRT_HIP(hipMalloc(&c.d_lights, sizeof(int) * (lights.empty() ? 1 : lights.size())));
    LRT_HIP(hipMemcpy(c.d_sph, sph.data(), sizeof(float4) * n, hipMemcpyHostToDevice));
    LRT_HIP(hipMemcpy(c.d_mats, mats.data(), sizeof(float4) * 3 * n, hipMemcpyHostToDevice));
    if (!lights.empty())
        LRT_HIP(hipMemcpy(c.d_lights, lights.data(), sizeof(int) * lights.size(), hipMemcpyHostToDevice));
    if (n > kBvhMinSpheres) {
        BvhHost B;
        build_bvh_host(s, n, sph, B);
        // the LDS traversal stack is sized to B.stack_levels entries per lane, which bounds
        // every push (StackPush: at most one entry per level above the current node)
        if (B.stack_levels > kBvhStackLevels) return fail(LRT_E_INVALID, "BVH deeper than the traversal stack");
        LRT_HIP(hipMalloc(&c.d_bvh_nodes, sizeof(float4) * std::max<size_t>(B.nodes.size(), 4)));
        LRT_HIP(hipMalloc(&c.d_bvh_lsph, sizeof(float4) * B.lsph.size()));
        LRT_HIP(hipMalloc(&c.d_bvh_lid, sizeof(int) * B.lid.size()));
        if (!B.nodes.empty())
            LRT_HIP(hipMemcpy(c.d_bvh_nodes, B.nodes.data(), sizeof(float4) * B.nodes.size(), hipMemcpyHostToDevice));
        LRT_HIP(hipMemcpy(c.d_bvh_lsph, B.lsph.data(), sizeof(float4) * B.lsph.size(), hipMemcpyHostToDevice));
        LRT_HIP(hipMemcpy(c.d_bvh_lid, B.lid.data(), sizeof(int) * B.lid.size(), hipMemcpyHostToDevice));
        c.bvh_nodes = (int)(B.nodes.size() / 8);
        c.bvh_big0 = B.big0;
        c.bvh_nbig = B.nbig;
        c.bvh_margin = B.margin;
        c.bvh_stack_levels = B.stack_levels;
        c.bvh_on = 1;
    }
    c.count = n;
    ++c.scene_version;
    c.nlights = (int)lights.size();
    c.spheres.assign(s, s + n);
    c.mats.assign(m, m + n);
    return LRT_OK;
}

lrt_float3 L3(float x, float y, float z) {
    lrt_float3 r = {x, y, z};
    return r;
}
// Host float3 helpers for the camera constructor (maths.h:63-97).
lrt_float3 h_sub(lrt_float3 a, lrt_float3 b) { return L3(a.x - b.x, a.y - b.y, a.z - b.z); }
lrt_float3 h_smul(float a, lrt_float3 b) { return L3(a * b.x, a * b.y, a * b.z); }
lrt_float3 h_cross(lrt_float3 a, lrt_float3 b) {
    return L3(a.y * b.z - a.z * b.y, -(a.x * b.z - a.z * b.x), a.x * b.y - a.y * b.x);
}
lrt_float3 h_normalize(lrt_float3 v) {
    float k = 1.0f / sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    return L3(v.x * k, v.y * k, v.z * k);
}

int validate(const lrt_render_desc* d) {
    if (!d) return fail(LRT_E_INVALID, "desc is NULL");
    if (d->width < 1 || d->height < 1) return fail(LRT_E_INVALID, "width/height must be >= 1");
    if (d->x0 < 0 || d->x_count < 0 || (long long)d->x0 + d->x_count > d->width)
        return fail(LRT_E_INVALID, "column window outside the image");
    if (d->row_block < 1 || d->row_period < 1 || d->row_phase < 0 || d->row_phase >= d->row_period)
        return fail(LRT_E_INVALID, "row_block/row_period/row_phase invalid");
    if (d->y0 < 0 || d->row_count < 0) return fail(LRT_E_INVALID, "y0/row_count must be >= 0");
    if (d->row_count > 0) {
        long long ly = d->row_count - 1;
        long long y = d->y0 + (ly / d->row_block) * (long long)d->row_block * d->row_period +
                      (long long)d->row_phase * d->row_block + ly % d->row_block;
        if (y >= d->height) return fail(LRT_E_INVALID, "local rows map outside the image");
    }
    if (d->frame0 < 0 || d->frames < 0) return fail(LRT_E_INVALID, "frame0/frames must be >= 0");
    if ((long long)d->frame0 + d->frames > 0x7fffffffLL) return fail(LRT_E_INVALID, "frame range overflows int");
    if (d->max_depth < 0 || d->max_depth > kMaxDepthSupported)
        return fail(LRT_E_INVALID, "max_depth must be in 0..64");
    return LRT_OK;
}

#ifdef LRT_EXP_WAVETRACE
// Diagnostic build only: per-wave lifetimes of every v0 launch, appended to the binary
// file $LRT_WAVETRACE (u64 nwaves, then nwaves x {t0, t1, hw_id, xcc_id}; t in 100 MHz ticks).
unsigned long long* wavetrace_buffer(size_t waves) {
    static unsigned long long* d = nullptr;
    static size_t cap = 0;
    if (waves > cap) {
        if (d) (void)hipFree(d);
        (void)hipMalloc(&d, sizeof(unsigned long long) * 4 * waves);
        cap = waves;
    }
    return d;
}
void wavetrace_dump(unsigned long long* d, size_t waves, hipStream_t s) {
    const char* path = getenv("LRT_WAVETRACE");
    if (!path) return;
    std::vector<unsigned long long> h(4 * waves);
    (void)hipMemcpyAsync(h.data(), d, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    FILE* f = fopen(path, "ab");
    if (!f) return;
    unsigned long long n = waves;
    fwrite(&n, sizeof(n), 1, f);
    fwrite(h.data(), sizeof(unsigned long long), h.size(), f);
    fclose(f);
}
#endif

#ifdef LRT_EXP_SECSTATS
unsigned long long* secstats_buffer(hipStream_t s) {
    static unsigned long long* d_sec = nullptr;
    if (!d_sec) (void)hipMalloc(&d_sec, sizeof(unsigned long long) * 3 * kSecN * 16);
    (void)hipMemsetAsync(d_sec, 0, sizeof(unsigned long long) * 3 * kSecN * 16, s);
    return d_sec;
}
void secstats_dump(const unsigned long long* d_sec, hipStream_t s) {
        unsigned long long h[3 * kSecN * 16];
        (void)hipMemcpyAsync(h, d_sec, sizeof(h), hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        const char* names[kSecN] = {"hit", "lambert", "shadow", "metal", "dielectric", "post", "fold", "camera", "other",
                                    "hit0", "shadow0"};
        double tot = 0;
        for (int k = 0; k < kSecN; ++k)
            for (int j = 0; j < 16; ++j) tot += (double)h[3 * (k + kSecN * j) + 2];
        for (int k = 0; k < kSecN; ++k) {
            unsigned long long ex = 0, ln = 0, cy = 0;
            for (int j = 0; j < 16; ++j) {
                ex += h[3 * (k + kSecN * j)];
                ln += h[3 * (k + kSecN * j) + 1];
                cy += h[3 * (k + kSecN * j) + 2];
            }
            fprintf(stderr, "secstats %-10s wave-execs %12llu  lanes/exec %6.2f  cycles %5.1f%%  cyc/exec %8.1f\n", names[k], ex,
                    ex ? (double)ln / ex : 0.0, 100.0 * cy / tot, ex ? (double)cy / ex : 0.0);
        }
}
#endif

#ifndef LRT_V0_GRID_MULT
#define LRT_V0_GRID_MULT 1
#endif

// Resident blocks per CU for (kernel, LDS bytes), cached: the query costs host time on
// every launch otherwise.
hipError_t occupancy(int* per_cu, const void* kern, int block, size_t lds) {
    struct Entry { const void* k; int b; size_t l; int v; };
    static Entry cache[32];
    static int n = 0;
    for (int i = 0; i < n; ++i)
        if (cache[i].k == kern && cache[i].b == block && cache[i].l == lds) {
            *per_cu = cache[i].v;
            return hipSuccess;
        }
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, kern, block, lds);
    if (e == hipSuccess && n < 32) cache[n++] = {kern, block, lds, *per_cu};
    return e;
}

#ifndef LRT_MAX_SPLIT
#define LRT_MAX_SPLIT 16
#endif

template <int MAXD, int kSplit, bool kFeat = false>
int launch_depth(KernelArgs a, bool lds, int xc, int rows, hipStream_t s) {
    constexpr int kTileRows = kBlockWavesY * (64 / kSplit / WaveCols(kSplit));
    constexpr int kTileX = WaveCols(kSplit) * kBlockWavesX;
    const long long ntiles = (long long)((xc + kTileX - 1) / kTileX) * ((rows + kTileRows - 1) / kTileRows);
    const size_t stack = sizeof(float4) * kTraceLdsLevels * kBlock + kPowTableBytes + (a.bv.on ? 0 : kRenormBytes);
    const size_t scene = lds ? sizeof(float4) * (4 * (size_t)a.count + (size_t)(a.nlights + 3) / 4 + 1) : 0;
    a.bvh_stack_offset = (int)(stack + scene);
    // v0 sizes the LDS traversal stack to this scene's BVH depth (1000 spheres: ~9
    // levels, 1.2 KB instead of 3 KB per wave -- the difference between 13 and 16 waves/CU)
    const size_t bstk = a.bv.on ? sizeof(unsigned short) * ctx().bvh_stack_levels * kBlock : 0;
    const size_t ldsb = stack + (lds ? scene : 0) + bstk;
    // the reference's own scene size (parallel.cpp:27) gets the unrolled-scan instances
    const bool fixed = lds && !a.bv.on && a.count == kFixedSpheres;
    const void* kern = a.bv.on ? (lds ? (const void*)trace_kernel<MAXD, true, true, kSplit, kFeat>
                                      : (const void*)trace_kernel<MAXD, false, true, kSplit, kFeat>)
                               : (fixed ? (const void*)trace_kernel<MAXD, true, false, kSplit, kFeat, false, kFixedSpheres>
                                  : lds ? (const void*)trace_kernel<MAXD, true, false, kSplit, kFeat>
                                        : (const void*)trace_kernel<MAXD, false, false, kSplit, kFeat>);
    int per_cu = 0;
    hipError_t e = occupancy(&per_cu, kern, kBlock, ldsb);
    if (e != hipSuccess) return hip_fail(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    if (per_cu < 1) return fail(LRT_E_INVALID, "trace_kernel does not fit on a CU");
    // a CU-masked render stream (lrt_stream_create) gets a grid for the CUs it may use:
    // persistent blocks beyond those would only start when others finish
    int cus = ctx().num_cus;
    for (const auto& m : ctx().masked_streams)
        if (m.first == s) cus = m.second;
    // Sample mode (kSamp): several rounds per pixel and fewer than 16 tasks per resident
    // wave (a row shard of a multi-GPU frame at N x spp) -- one task per (tile, round)
    // plus a merge pass, instead of one long task per tile (shard of 8: 7,200 tiles of 2
    // rounds on 4,096 waves). LRT_SAMPLE_MODE=0 turns it off, 2 forces it (A/B, tests).
    const int rounds = (a.frames + kSplit - 1) / kSplit;
    const size_t npix = (size_t)xc * rows;
    bool samp = false;
    if constexpr (!kFeat && kSplit == 1) samp = a.sampOnly && lds && !a.bv.on;
    if constexpr (!kFeat && kSplit >= 4) {
        static int mode = -1;
        if (mode < 0) {
            const char* v = getenv("LRT_SAMPLE_MODE");
            mode = v ? atoi(v) : 1;
        }
        const long long slots = (long long)per_cu * cus;
        samp = mode > 0 && lds && !a.bv.on && rounds >= 2 && npix * (size_t)a.frames * sizeof(float4) <= (2ull << 30) &&
               (mode == 2 || ntiles < 16 * slots);
    }
    if (a.sampOnly && !samp) return fail(LRT_E_INVALID, "colours-only render: needs the LDS linear scan, one frame lane");
    const long long tasks = samp ? ntiles * rounds : ntiles;
    long long blocks = (long long)per_cu * cus * LRT_V0_GRID_MULT;
    // block b serves queue b % kV0Queues: every queue that owns a task needs a block, even
    // on a CU-masked stream left with fewer slots than queues (those blocks start later)
    blocks = std::max(blocks, (long long)kV0Queues);
    if (blocks > tasks) blocks = tasks;
    const dim3 grid((unsigned)blocks);
    if (!a.sampOnly) a.samp = nullptr;
    a.ovf = nullptr;
    a.tiles = ctx().d_tiles + (size_t)(ctx().tiles_next++ % kQueueSlots) * kTileSetU64;
#ifdef LRT_EXP_SECSTATS
    unsigned long long* d_sec = secstats_buffer(s);
    a.wtrace = d_sec;
#endif
#ifdef LRT_EXP_WAVETRACE
    a.wtrace = wavetrace_buffer((size_t)grid.x * (kBlock / 64));
#endif
    if (a.maxDepth > kTraceLdsLevels) {   // per resident thread: bounded by the persistent grid
        const size_t gthreads = (size_t)grid.x * kBlock;
        e = hipMallocAsync((void**)&a.ovf, sizeof(float4) * gthreads * (size_t)(a.maxDepth - kTraceLdsLevels), s);
        if (e != hipSuccess) return hip_fail(e, "hipMallocAsync(trace stack overflow)");
    }
    if constexpr (!kFeat && (kSplit >= 4 || kSplit == 1)) {
        if (samp && a.sampOnly) {   // the caller lerps the planes (render_host's pipeline)
            if (fixed)
                trace_kernel<MAXD, true, false, kSplit, false, true, kFixedSpheres><<<grid, kBlock, ldsb, s>>>(a);
            else
                trace_kernel<MAXD, true, false, kSplit, false, true><<<grid, kBlock, ldsb, s>>>(a);
            e = hipGetLastError();
            if (e != hipSuccess) return hip_fail(e, "trace_kernel (colours) launch");
        } else if (samp) {
            e = hipMallocAsync((void**)&a.samp, sizeof(float4) * npix * (size_t)a.frames, s);
            if (e != hipSuccess) return hip_fail(e, "hipMallocAsync(sample planes)");
            if (fixed)
                trace_kernel<MAXD, true, false, kSplit, false, true, kFixedSpheres><<<grid, kBlock, ldsb, s>>>(a);
            else
                trace_kernel<MAXD, true, false, kSplit, false, true><<<grid, kBlock, ldsb, s>>>(a);
            e = hipGetLastError();
            if (e != hipSuccess) return hip_fail(e, "trace_kernel (samples) launch");
            merge_samples_kernel<<<(unsigned)((npix + 255) / 256), 256, 0, s>>>(a.samp, a.out, a.lerp, (int)npix,
                                                                               a.frame0, a.frames, npix, a, 0);
            e = hipGetLastError();
            if (e != hipSuccess) return hip_fail(e, "merge_samples_kernel launch");
            e = hipFreeAsync(a.samp, s);
            if (e != hipSuccess) return hip_fail(e, "hipFreeAsync(sample planes)");
        }
    }
    if (samp) {
    } else if (a.bv.on) {
        if (lds)
            trace_kernel<MAXD, true, true, kSplit, kFeat><<<grid, kBlock, ldsb, s>>>(a);
        else
            trace_kernel<MAXD, false, true, kSplit, kFeat><<<grid, kBlock, ldsb, s>>>(a);
    } else {
        if (fixed)
            trace_kernel<MAXD, true, false, kSplit, kFeat, false, kFixedSpheres><<<grid, kBlock, ldsb, s>>>(a);
        else if (lds)
            trace_kernel<MAXD, true, false, kSplit, kFeat><<<grid, kBlock, ldsb, s>>>(a);
        else
            trace_kernel<MAXD, false, false, kSplit, kFeat><<<grid, kBlock, ldsb, s>>>(a);
    }
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "trace_kernel launch");
    snprintf(g_last_launch, sizeof(g_last_launch),
             "kernel=trace_kernel maxd=%d lds=%d bvh=%d split=%d samp=%d feat=%d ns=%d grid=%u tasks=%lld per_cu=%d",
             MAXD, lds ? 1 : 0, a.bv.on ? 1 : 0, kSplit, samp ? 1 : 0, kFeat ? 1 : 0, fixed ? kFixedSpheres : 0,
             grid.x, tasks, per_cu);

#ifdef LRT_EXP_WAVETRACE
    wavetrace_dump(a.wtrace, (size_t)grid.x * (kBlock / 64), s);
#endif
#ifdef LRT_EXP_SECSTATS
    secstats_dump(d_sec, s);
#endif
    if (a.ovf) {
        e = hipFreeAsync(a.ovf, s);
        if (e != hipSuccess) return hip_fail(e, "hipFreeAsync(trace stack overflow)");
    }
    return LRT_OK;
}

template <int MAXD>
int launch_split(const KernelArgs& a, bool lds, int xc, int rows, int frames, bool feat, hipStream_t s) {
    if (feat) return launch_depth<MAXD, 1, true>(a, lds, xc, rows, s);
    // one lane per frame of a pixel: the largest power of two <= frames, up to
    // LRT_MAX_SPLIT lanes per pixel. Fewer lanes per pixel than frames means several
    // rounds per wave task, i.e. fewer, longer tasks: with few pixels (one GPU's row shard
    // at 8 GPUs: 115,200 pixels at 32 spp) 7,200 tasks of 8 rounds on 4,096 waves left a
    // 1.7x tail (0.635 ms vs 0.365 for the same rays). Each lane replays its group's lerp
    // chain, so the merge costs kSplit steps per round: 16 measured best (shard of 8:
    // 0.437 ms, 32 lanes: 0.446; config 4 at 64 spp: 457 ms, 64 lanes: 478).
    int split = 1;
    while (split * 2 <= frames && split * 2 <= LRT_MAX_SPLIT) split *= 2;
    switch (split) {
        case 64: return launch_depth<MAXD, (LRT_MAX_SPLIT >= 64 ? 64 : 1)>(a, lds, xc, rows, s);
        case 32: return launch_depth<MAXD, (LRT_MAX_SPLIT >= 32 ? 32 : 1)>(a, lds, xc, rows, s);
        case 16: return launch_depth<MAXD, (LRT_MAX_SPLIT >= 16 ? 16 : 1)>(a, lds, xc, rows, s);
        case 8: return launch_depth<MAXD, (LRT_MAX_SPLIT >= 8 ? 8 : 1)>(a, lds, xc, rows, s);
        case 4: return launch_depth<MAXD, (LRT_MAX_SPLIT >= 4 ? 4 : 1)>(a, lds, xc, rows, s);
        case 2: return launch_depth<MAXD, (LRT_MAX_SPLIT >= 2 ? 2 : 1)>(a, lds, xc, rows, s);
        default: return launch_depth<MAXD, 1>(a, lds, xc, rows, s);
    }
}

// v5 (lrt_pool.h): v0's LDS layout, queues, counters and overflow stack, plus the
// per-block colour slots.
// Heaviest-first tile order for the pool kernel (LRT_POOL_ORDER=0: off). A pool tile is
// 4x a v0 task, and a tile over a glass sphere costs several average ones, so a launch in
// queue order ends with a few waves finishing heavy tiles while the rest of the chip idles
// (profiles/r2_p8). The first launch of a render signature (window, frames, depth, flags,
// camera, scene, tile size) records each tile's cost; once it has finished, the next launch
// of that signature sorts the costs on the host and hands tiles out heaviest first -- the
// classic LPT order -- and so does every later one. Each pixel's result is unchanged: only
// the order in which tiles are taken changes.
// The last kOrderSlots signatures keep their orders, so callers alternating renders (two
// windows, a DrawTest beside a device render) neither start over nor wait. A new view of the
// same geometry (the camera moved, the scene was edited) borrows the newest ready order of
// that geometry for its own recording launch and until its costs are in: its first launch
// already runs heaviest-first by the previous view's measure.
uint64_t fnv(uint64_t h, const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}
bool pool_order_on() {
    static const bool on = [] {
        const char* e = getenv("LRT_POOL_ORDER");
        return !(e && atoi(e) == 0);
    }();
    return on;
}
// Waits until every launch that used entry e has passed it (only those streams' events).
int order_release(Context::TileOrder& e) {
    for (auto& u : e.uses) LRT_HIP(hipEventSynchronize(u.second));
    return LRT_OK;
}
// After a launch on stream s that read e's permutation or wrote its costs.
int order_used(Context::TileOrder& e, hipStream_t s) {
    for (auto& u : e.uses)
        if (u.first == s) {
            LRT_HIP(hipEventRecord(u.second, s));
            return LRT_OK;
        }
    hipEvent_t ev = nullptr;
    LRT_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    e.uses.emplace_back(s, ev);
    LRT_HIP(hipEventRecord(ev, s));
    return LRT_OK;
}
// Picks a's order for this launch: a.perm (null: queue order) and, for the recording launch,
// a.tcost. *users gets the entries whose buffers the launch touches (order_used after it).
hipError_t sort_tiles_desc(const unsigned* cost_in, unsigned* keys_out, const int* ids_in, int* perm_out, int n,
                           void* tmp, size_t* tmp_bytes, hipStream_t s, unsigned end_bit = 32);   // lrt_sort.hip
// LRT_POOL_PROBE: 0 off; 1 (default) a new signature without an order of the same geometry
// to borrow probes its tiles (probe_kernel) and runs its recording launch in the probe's
// order; 2 probes even when it could borrow
int pool_probe_mode() {
    static const int m = [] {
        const char* e = getenv("LRT_POOL_PROBE");
        return e ? atoi(e) : 1;
    }();
    return m;
}
hipError_t fill_iota(int* v, int n, hipStream_t s);

// Sizes entry e for ntiles tiles (at least 65,536, so views of other sizes rarely reallocate).
// Entries are allocated together on first use, so a new view's first launch does not wait
// for hipMalloc.
int order_alloc(Context::TileOrder& e, long long ntiles, hipStream_t s) {
    if (e.cap >= ntiles) return LRT_OK;
    const long long cap = std::max(ntiles, 65536LL);
    size_t tmp = 0;
    LRT_HIP(sort_tiles_desc(nullptr, nullptr, nullptr, nullptr, (int)cap, nullptr, &tmp, s));
    const size_t arr = ((size_t)cap * 4 + 255) & ~(size_t)255;
    if (e.d_base) (void)hipFree(e.d_base);   // (its launches have passed: order_release)
    e.d_base = nullptr;
    e.cap = 0;
    if (hipMalloc(&e.d_base, 4 * arr + tmp) != hipSuccess) {
        e.d_base = nullptr;
        return fail(LRT_E_NOMEM, "hipMalloc(tile order)");
    }
    char* b = static_cast<char*>(e.d_base);
    e.d_cost = reinterpret_cast<unsigned*>(b);
    e.d_keys = reinterpret_cast<unsigned*>(b + arr);
    e.d_ids = reinterpret_cast<int*>(b + 2 * arr);
    e.d_perm = reinterpret_cast<int*>(b + 3 * arr);
    e.d_tmp = b + 4 * arr;
    e.tmp_bytes = tmp;
    LRT_HIP(fill_iota(e.d_ids, (int)cap, s));
    e.cap = cap;
    return LRT_OK;
}

int tile_order(KernelArgs& a, int kPix, long long ntiles, bool& record, Context::TileOrder* users[2], hipStream_t s) {
    record = false;
    users[0] = users[1] = nullptr;
    if (!pool_order_on() || ntiles < 2 * kV0Queues) return LRT_OK;
    Context& c = ctx();
    const int geo[] = {a.width, a.height, a.x0, a.xc, a.y0, a.rows, a.rb, a.rp, a.rph, a.frames, a.maxDepth,
                       a.ndl, a.bv.on, a.count, kPix, a.sph == c.d_sph ? 0 : 1};
    const uint64_t gkey = fnv(1469598103934665603ull, geo, sizeof(geo));
    uint64_t sig = fnv(gkey, &c.scene_version, sizeof(c.scene_version));
    sig = fnv(sig, &a.cam, sizeof(a.cam));
    Context::TileOrder* e = nullptr;
    for (auto& o : c.order)
        if (o.state != 0 && o.sig == sig && o.ntiles == ntiles) e = &o;
    if (!e) {   // a new signature: take a free entry, else the least recently used one
        for (auto& o : c.order)
            if (!e && o.state == 0) e = &o;
        if (!e) {
            e = &c.order[0];
            for (auto& o : c.order)
                if (o.tick < e->tick) e = &o;
        }
        int donor = -1;   // the newest ready order of the same geometry
        for (int i = 0; i < Context::kOrderSlots; ++i) {
            const auto& o = c.order[i];
            if (&o != e && o.state == 2 && o.gkey == gkey && o.ntiles == ntiles &&
                (donor < 0 || o.tick > c.order[donor].tick))
                donor = i;
        }
        if (e->state != 0) {
            // launches that read this entry's permutation (also as a donor) must be done
            // with it; the entries borrowing it lose their donor
            if (int rc = order_release(*e)) return rc;
            for (auto& o : c.order)
                if (o.donor == (int)(e - c.order)) o.donor = -1;
        }
        if (e->cap < ntiles) {
            e->state = 0;
            for (auto& o : c.order)   // the first use sizes every unallocated entry at once
                if (&o == e || (o.cap == 0 && o.state == 0))
                    if (int rc = order_alloc(o, ntiles, s)) return rc;
        }
        if (!e->ev_rec) LRT_HIP(hipEventCreateWithFlags(&e->ev_rec, hipEventDisableTiming));
        e->sig = sig;
        e->gkey = gkey;
        e->ntiles = ntiles;
        // the recording launch writes d_cost and the sort behind it (launch_pool) d_perm:
        // ready for every later launch once ev_rec has passed, which each of them waits for
        e->state = 2;
        e->donor = donor;
        a.tcost = e->d_cost;
        record = true;
        if (donor >= 0) {   // meanwhile the newest order of the same geometry
            users[1] = &c.order[donor];
            LRT_HIP(hipStreamWaitEvent(s, users[1]->ev_rec, 0));
            a.perm = users[1]->d_perm;
            users[1]->tick = ++c.order_tick;
        }
    } else {
        LRT_HIP(hipStreamWaitEvent(s, e->ev_rec, 0));
        a.perm = e->d_perm;
    }
    users[0] = e;
    e->tick = ++c.order_tick;
    return LRT_OK;
}

template <int MAXD, int kPix>
int launch_pool(KernelArgs a, bool lds, int xc, int rows, hipStream_t s) {
    constexpr int TX = PoolTile<kPix>::X, TY = PoolTile<kPix>::Y;
    const long long ntiles = (long long)((xc + TX - 1) / TX) * ((rows + TY - 1) / TY);
    const size_t stack = sizeof(float4) * kTraceLdsLevels * 64 + kPowTableBytes + (a.bv.on ? 0 : kRenormBytes);
    const size_t scene = lds ? sizeof(float4) * (4 * (size_t)a.count + (size_t)(a.nlights + 3) / 4 + 1) : 0;
    a.bvh_stack_offset = (int)(stack + scene);
    const size_t bstk = a.bv.on ? sizeof(unsigned short) * ctx().bvh_stack_levels * 64 : 0;
    const size_t ldsb = stack + scene + bstk;
    const bool fixed = lds && !a.bv.on && a.count == kFixedSpheres;
    const void* kern = a.bv.on ? (lds ? (const void*)pool_kernel<MAXD, true, true, kPix>
                                      : (const void*)pool_kernel<MAXD, false, true, kPix>)
                               : (fixed ? (const void*)pool_kernel<MAXD, true, false, kPix, kFixedSpheres>
                                  : lds ? (const void*)pool_kernel<MAXD, true, false, kPix>
                                        : (const void*)pool_kernel<MAXD, false, false, kPix>);
    int per_cu = 0;
    hipError_t e = occupancy(&per_cu, kern, 64, ldsb);
    if (e != hipSuccess) return hip_fail(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    if (per_cu < 1) return fail(LRT_E_INVALID, "pool_kernel does not fit on a CU");
    int cus = ctx().num_cus;
    for (const auto& m : ctx().masked_streams)
        if (m.first == s) cus = m.second;
    long long blocks = std::max((long long)per_cu * cus, (long long)kV0Queues);   // a block per queue (as v0)
    if (blocks > ntiles) blocks = ntiles;
    const dim3 grid((unsigned)blocks);
    a.ovf = nullptr;
    a.colbuf = nullptr;
    a.tiles = ctx().d_tiles + (size_t)(ctx().tiles_next++ % kQueueSlots) * kTileSetU64;
    {   // waiting lanes that trigger a refill (fold + next samples); LRT_POOL_REFILL_MIN.
        // Measured (profiles/r2_p2): config 3 2.31 -> 2.05 ms/step at 16 (vs 1), config 4 and
        // config 2 neutral
        static int env = -1;
        if (env < 0) {
            const char* v = getenv("LRT_POOL_REFILL_MIN");
            env = v ? atoi(v) : 0;
            if (env <= 0 || env > 64) env = 16;
        }
        a.regenMin = env;
    }
    a.poolSlots = kPix * std::min(a.frames, kPoolSamples / kPix);   // one round's samples
    e = hipMallocAsync((void**)&a.colbuf, sizeof(float4) * (size_t)a.poolSlots * grid.x, s);
    if (e != hipSuccess) return hip_fail(e, "hipMallocAsync(pool colour slots)");
    if (a.maxDepth > kTraceLdsLevels) {
        const size_t gthreads = (size_t)grid.x * 64;
        e = hipMallocAsync((void**)&a.ovf, sizeof(float4) * gthreads * (size_t)(a.maxDepth - kTraceLdsLevels), s);
        if (e != hipSuccess) return hip_fail(e, "hipMallocAsync(trace stack overflow)");
    }
#ifdef LRT_EXP_SECSTATS
    unsigned long long* d_sec = secstats_buffer(s);
    a.wtrace = d_sec;
#endif
#ifdef LRT_EXP_WAVETRACE
    a.wtrace = wavetrace_buffer(grid.x);
#endif
    bool record = false;
    Context::TileOrder* users[2];
    if (int rc = tile_order(a, kPix, ntiles, record, users, s)) return rc;
    bool probed = false;
    if (record && pool_probe_mode() > 0 && (pool_probe_mode() == 2 || !users[1])) {
        // no measured order to go by: probe the tiles' costs, sort them, and let this
        // (recording) launch take its tiles in that order (probe_kernel, lrt_pool.h)
        Context::TileOrder& o = *users[0];
        KernelArgs pa = a;
        pa.bvh_stack_offset = 0;
        const unsigned pblocks = (unsigned)((ntiles + 64 / kProbe - 1) / (64 / kProbe));
        if (a.bv.on) probe_kernel<true><<<pblocks, 64, bstk, s>>>(pa, o.d_cost, (int)ntiles, TX, TY);
        else probe_kernel<false><<<pblocks, 64, 0, s>>>(pa, o.d_cost, (int)ntiles, TX, TY);
        e = hipGetLastError();
        if (e == hipSuccess) {
            probe_order_kernel<<<1, 1024, 0, s>>>(o.d_cost, o.d_perm, (int)ntiles);
            e = hipGetLastError();
        }
        if (e != hipSuccess) {
            o.state = 0;
            return hip_fail(e, "tile cost probe");
        }
        a.perm = o.d_perm;
        users[1] = nullptr;   // (a borrowed order, if any, is not used)
        probed = true;
    }
    if (a.bv.on) {
        if (lds) pool_kernel<MAXD, true, true, kPix><<<grid, 64, ldsb, s>>>(a);
        else pool_kernel<MAXD, false, true, kPix><<<grid, 64, ldsb, s>>>(a);
    } else if (fixed) {
        pool_kernel<MAXD, true, false, kPix, kFixedSpheres><<<grid, 64, ldsb, s>>>(a);
    } else {
        if (lds) pool_kernel<MAXD, true, false, kPix><<<grid, 64, ldsb, s>>>(a);
        else pool_kernel<MAXD, false, false, kPix><<<grid, 64, ldsb, s>>>(a);
    }
    e = hipGetLastError();
    if (e != hipSuccess) {
        if (record) users[0]->state = 0;   // nothing recorded: the entry is free again
        return hip_fail(e, "pool_kernel launch");
    }
    if (record) {   // the costs just recorded, sorted on the device behind the launch
        Context::TileOrder& o = *users[0];
        e = sort_tiles_desc(o.d_cost, o.d_keys, o.d_ids, o.d_perm, (int)ntiles, o.d_tmp, &o.tmp_bytes, s);
        if (e == hipSuccess) e = hipEventRecord(o.ev_rec, s);
        if (e != hipSuccess) {
            o.state = 0;   // no order for this signature: the next launch records again
            return hip_fail(e, "tile order sort");
        }
    }
    for (auto* u : users)
        if (u)
            if (int rc = order_used(*u, s)) return rc;
    // order: 0 queue order (tile order off), 1 recording in queue order, 2 the signature's own
    // sorted order, 3 recording with the order borrowed from the same geometry, 4 recording in
    // the probe's order
    snprintf(g_last_launch, sizeof(g_last_launch),
             "kernel=pool_kernel maxd=%d lds=%d bvh=%d pix=%d ns=%d grid=%u tasks=%lld order=%d per_cu=%d", MAXD,
             lds ? 1 : 0, a.bv.on ? 1 : 0, kPix, fixed ? kFixedSpheres : 0, grid.x, ntiles,
             !users[0] ? 0 : !record ? 2 : probed ? 4 : users[1] ? 3 : 1, per_cu);
#ifdef LRT_EXP_SECSTATS
    secstats_dump(d_sec, s);
#endif
#ifdef LRT_EXP_WAVETRACE
    wavetrace_dump(a.wtrace, grid.x, s);
#endif
    e = hipFreeAsync(a.colbuf, s);
    if (e != hipSuccess) return hip_fail(e, "hipFreeAsync(pool colour slots)");
    if (a.ovf) {
        e = hipFreeAsync(a.ovf, s);
        if (e != hipSuccess) return hip_fail(e, "hipFreeAsync(trace stack overflow)");
    }
    return LRT_OK;
}

// Pixels per pool tile: a round holds kPoolSamples samples, so more frames -> fewer pixels.
// Bigger tiles make bigger pools (a round's tail, its last paths with most lanes idle, is a
// smaller share) but fewer tiles per wave (the launch's tail). 64 px at most by default:
// 128-px tiles (LRT_POOL_PIX_MAX=128; taken only while every resident wave still gets one)
// run config 2 pipelined over two streams at 0.2357/0.2373 ms/step against 0.2465/0.2476 and
// config 3 at 1.942/1.936 against 1.950/1.953, but a launch alone at 0.363-0.412 ms against
// 0.286-0.300 (config 3: 2.47-2.66 ms against 2.07-2.09): the few heavy 128-px tiles set the
// end of a launch that no other launch overlaps (profiles/r3_ag, r3_fin2). 256 px left waves
// idle on config 2 (39.4 vs 46.3 Grays/s, r3_g).
int pool_tiles(int pix, int xc, int rows) {
    const int tx = pix >= 128 ? 16 : pix >= 32 ? 8 : pix >= 8 ? 4 : pix >= 2 ? 2 : 1, ty = pix / tx;
    return ((xc + tx - 1) / tx) * ((rows + ty - 1) / ty);
}
int pool_pixels(int frames, int xc, int rows) {
    static const int cap = [] {   // LRT_POOL_PIX_MAX: largest tile (A/B)
        const char* e = getenv("LRT_POOL_PIX_MAX");
        return e ? atoi(e) : 64;
    }();
    const long long slots = 16LL * ctx().num_cus;   // resident waves (4 per SIMD)
    for (int pix : {256, 128, 64, 32, 16})
        if (cap >= pix && pix * frames <= kPoolSamples && (pix <= 64 || pool_tiles(pix, xc, rows) >= slots))
            return pix;
    return 4 * frames <= kPoolSamples ? 4 : 1;
}
template <int MAXD>
int launch_pool_split(const KernelArgs& a, bool lds, int xc, int rows, int frames, hipStream_t s) {
    switch (pool_pixels(frames, xc, rows)) {
        case 256: return launch_pool<MAXD, 256>(a, lds, xc, rows, s);
        case 128: return launch_pool<MAXD, 128>(a, lds, xc, rows, s);
        case 64: return launch_pool<MAXD, 64>(a, lds, xc, rows, s);
        case 32: return launch_pool<MAXD, 32>(a, lds, xc, rows, s);
        case 16: return launch_pool<MAXD, 16>(a, lds, xc, rows, s);
        case 4: return launch_pool<MAXD, 4>(a, lds, xc, rows, s);
        default: return launch_pool<MAXD, 1>(a, lds, xc, rows, s);
    }
}

// v4 (lrt_wavefront.h): chunks of whole pixels, maxDepth + 1 extend/shade rounds each,
// then the chunk's frame planes merged into the window. Path state is ~100 B + 16 B per
// recursion level per pixel-sample; chunks are sized to a 2 GB budget.
int launch_wavefront(KernelArgs a, bool lds, hipStream_t s) {
    const int frames = a.frames, levels = std::max(1, a.maxDepth);
    const size_t npix = (size_t)a.xc * a.rows;
    const size_t per_path = 4 + 4 * 16 + 16 + 5 * 4 + 16 * (size_t)levels;
    const size_t budget = (size_t)2 << 30;
    size_t cpix = std::max<size_t>(1, budget / (per_path * (size_t)frames));
    cpix = std::min(cpix, npix);
    const size_t C = cpix * (size_t)frames;
    if (C > 0x7fffffff) return fail(LRT_E_INVALID, "wavefront chunk too large");
    // the persistent grid: every wavefront kernel runs B blocks, block j on region j
    const size_t head = kPowTableBytes + kRenormBytes;
    const size_t scene = lds ? sizeof(float4) * (4 * (size_t)a.count + (size_t)(a.nlights + 3) / 4 + 1) : 0;
    const size_t bstk = a.bv.on ? sizeof(unsigned short) * ctx().bvh_stack_levels * kWfBlock : 0;
    const size_t ldsb = head + scene + bstk;
    const bool bvh = a.bv.on != 0, fixed = lds && !bvh && a.count == kFixedSpheres;
    const void* kx = bvh ? (const void*)wf_extend<true, 0> : fixed ? (const void*)wf_extend<false, kFixedSpheres>
                                                                   : (const void*)wf_extend<false, 0>;
    const void* ks = bvh ? (const void*)wf_shade<true, 0> : fixed ? (const void*)wf_shade<false, kFixedSpheres>
                                                                  : (const void*)wf_shade<false, 0>;
    int per_cu = 0, per_cu_s = 0;
    hipError_t e = occupancy(&per_cu, kx, kWfBlock, ldsb);
    if (e == hipSuccess) e = occupancy(&per_cu_s, ks, kWfBlock, ldsb);
    if (e != hipSuccess) return hip_fail(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    per_cu = std::min(per_cu, per_cu_s);
    if (per_cu < 1) return fail(LRT_E_INVALID, "wavefront kernels do not fit on a CU");
    const int B = per_cu * ctx().num_cus;
    const size_t cnt_bytes = sizeof(unsigned int) * 4 * (size_t)(a.maxDepth + 2) * B;
    const size_t need = per_path * (C + (size_t)B) + cnt_bytes + 256 * 12;
    auto& wf = ctx().wf;
    if (wf.bytes < need) {
        if (wf.buf) (void)hipFree(wf.buf);
        wf.buf = nullptr;
        wf.bytes = 0;
        if (hipMalloc(&wf.buf, need) != hipSuccess) return fail(LRT_E_NOMEM, "hipMalloc(wavefront state)");
        wf.bytes = need;
    }
    if (!wf.rayp) {
        LRT_HIP(hipMalloc(&wf.rayp, sizeof(unsigned long long) * kV0Queues * kCtrStride));
        LRT_HIP(hipMemset(wf.rayp, 0, sizeof(unsigned long long) * kV0Queues * kCtrStride));
    }
    WfArgs w;
    w.a = a;
    char* b = static_cast<char*>(wf.buf);
    auto take = [&](size_t bytes) { void* p = b; b += (bytes + 255) / 256 * 256; return p; };
    const size_t qslots = C + (size_t)B;   // B regions of R0 = ceil(C / B) state slots
    w.o = static_cast<float4*>(take(16 * qslots));
    w.d = static_cast<float4*>(take(16 * qslots));
    w.sl = static_cast<float4*>(take(16 * qslots));
    w.lit = static_cast<float4*>(take(16 * qslots));
    w.samp = static_cast<float4*>(take(16 * C));
    w.stack = static_cast<float4*>(take(16 * qslots * (size_t)levels));
    w.rng = static_cast<uint32_t*>(take(4 * qslots));
    w.qa[0] = static_cast<uint32_t*>(take(4 * qslots));
    w.qa[1] = static_cast<uint32_t*>(take(4 * qslots));
    for (int t = 0; t < 3; ++t) w.qm[t] = static_cast<uint32_t*>(take(4 * qslots));
    w.cnt = static_cast<unsigned int*>(take(cnt_bytes));
    w.rayp = wf.rayp;
    // LDS: [powf tables][renormalize table][scene if staged][bvh traversal stack]
    w.lds = lds ? 1 : 0;
    w.bstk_off = (int)(head + scene);
    const dim3 grid((unsigned)B), block(kWfBlock);
    for (size_t pix0 = 0; pix0 < npix; pix0 += cpix) {
        const size_t cp = std::min(cpix, npix - pix0);
        w.pix0 = (int)pix0;
        w.cpix = (int)cp;
        w.C = (int)(cp * (size_t)frames);
        w.R0 = (int)((w.C + B - 1) / B);
        w.Cs = w.R0 * B;
        LRT_HIP(hipMemsetAsync(w.cnt, 0, cnt_bytes, s));
        wf_camera<<<grid, block, kRenormBytes, s>>>(w);
        for (int it = 0; it <= a.maxDepth; ++it) {
            if (bvh) {
                wf_extend<true, 0><<<grid, block, ldsb, s>>>(w, it);
                wf_shade<true, 0><<<grid, block, ldsb, s>>>(w, it);
            } else if (fixed) {
                wf_extend<false, kFixedSpheres><<<grid, block, ldsb, s>>>(w, it);
                wf_shade<false, kFixedSpheres><<<grid, block, ldsb, s>>>(w, it);
            } else {
                wf_extend<false, 0><<<grid, block, ldsb, s>>>(w, it);
                wf_shade<false, 0><<<grid, block, ldsb, s>>>(w, it);
            }
        }
        merge_samples_kernel<<<(unsigned)((cp + 255) / 256), 256, 0, s>>>(w.samp, a.out + pix0, a.lerp, (int)cp,
                                                                         a.frame0, a.frames, cp, a, (int)pix0);
        e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(e, "wavefront launch");
    }
    snprintf(g_last_launch, sizeof(g_last_launch), "kernel=wf_extend lds=%d bvh=%d grid=%u", lds ? 1 : 0, bvh ? 1 : 0, grid.x);
    wf_rays_collect<<<1, 64, 0, s>>>(wf.rayp, a.rays);
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "wavefront ray collect");
    return LRT_OK;
}

int auto_kernel(const KernelArgs& a, const lrt_render_desc* d, bool feat);

// colours_out (render_host's pipeline): no lerp -- frame f's sample colours go to plane
// f - frame0 of colours_out (x_count * row_count float4 each) and d_buf is not touched.
// frame (lrt_render_device_to_frame): every finished pixel is stored there too, at its global
// row -- the whole width x height RGBA frame, possibly another device's memory.
int render_device(const lrt_render_desc* d, float* d_buf, unsigned long long* d_rays, const lrt_features* feat,
                  hipStream_t s, float4* colours_out = nullptr, float* frame = nullptr) {
    int rc = validate(d);
    if (rc) return rc;
    if (!ctx().ready) return fail(LRT_E_STATE, "lrt_initialize() has not been called");
    if (!d_buf || !d_rays) return fail(LRT_E_INVALID, "device buffer / ray counter is NULL");
    if (d->x_count == 0 || d->row_count == 0 || d->frames == 0) return LRT_OK;
    KernelArgs a;
    const lrt_camera& c = d->camera;
    a.cam.origin = f3(c.origin.x, c.origin.y, c.origin.z);
    a.cam.a = f3(c.a.x, c.a.y, c.a.z);
    a.cam.u = f3(c.u.x, c.u.y, c.u.z);
    a.cam.r = f3(c.r.x, c.r.y, c.r.z);
    a.cam.llc = f3(c.lowerLeftCorner.x, c.lowerLeftCorner.y, c.lowerLeftCorner.z);
    a.cam.horiz = f3(c.horizontalVec.x, c.horizontalVec.y, c.horizontalVec.z);
    a.cam.vert = f3(c.verticalVec.x, c.verticalVec.y, c.verticalVec.z);
    a.cam.lensRadius = c.lensRadius;
    a.sph = ctx().d_sph;
    a.mats = ctx().d_mats;
    a.lights = ctx().d_lights;
    a.count = ctx().count;
    a.nlights = ctx().nlights;
    a.width = d->width;
    a.height = d->height;
    a.x0 = d->x0;
    a.xc = d->x_count;
    a.y0 = d->y0;
    a.rows = d->row_count;
    a.rb = d->row_block;
    a.rp = d->row_period;
    a.rph = d->row_phase;
    a.frame0 = d->frame0;
    a.frames = d->frames;
    a.maxDepth = d->max_depth;
    a.out = reinterpret_cast<float4*>(d_buf);
    a.rays = d_rays;
    a.ndl = (d->flags & LRT_F_NO_DOUBLE_LIGHT) ? 1 : 0;
    bool want_feat = false;
    {
        float* const fp[6] = {feat ? feat->normal : nullptr,    feat ? feat->world_pos : nullptr,
                              feat ? feat->albedo : nullptr,    feat ? feat->color_std : nullptr,
                              feat ? feat->normal_std : nullptr, feat ? feat->world_pos_std : nullptr};
        for (int k = 0; k < 6; ++k) {
            a.feat[k] = reinterpret_cast<float4*>(fp[k]);
            want_feat = want_feat || fp[k] != nullptr;
        }
        a.featMax = feat ? feat->max_frame : -1;
    }
    a.bv.nodes = ctx().d_bvh_nodes;
    a.bv.lsph = ctx().d_bvh_lsph;
    a.bv.lid = ctx().d_bvh_lid;
    a.bv.margin = ctx().bvh_margin;
    a.bv.on = (ctx().bvh_on && !(d->flags & LRT_F_NO_BVH)) ? 1 : 0;
    a.bv.nnodes = ctx().bvh_nodes;
    a.bv.big0 = ctx().bvh_big0;
    a.bv.nbig = ctx().bvh_nbig;
    a.bvh_stack_offset = 0;
    const bool lds = !(d->flags & LRT_F_SCENE_GLOBAL) &&
                     sizeof(float4) * (kTraceLdsLevels * kBlock + 4 * (size_t)a.count + a.nlights / 4 + 1) <= 64 * 1024;
    // Kernel policy (auto_kernel, measured): v5 (pool) for calls with >= 4 frames and >= 2
    // tiles per resident wave, v0 otherwise; v4 (wavefront) stays selectable for A/B. The
    // round-1 per-lane state machines (v1/v2/v2s) and round-1's v3 regeneration kernel (slower
    // than v0 or v5 on every config) were removed: their flags are rejected.
    a.regenMin = 0;
    a.lerp = ctx().d_lerp;
    a.colbuf = nullptr;
    a.poolSlots = 0;
    a.perm = nullptr;
    a.tcost = nullptr;
    a.samp = colours_out;
    a.sampOnly = colours_out ? 1 : 0;
    a.frame = reinterpret_cast<float4*>(frame);
    if (frame && (want_feat || colours_out))
        return fail(LRT_E_INVALID, "a frame destination is for plain renders (no features, no colours-only)");
    if (colours_out) {   // v0, one frame lane per pixel, sample mode
        if (want_feat || !lds || a.bv.on) return fail(LRT_E_INVALID, "colours-only render: LDS linear-scan scenes only");
        if (d->max_depth <= 8) return launch_depth<8, 1>(a, lds, d->x_count, d->row_count, s);
        return launch_depth<64, 1>(a, lds, d->x_count, d->row_count, s);
    }
    if (d->flags & (LRT_F_V1 | LRT_F_V2S | LRT_F_V2 | LRT_F_V3))
        return fail(LRT_E_INVALID, "LRT_F_V1/LRT_F_V2S/LRT_F_V2/LRT_F_V3 kernels were removed (the default picks v0 or v5)");
    int kflags = d->flags & (LRT_F_SIMPLE | LRT_F_WAVEFRONT | LRT_F_POOL);
    if (kflags == 0) kflags = auto_kernel(a, d, want_feat);
    if (want_feat && !(kflags & LRT_F_SIMPLE))
        return fail(LRT_E_INVALID, "features are implemented by the v0 kernel only");
    if (kflags & LRT_F_WAVEFRONT) return launch_wavefront(a, lds, s);
    if (kflags & LRT_F_POOL) {
        a.colbuf = nullptr;
        if (d->max_depth <= 8) return launch_pool_split<8>(a, lds, d->x_count, d->row_count, d->frames, s);
        return launch_pool_split<64>(a, lds, d->x_count, d->row_count, d->frames, s);
    }
    if (d->max_depth <= 8) return launch_split<8>(a, lds, d->x_count, d->row_count, d->frames, want_feat, s);
    // depth 9..64: one instance (MAXD only decides whether stack levels beyond the 8 in LDS
    // exist; 20 and 64 compiled to the same code)
    return launch_split<64>(a, lds, d->x_count, d->row_count, d->frames, want_feat, s);
}

// The library's kernel policy (measured, profiles/r2_p2, r2_p9, r3_t): the pool kernel (v5) given
// at least 4 frames and a tile per resident wave -- BVH scenes (config 4: 223 vs 303
// ms, config 5), bounce budgets above 8 (config 3: 2.45 vs 2.87 ms) and, with its
// heaviest-first tile order (tile_order), the 8-bounce default scene too (config 2: 0.254 vs
// 0.289 ms/step, 0.297 vs 0.329 ms for a launch alone); v0 otherwise (few pixels with many
// frames, a GPU's row shard, take v0's frame lanes and sample mode; features are v0's).
int auto_kernel(const KernelArgs& a, const lrt_render_desc* d, bool feat) {
    if (feat || d->frames < 4) return LRT_F_SIMPLE;
    if (!(a.bv.on || d->max_depth > 8) && !pool_order_on()) return LRT_F_SIMPLE;
    const int pix = pool_pixels(d->frames, d->x_count, d->row_count);
    const long long tiles = pool_tiles(pix, d->x_count, d->row_count);
    const long long slots = 16LL * ctx().num_cus;   // resident waves (4 per SIMD)
    // at least a tile per resident wave: config 2's row shard of 2 (7,200 tiles) runs 0.1316 ms
    // on the pool kernel against 0.1473 on v0; a shard of 4 (3,680 tiles) 0.1456 against 0.0773
    // (profiles/r3_t)
    return tiles >= slots ? LRT_F_POOL : LRT_F_SIMPLE;
}

int ensure_frame(size_t bytes) {
    if (ctx().frame_bytes >= bytes) return LRT_OK;
    if (ctx().d_frame) (void)hipFree(ctx().d_frame);
    ctx().d_frame = nullptr;
    ctx().frame_bytes = 0;
    if (hipMalloc(&ctx().d_frame, bytes) != hipSuccess) return fail(LRT_E_NOMEM, "hipMalloc(frame) failed");
    ctx().frame_bytes = bytes;
    return LRT_OK;
}

// The device address of buf when it is page-locked host memory (hipHostMalloc /
// hipHostRegister, e.g. a torch pin_memory tensor), else nullptr.
float* host_pinned(float* buf) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, buf) != hipSuccess) {
        (void)hipGetLastError();   // pageable memory: clear the error so no later check sees it
        return nullptr;
    }
    if (at.type != hipMemoryTypeHost) return nullptr;
    return at.devicePointer ? (float*)at.devicePointer : buf;
}

// Registration cache for pageable DrawTest buffers. The reference's caller allocates its
// backbuffer with `new float[]` once (main.cpp:40) and hands the same pointer to every
// DrawTest (main.cpp:165); pageable memory can only be staged (H2D + render + D2H: 0.77 ms
// per 1280x720 frame). A pageable buffer seen by two consecutive lrt_draw_test
// calls is page-locked in place (hipHostRegister, portable to every device in use) and from
// then on takes the page-locked paths (pipelined DMA + lerp written over PCIe: 0.52 ms).
// A registered range must not be freed while registered -- the GPU would later address
// pages the process no longer maps -- so the contract is DrawTest's own (one buffer for the
// run): lrt_host_unregister drops one before the caller frees it (the Python binding does it
// when the array dies), lrt_shutdown drops all, at most kHostRegs stay registered (least
// recently used dropped first). lrt_render_host never registers. LRT_HOST_REGISTER=0: off.
struct HostReg {
    void* p = nullptr;
    size_t bytes = 0;
    unsigned long long tick = 0;
};
constexpr int kHostRegs = 8;
HostReg g_host_regs[kHostRegs];
unsigned long long g_host_reg_tick = 0;
HostReg g_host_last;   // the last pageable buffer rendered (registered when seen again)

bool host_register_on() {
    static const bool on = [] {
        const char* e = getenv("LRT_HOST_REGISTER");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

int host_unregister(void* p) {
    for (auto& r : g_host_regs)
        if (r.p == p) {
            const hipError_t e = hipHostUnregister(r.p);
            r = HostReg();
            if (e != hipSuccess) return hip_fail(e, "hipHostUnregister");
            return LRT_OK;
        }
    return fail(LRT_E_INVALID, "not a buffer the library registered");
}

bool host_registered_here(const void* p) {
    for (const auto& r : g_host_regs)
        if (r.p == p) return true;
    return false;
}

// The device address of pageable buf once it is registered (see above), else nullptr.
float* host_register(float* buf, size_t bytes) {
    if (!host_register_on()) return nullptr;
    const bool again = g_host_last.p == buf && g_host_last.bytes == bytes;
    g_host_last.p = buf;
    g_host_last.bytes = bytes;
    if (!again) return nullptr;
    HostReg* slot = &g_host_regs[0];
    for (auto& r : g_host_regs)
        if (r.tick < slot->tick) slot = &r;
    if (slot->p) (void)host_unregister(slot->p);
    if (hipHostRegister(buf, bytes, hipHostRegisterPortable | hipHostRegisterMapped) != hipSuccess) {
        (void)hipGetLastError();   // e.g. overlaps a registered range: stay on the staged path
        return nullptr;
    }
    slot->p = buf;
    slot->bytes = bytes;
    slot->tick = ++g_host_reg_tick;
    return host_pinned(buf);
}

// Page-locked host backbuffers are rendered in place (zero copy): the kernel's 16 B read
// and 16 B write per pixel cross PCIe inside the launch instead of a staging copy either
// side of it (DrawTest at 1280x720: 0.66 ms per frame vs 0.77 staged; staging in row chunks
// on copy streams measured 0.84 ms at 4 chunks -- per-chunk launch tails and cross-stream
// waits; staging only the previous values and letting the kernel write the host pixels
// measured 0.64 ms, within noise of this). LRT_HOST_ZEROCOPY=0 stages them like pageable memory.
bool host_zero_copy() {
    static const bool on = [] {
        const char* e = getenv("LRT_HOST_ZEROCOPY");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

// The pipelined host path for page-locked backbuffers (lrt_draw_test at 1280x720 is
// PCIe-bound). The sample colours do not depend on the buffer's previous values -- only the
// lerp does (parallel.cpp:282) -- so the colours are rendered into device memory while the
// previous values travel host -> device by DMA (LRT_HOST_CHUNKS row chunks on a copy
// stream); each chunk's lerp runs once its copy lands and writes the result straight into
// the caller's pixels over PCIe, while the next chunk's copy comes the other way. Measured
// alternatives (profiles/r2_p2): zero copy for the whole render (kernel reads and writes
// over PCIe, 0.66 ms; GPU-initiated reads and writes share ~64 GB/s); render + one
// streaming zero-copy lerp (0.70 ms); DMA both ways in 8 chunks (0.72 ms: ~20 us per copy
// command, and D2H ran as blit kernels). Pageable buffers stay staged (their async copies
// go through bounce buffers: 1.2 ms pipelined vs 0.77 staged). LRT_HOST_PIPELINE=0: off.
bool host_pipeline(const lrt_render_desc* d, size_t bytes) {
    static const int mode = [] {
        const char* e = getenv("LRT_HOST_PIPELINE");
        return e ? atoi(e) : 1;
    }();
    const bool bvh = ctx().bvh_on && !(d->flags & LRT_F_NO_BVH);
    const bool lds = !(d->flags & LRT_F_SCENE_GLOBAL) &&
                     sizeof(float4) * (kTraceLdsLevels * kBlock + 4 * (size_t)ctx().count + ctx().nlights / 4 + 1) <=
                         64 * 1024;
    const int kflags = d->flags & (LRT_F_SIMPLE | LRT_F_WAVEFRONT | LRT_F_POOL);
    return mode != 0 && d->frames <= 4 && bytes * (size_t)d->frames <= (256u << 20) && !bvh && lds &&
           (kflags == 0 || kflags == LRT_F_SIMPLE) && !(d->flags & LRT_F_NO_DOUBLE_LIGHT) &&
           d->row_count >= Context::kHostChunks;
}

// Row chunks of the DMA copy (LRT_HOST_CHUNKS, 1..8; default 4 for DrawTest's look-ahead calls,
// whose lerps follow the copy chunk by chunk: 0.47 vs 0.50 ms at 2; 2 otherwise, where the
// render sets the pace: 0.53 vs 0.54 ms at 4 -- profiles/r3_m, r3_o).
int host_chunks(bool lookahead) {
    static const int k = [] {
        const char* e = getenv("LRT_HOST_CHUNKS");
        const int v = e ? atoi(e) : 0;
        return v < 0 ? 1 : v > Context::kHostChunks ? Context::kHostChunks : v;
    }();
    return k > 0 ? k : lookahead ? 4 : 2;
}

// lrt_draw_test's look-ahead (LRT_DRAW_LOOKAHEAD, default on). DrawTest's colours depend on
// frameCount, the size and the scene only (parallel.cpp:297-323: `time` is unused, the camera
// is rebuilt from the size), and the reference's caller asks for frameCount + 1 next
// (main.cpp:165,187). So a pipelined DrawTest call also renders the colours of the next
// frame, on a stream of their own that runs beside this call's DMA and PCIe-write lerps (a
// hit: from the call's start; a miss: after its own render), CU-masked so that the lerps
// still find CUs (LRT_LOOKAHEAD_RESERVED, default 32 = 4 per XCD; 0-32 within 0.01 ms pinned,
// 32 best pageable: profiles/r3_o); the call returns once its
// own work is done. A later call asking for exactly that render (desc and scene version
// compared) lerps those colours and skips its render, so the render leaves the critical
// path (DMA in -> lerp -> PCIe out); any other call renders as before. Same kernel, same
// seeds: the same bits. Two colour buffers alternate (one read by this call's lerps, the
// other written by the next look-ahead).
bool draw_lookahead_on() {
    static const bool on = [] {
        const char* e = getenv("LRT_DRAW_LOOKAHEAD");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

int lookahead_reserved_cus() {
    static const int k = [] {
        const char* e = getenv("LRT_LOOKAHEAD_RESERVED");
        return e ? atoi(e) : 32;
    }();
    return k;
}

// The lerp grid: a few blocks per CU, each striding over the chunk (posted PCIe writes need
// no more in flight; a full grid would wait for CUs behind the look-ahead render)
unsigned merge_blocks(size_t n) {
    const size_t want = (n + 255) / 256, cap = (size_t)4 * ctx().num_cus;
    return (unsigned)std::max<size_t>(1, std::min(want, cap));
}

int render_host_pipelined(const lrt_render_desc* d, float* buf, float* hdev, size_t bytes, long long* out_rays,
                          bool lookahead, int* ahead_state) {
    hipStream_t s = ctx().stream;
    Context::Lookahead& la = ctx().ahead;
    if (!ctx().s_in) {
        LRT_HIP(hipStreamCreateWithFlags(&ctx().s_in, hipStreamNonBlocking));
        for (int c = 0; c < Context::kHostChunks; ++c)
            LRT_HIP(hipEventCreateWithFlags(&ctx().ev_in[c], hipEventDisableTiming));
        LRT_HIP(hipEventCreateWithFlags(&ctx().ev_ret, hipEventDisableTiming));
    }
    const size_t cbytes = bytes * (size_t)d->frames;
    // a hit: the look-ahead rendered exactly this (this call's lerps wait for its event)
    const bool hit = la.on && la.scene_version == ctx().scene_version && memcmp(&la.d, d, sizeof(*d)) == 0;
    la.on = false;
    *ahead_state = hit ? 1 : 0;
    if (!hit && ctx().col_bytes < cbytes) {
        if (ctx().d_col) (void)hipFree(ctx().d_col);
        ctx().d_col = nullptr;
        ctx().col_bytes = 0;
        if (hipMalloc(&ctx().d_col, cbytes) != hipSuccess) return fail(LRT_E_NOMEM, "hipMalloc(sample colours)");
        ctx().col_bytes = cbytes;
    }
    const bool ahead_on = lookahead && draw_lookahead_on() && d->frames == 1 && d->frame0 < INT_MAX - 1;
    const int K = host_chunks(ahead_on || hit), rows = d->row_count, xc = d->x_count;
    const size_t npix = (size_t)xc * rows;
    auto chunk = [&](int c, size_t& p0, size_t& n) {   // chunk c: rows [c rows / K, (c + 1) rows / K)
        const size_t r0 = (size_t)rows * c / K, r1 = (size_t)rows * (c + 1) / K;
        p0 = r0 * xc;
        n = (r1 - r0) * xc;
    };
    for (int c = 0; c < K; ++c) {   // previous values, host -> device (DMA), beside the render
        size_t p0, n;
        chunk(c, p0, n);
        LRT_HIP(hipMemcpyAsync(ctx().d_frame + 4 * p0, buf + 4 * p0, n * 16, hipMemcpyHostToDevice, ctx().s_in));
        LRT_HIP(hipEventRecord(ctx().ev_in[c], ctx().s_in));
    }
    float4* col = hit ? la.col[la.cur] : ctx().d_col;
    unsigned long long* d_rays = hit ? la.d_rays + la.cur : ctx().d_rays;
    if (hit) {
        LRT_HIP(hipStreamWaitEvent(s, la.ev, 0));
    } else {
        LRT_HIP(hipMemsetAsync(d_rays, 0, sizeof(unsigned long long), s));
        int rc = render_device(d, ctx().d_frame, d_rays, nullptr, s, col);
        if (rc) {
            (void)hipStreamSynchronize(ctx().s_in);
            return rc;
        }
    }
    if (ahead_on) {
        // the next frame's colours into the buffer pair this call does not read
        const int nx = hit ? la.cur ^ 1 : la.cur;
        lrt_render_desc nd = *d;
        nd.frame0 = d->frame0 + 1;
        bool ok = true;
        if (!la.stream) {
            const int n = ctx().num_cus, keep = std::max(1, n - std::max(0, lookahead_reserved_cus()));
            std::vector<uint32_t> mask((size_t)(n + 31) / 32, 0u);
            for (int c = 0; c < keep; ++c) mask[c / 32] |= 1u << (c % 32);   // spread over XCDs (c % 8)
            ok = hipExtStreamCreateWithCUMask(&la.stream, (uint32_t)mask.size(), mask.data()) == hipSuccess &&
                 hipEventCreateWithFlags(&la.ev, hipEventDisableTiming) == hipSuccess &&
                 hipEventCreateWithFlags(&la.ev_render, hipEventDisableTiming) == hipSuccess;
            if (ok) ctx().masked_streams.emplace_back(la.stream, keep);
        }
        if (ok && la.bytes[nx] < cbytes) {
            if (la.col[nx]) (void)hipFree(la.col[nx]);
            la.col[nx] = nullptr;
            la.bytes[nx] = 0;
            ok = hipMalloc(&la.col[nx], cbytes) == hipSuccess;
            if (ok) la.bytes[nx] = cbytes;
        }
        if (ok && !la.d_rays) ok = hipMalloc(&la.d_rays, 2 * sizeof(unsigned long long)) == hipSuccess;
        // a miss: after this call's own render (the two would share the CUs it needs)
        if (ok && !hit)
            ok = hipEventRecord(la.ev_render, s) == hipSuccess && hipStreamWaitEvent(la.stream, la.ev_render, 0) == hipSuccess;
        if (ok) ok = hipMemsetAsync(la.d_rays + nx, 0, sizeof(unsigned long long), la.stream) == hipSuccess;
        char keep[sizeof(g_last_launch)];   // the launch string stays this call's
        memcpy(keep, g_last_launch, sizeof(keep));
        if (ok) ok = render_device(&nd, ctx().d_frame, la.d_rays + nx, nullptr, la.stream, la.col[nx]) == LRT_OK;
        memcpy(g_last_launch, keep, sizeof(keep));
        if (ok) ok = hipEventRecord(la.ev, la.stream) == hipSuccess;
        if (ok) {
            la.on = true;
            la.cur = nx;
            la.d = nd;
            la.scene_version = ctx().scene_version;
        } else {
            (void)hipGetLastError();   // no look-ahead: the next call renders for itself
        }
    }
    for (int c = 0; c < K; ++c) {   // each chunk's lerp once its values are in, written to the host pixels
        size_t p0, n;
        chunk(c, p0, n);
        LRT_HIP(hipStreamWaitEvent(s, ctx().ev_in[c], 0));
        merge_to_host_kernel<<<merge_blocks(n), 256, 0, s>>>(
            col + p0, reinterpret_cast<const float4*>(ctx().d_frame) + p0, reinterpret_cast<float4*>(hdev) + p0,
            ctx().d_lerp, (int)n, d->frame0, d->frames, npix);
        LRT_HIP(hipGetLastError());
    }
    unsigned long long rays = 0;
    LRT_HIP(hipMemcpyAsync(&rays, d_rays, sizeof(rays), hipMemcpyDeviceToHost, s));
    LRT_HIP(hipEventRecord(ctx().ev_ret, s));
    LRT_HIP(hipEventSynchronize(ctx().ev_ret));
    if (out_rays) *out_rays = (long long)rays;
    return LRT_OK;
}

// Makes context k the one ctx() returns and its device the calling thread's current one, for
// the scope's lifetime (both restored after).
struct DeviceScope {
    int prev_cur, prev_dev = -1;
    explicit DeviceScope(int k) : prev_cur(g_cur) {
        g_cur = k;
        int dev = 0;
        if (hipGetDevice(&dev) == hipSuccess && dev != g_devs[k].device) {
            prev_dev = dev;
            (void)hipSetDevice(g_devs[k].device);
        }
    }
    ~DeviceScope() {
        if (prev_dev >= 0) (void)hipSetDevice(prev_dev);
        g_cur = prev_cur;
    }
};

int ensure_buffer(float*& p, size_t& have, size_t bytes, const char* what) {
    if (have >= bytes) return LRT_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    have = 0;
    if (hipMalloc(&p, bytes) != hipSuccess) return fail(LRT_E_NOMEM, std::string("hipMalloc(") + what + ")");
    have = bytes;
    return LRT_OK;
}

// One host render split over the g_ndev devices of lrt_initialize_devices (BASELINE config 5:
// "row-tiled across 8xMI355X with RCCL gather over xGMI"). The caller's rows are dealt in
// blocks of g_multi.row_block rows round-robin (row-block-cyclic: contiguous bands are
// imbalanced); device k
//   1. receives the previous values of its rows from the caller's buffer (one strided DMA),
//   2. renders them densely into its shard buffer (lrt_render_desc's row map: row_period =
//      N, row_phase = k; any kernel the policy picks),
// then ONE collective brings the shards to device 0: a grouped ncclGather over RCCL
// (rccl.h:745) when the devices are distinct, device-to-device copies when a device is
// listed twice (RCCL refuses two ranks on one GPU: the 1-GPU rehearsal); device 0 assembles
// the frame (unshard_kernel) and copies it to the caller. Per-pixel seeds make the frame
// bit-identical to a 1-device render for any N and block size.
int render_host_multi_enqueue(const lrt_render_desc* d, float* buf, size_t bytes, unsigned long long* rays);
int render_host_multi(const lrt_render_desc* d, float* buf, size_t bytes, long long* out_rays) {
    std::vector<unsigned long long> rays(g_ndev, 0ull);
    const int rc = render_host_multi_enqueue(d, buf, bytes, rays.data());
    long long total = 0;
    for (int k = 0; k < g_ndev; ++k) {   // also after a failure: nothing may still write `rays`
        DeviceScope ds(k);
        const hipError_t e = hipStreamSynchronize(ctx().stream);
        if (e != hipSuccess && rc == LRT_OK) return hip_fail(e, "hipStreamSynchronize(multi-device render)");
        total += (long long)rays[k];
    }
    if (rc) return rc;
    snprintf(g_last_launch + strlen(g_last_launch), sizeof(g_last_launch) - strlen(g_last_launch),
             " devices=%d exchange=%s row_block=%d", g_ndev, g_multi.rccl ? "rccl" : "copy", g_multi.row_block);
    if (out_rays) *out_rays = total;
    return LRT_OK;
}
int render_host_multi_enqueue(const lrt_render_desc* d, float* buf, size_t bytes, unsigned long long* rays) {
    const int N = g_ndev, b = g_multi.row_block, xc = d->x_count, rows = d->row_count;
    const size_t rowBytes = (size_t)xc * 16;
    const int maxRows = lrt_shard_rows(rows, b, N, 0);
    const size_t shardBytes = (size_t)maxRows * rowBytes;
    for (int k = 0; k < N; ++k) {
        DeviceScope ds(k);
        Context& c = ctx();
        if (int rc = ensure_buffer(c.d_shard, c.shard_bytes, shardBytes, "shard")) return rc;
        if (!c.ev_done) LRT_HIP(hipEventCreateWithFlags(&c.ev_done, hipEventDisableTiming));
        const int rk = lrt_shard_rows(rows, b, N, k);
        if (rk > 0) {
            // shard row j is the caller's row (j / b) * b * N + k * b + j % b: whole blocks
            // are one 2D copy (pitch N blocks), a last partial block one more
            const int full = rk / b, tail = rk % b;
            const size_t blk = (size_t)b * rowBytes;
            const char* src = reinterpret_cast<const char*>(buf) + (size_t)k * blk;
            if (full > 0)
                LRT_HIP(hipMemcpy2DAsync(c.d_shard, blk, src, blk * N, blk, (size_t)full, hipMemcpyHostToDevice,
                                         c.stream));
            if (tail > 0)
                LRT_HIP(hipMemcpyAsync(reinterpret_cast<char*>(c.d_shard) + (size_t)full * blk,
                                       src + (size_t)full * blk * N, (size_t)tail * rowBytes, hipMemcpyHostToDevice,
                                       c.stream));
        }
        LRT_HIP(hipMemsetAsync(c.d_rays, 0, sizeof(unsigned long long), c.stream));
        lrt_render_desc sd = *d;
        sd.row_count = rk;
        sd.row_block = b;
        sd.row_period = N;
        sd.row_phase = k;
        if (int rc = render_device(&sd, c.d_shard, c.d_rays, nullptr, c.stream)) return rc;
        LRT_HIP(hipMemcpyAsync(&rays[k], c.d_rays, sizeof(unsigned long long), hipMemcpyDeviceToHost, c.stream));
        LRT_HIP(hipEventRecord(c.ev_done, c.stream));
    }
    {   // the exchange: every shard into device 0's gather buffer
        DeviceScope ds0(0);
        Context& c0 = ctx();
        if (int rc = ensure_buffer(c0.d_gath, c0.gath_bytes, shardBytes * N, "gather")) return rc;
        if (int rc = ensure_frame(bytes)) return rc;
        if (g_multi.rccl) {
            const size_t count = shardBytes / sizeof(float);
            if (ncclGroupStart() != ncclSuccess) return fail(LRT_E_HIP, "ncclGroupStart");
            ncclResult_t r = ncclSuccess;
            for (int k = 0; k < N && r == ncclSuccess; ++k) {
                DeviceScope ds(k);
                r = ncclGather(g_devs[k].d_shard, k == 0 ? c0.d_gath : nullptr, count, ncclFloat, 0, g_multi.comms[k],
                               g_devs[k].stream);
            }
            const ncclResult_t r2 = ncclGroupEnd();
            if (r != ncclSuccess || r2 != ncclSuccess)
                return fail(LRT_E_HIP, std::string("ncclGather: ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
        } else {
            for (int k = 0; k < N; ++k) {
                LRT_HIP(hipStreamWaitEvent(c0.stream, g_devs[k].ev_done, 0));
                char* dst = reinterpret_cast<char*>(c0.d_gath) + (size_t)k * shardBytes;
                if (g_devs[k].device == c0.device)
                    LRT_HIP(hipMemcpyAsync(dst, g_devs[k].d_shard, shardBytes, hipMemcpyDeviceToDevice, c0.stream));
                else
                    LRT_HIP(hipMemcpyPeerAsync(dst, c0.device, g_devs[k].d_shard, g_devs[k].device, shardBytes,
                                               c0.stream));
            }
        }
        dim3 grid((unsigned)((xc + 255) / 256), (unsigned)rows);
        unshard_kernel<<<grid, 256, 0, c0.stream>>>(reinterpret_cast<const float4*>(c0.d_gath),
                                                   reinterpret_cast<float4*>(c0.d_frame), xc, rows, b, N, maxRows);
        LRT_HIP(hipGetLastError());
        LRT_HIP(hipMemcpyAsync(buf, c0.d_frame, bytes, hipMemcpyDeviceToHost, c0.stream));
    }
    return LRT_OK;
}

// allow_register: the reference API's call (lrt_draw_test), whose caller keeps one buffer for
// the whole run (main.cpp:40,165): a pageable buffer may be page-locked (host_register).
int render_host(const lrt_render_desc* d, float* buf, long long* out_rays, const lrt_features* feat = nullptr,
                bool allow_register = false) {
    int rc = validate(d);
    if (rc) return rc;
    if (!ctx().ready) return fail(LRT_E_STATE, "lrt_initialize() has not been called");
    if (!buf) return fail(LRT_E_INVALID, "backbuffer is NULL");
    const size_t bytes = (size_t)d->x_count * d->row_count * 4 * sizeof(float);
    if (bytes == 0 || d->frames == 0) {
        if (out_rays) *out_rays = 0;
        return LRT_OK;
    }
    // lrt_initialize_devices: the caller's rows are split over every device (a window of
    // contiguous rows; a caller's own row-block-cyclic shard, or features, stay on device 0)
    if (g_multi.on && d->row_period == 1 && !feat) return render_host_multi(d, buf, bytes, out_rays);
    // lrt_last_launch() names the host path too: host=pipelined | zerocopy | staged, with
    // "registered-" when the registration cache page-locked a pageable buffer
    auto note = [](const char* path, bool registered) {
        const size_t n = strlen(g_last_launch);
        snprintf(g_last_launch + n, sizeof(g_last_launch) - n, " host=%s%s", registered ? "registered-" : "", path);
    };
    float* hdev = (!feat && host_zero_copy()) ? host_pinned(buf) : nullptr;
    bool registered = hdev && host_registered_here(buf);
    if (allow_register && !hdev && !feat && host_zero_copy()) registered = (hdev = host_register(buf, bytes)) != nullptr;
    if (hdev && host_pipeline(d, bytes)) {
        if ((rc = ensure_frame(bytes))) return rc;
        int ahead = 0;
        if ((rc = render_host_pipelined(d, buf, hdev, bytes, out_rays, allow_register, &ahead))) return rc;
        note("pipelined", registered);
        const size_t m = strlen(g_last_launch);
        snprintf(g_last_launch + m, sizeof(g_last_launch) - m, " lookahead=%s", ahead ? "hit" : "miss");
        return LRT_OK;
    }
    if (hdev) {   // zero copy: the kernel reads and writes the caller's pixels over PCIe
        LRT_HIP(hipMemsetAsync(ctx().d_rays, 0, sizeof(unsigned long long), ctx().stream));
        if ((rc = render_device(d, hdev, ctx().d_rays, nullptr, ctx().stream))) return rc;
        unsigned long long rays = 0;
        LRT_HIP(hipMemcpyAsync(&rays, ctx().d_rays, sizeof(rays), hipMemcpyDeviceToHost, ctx().stream));
        LRT_HIP(hipStreamSynchronize(ctx().stream));
        if (out_rays) *out_rays = (long long)rays;
        note("zerocopy", registered);
        return LRT_OK;
    }
    if ((rc = ensure_frame(bytes))) return rc;
    hipStream_t s = ctx().stream;
    LRT_HIP(hipMemcpyAsync(ctx().d_frame, buf, bytes, hipMemcpyHostToDevice, s));
    LRT_HIP(hipMemsetAsync(ctx().d_rays, 0, sizeof(unsigned long long), s));
    // host feature buffers go through device mirrors like the backbuffer
    lrt_features dfeat;
    memset(&dfeat, 0, sizeof(dfeat));
    float* const hp[6] = {feat ? feat->normal : nullptr,    feat ? feat->world_pos : nullptr,
                          feat ? feat->albedo : nullptr,    feat ? feat->color_std : nullptr,
                          feat ? feat->normal_std : nullptr, feat ? feat->world_pos_std : nullptr};
    float** const dp[6] = {&dfeat.normal, &dfeat.world_pos, &dfeat.albedo,
                           &dfeat.color_std, &dfeat.normal_std, &dfeat.world_pos_std};
    if (feat) {
        dfeat.max_frame = feat->max_frame;
        for (int k = 0; k < 6; ++k) {
            if (!hp[k]) continue;
            if (ctx().feat_bytes[k] < bytes) {
                if (ctx().d_feat[k]) (void)hipFree(ctx().d_feat[k]);
                ctx().d_feat[k] = nullptr;
                ctx().feat_bytes[k] = 0;
                if (hipMalloc(&ctx().d_feat[k], bytes) != hipSuccess) return fail(LRT_E_NOMEM, "hipMalloc(features)");
                ctx().feat_bytes[k] = bytes;
            }
            *dp[k] = ctx().d_feat[k];
            LRT_HIP(hipMemcpyAsync(ctx().d_feat[k], hp[k], bytes, hipMemcpyHostToDevice, s));
        }
    }
    if ((rc = render_device(d, ctx().d_frame, ctx().d_rays, feat ? &dfeat : nullptr, s))) return rc;
    unsigned long long rays = 0;
    LRT_HIP(hipMemcpyAsync(buf, ctx().d_frame, bytes, hipMemcpyDeviceToHost, s));
    for (int k = 0; k < 6; ++k)
        if (hp[k]) LRT_HIP(hipMemcpyAsync(hp[k], ctx().d_feat[k], bytes, hipMemcpyDeviceToHost, s));
    LRT_HIP(hipMemcpyAsync(&rays, ctx().d_rays, sizeof(rays), hipMemcpyDeviceToHost, s));
    LRT_HIP(hipStreamSynchronize(s));
    if (out_rays) *out_rays = (long long)rays;
    note("staged", false);
    return LRT_OK;
}

int camera_make(lrt_float3 lookFrom, lrt_float3 lookAt, lrt_float3 vup, float vfov, float aspect, float aperture,
                float focusDist, lrt_camera* out) {   // maths.h:183-202
    if (!out) return fail(LRT_E_INVALID, "camera out is NULL");
    lrt_camera c;
    c.lensRadius = aperture / 2.0f;
    c.origin = lookFrom;
    c.a = h_normalize(h_sub(lookFrom, lookAt));
    c.r = h_normalize(h_cross(vup, c.a));
    c.u = h_normalize(h_cross(c.a, c.r));
    float theta = vfov * kPI / 180.0f;
    float halfHeightTan = tanf(theta / 2.0f);
    float halfWidthTan = aspect * halfHeightTan;
    c.lowerLeftCorner = h_sub(h_sub(h_sub(c.origin, h_smul(halfWidthTan * focusDist, c.r)),
                                    h_smul(halfHeightTan * focusDist, c.u)),
                              h_smul(focusDist, c.a));
    c.horizontalVec = h_smul(2.0f * halfWidthTan * focusDist, c.r);
    c.verticalVec = h_smul(2.0f * halfHeightTan * focusDist, c.u);
    *out = c;
    return LRT_OK;
}

int camera_default(int w, int h, lrt_camera* out) {   // parallel.cpp:299-307
    if (w < 1 || h < 1) return fail(LRT_E_INVALID, "width/height must be >= 1");
    return camera_make(L3(0, 2, 3), L3(0, 0, 0), L3(0, 1, 0), 60.0f, (float)w / (float)h, 0.1f, 3.0f, out);
}


// lrt_scatter_eval's case i: Scatter (lrt_trace.h, parallel.cpp:78-196) of material ids[i]
// for the ray rays[6i..] (through the Ray ctor) at the hit recs[7i..] under RNG state seeds[i].
template <bool kBvh>
LRT_DEV void scatter_case(const SceneView& sc, int i, const int* ids, const float* rays, const float* recs,
                          const uint32_t* seeds, float* out, int* ret, int* counted, uint32_t* state,
                          bool coherent = false) {
    const Ray r = make_ray(f3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]),
                           f3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]));
    Hit rec;
    rec.pos = f3(recs[7 * i], recs[7 * i + 1], recs[7 * i + 2]);
    rec.normal = f3(recs[7 * i + 3], recs[7 * i + 4], recs[7 * i + 5]);
    rec.t = recs[7 * i + 6];
    const Material mat = load_material(sc.mats, ids[i]);
    uint32_t rng = seeds[i];
    int rays_ = 0;
    F3 att = f3(0.0f, 0.0f, 0.0f), lightE = f3(0.0f, 0.0f, 0.0f);
    Ray sc_ray;
    sc_ray.orig = sc_ray.dir = f3(0.0f, 0.0f, 0.0f);
    const bool ok = Scatter<kBvh>(mat, r, rec, att, sc_ray, lightE, rays_, rng, sc, coherent);
    const F3 v[4] = {att, sc_ray.orig, sc_ray.dir, lightE};
    for (int k = 0; k < 4; ++k) {
        out[12 * i + 3 * k] = v[k].x;
        out[12 * i + 3 * k + 1] = v[k].y;
        out[12 * i + 3 * k + 2] = v[k].z;
    }
    ret[i] = ok ? 1 : 0;
    counted[i] = rays_;
    state[i] = rng;
}
template <bool kBvh>
__global__ __launch_bounds__(64) void scatter_probe_kernel(SceneView sc, const int* ids, const float* rays,
                                                           const float* recs, const uint32_t* seeds, int n,
                                                           float* out, int* ret, int* counted, uint32_t* state,
                                                           int coherent) {
    __shared__ unsigned short stk[kBvhStackLevels * 64];
    sc.pow = libm::pow_tables();   // the device's table addresses (the host filled in its own)
    sc.bstk = stk + threadIdx.x;
    sc.bstride = 64;
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i < n) scatter_case<kBvh>(sc, i, ids, rays, recs, seeds, out, ret, counted, state, coherent != 0);
}

// lrt_bvh_eval's device side: one thread per ray, per-lane or packet traversal.
__global__ __launch_bounds__(64) void bvh_probe_kernel(BvhView bv, const float* rays, int n, int* ids, float* ts,
                                                       int packet) {
    __shared__ unsigned short stk[kBvhStackLevels * 64];
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    const Ray r = make_ray(f3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]),
                           f3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]));
    float t = 0.0f;
    ids[i] = ClosestHitBVH(r.orig, r.dir, bv, t, stk + threadIdx.x, 64, nullptr, packet != 0);
    ts[i] = t;
}


// A device's context: its stream, counters, lerp table and the default scene (lrt_initialize,
// and each device of lrt_initialize_devices; the device is current).
int init_context(Context& c, int dev) {
    c = Context();
    c.device = dev;
    LRT_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    LRT_HIP(hipMalloc(&c.d_rays, sizeof(unsigned long long)));
    LRT_HIP(hipMalloc(&c.d_tiles, sizeof(unsigned long long) * kQueueSlots * kTileSetU64));
    LRT_HIP(hipMemset(c.d_tiles, 0, sizeof(unsigned long long) * kQueueSlots * kTileSetU64));
    {   // parallel.cpp:262's lerpFac per frame number, divided once here instead of per wave
        std::vector<float> t(kLerpTable);
        for (int f = 0; f < kLerpTable; ++f) t[f] = (float)f / (float)(f + 1);
        LRT_HIP(hipMalloc(&c.d_lerp, sizeof(float) * kLerpTable));
        LRT_HIP(hipMemcpy(c.d_lerp, t.data(), sizeof(float) * kLerpTable, hipMemcpyHostToDevice));
    }
    LRT_HIP(hipDeviceGetAttribute(&c.num_cus, hipDeviceAttributeMultiprocessorCount, dev));
    {   // keep freed stream-ordered blocks (the per-launch path-stack overflow) in the
        // pool instead of returning them to the driver at every synchronisation
        hipMemPool_t pool;
        if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
            uint64_t keep = UINT64_MAX;
            (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
        }
    }
    if (int rc = upload_scene(c, kDefaultSpheres, kDefaultMats, 9)) return rc;
    c.ready = true;
    return LRT_OK;
}

// Frees everything init_context and the render paths allocated (the device is current).
void free_context(Context& c) {
    if (c.stream) (void)hipStreamSynchronize(c.stream);
    (void)hipDeviceSynchronize();
    free_scene(c);
    for (float* p : {c.d_frame, c.d_shard, c.d_gath})
        if (p) (void)hipFree(p);
    if (c.d_rays) (void)hipFree(c.d_rays);
    if (c.d_tiles) (void)hipFree(c.d_tiles);
    if (c.d_lerp) (void)hipFree(c.d_lerp);
    if (c.wf.buf) (void)hipFree(c.wf.buf);
    if (c.wf.rayp) (void)hipFree(c.wf.rayp);
    for (auto* f : c.d_feat)
        if (f) (void)hipFree(f);
    for (auto& m : c.masked_streams) (void)hipStreamDestroy(m.first);
    if (c.d_col) (void)hipFree(c.d_col);
    for (auto& o : c.order) {
        if (o.d_base) (void)hipFree(o.d_base);
        if (o.ev_rec) (void)hipEventDestroy(o.ev_rec);
        for (auto& u : o.uses) (void)hipEventDestroy(u.second);
    }
    for (int k = 0; k < Context::kHostChunks; ++k)
        if (c.ev_in[k]) (void)hipEventDestroy(c.ev_in[k]);
    if (c.ev_ret) (void)hipEventDestroy(c.ev_ret);
    for (int k = 0; k < 2; ++k)
        if (c.ahead.col[k]) (void)hipFree(c.ahead.col[k]);
    if (c.ahead.d_rays) (void)hipFree(c.ahead.d_rays);
    if (c.ahead.ev) (void)hipEventDestroy(c.ahead.ev);
    if (c.ahead.ev_render) (void)hipEventDestroy(c.ahead.ev_render);
    // (c.ahead.stream is one of c.masked_streams, destroyed with them)
    if (c.ev_done) (void)hipEventDestroy(c.ev_done);
    if (c.s_in) (void)hipStreamDestroy(c.s_in);
    if (c.stream) (void)hipStreamDestroy(c.stream);
    c = Context();
}
}  // namespace lrt

using namespace lrt;

// roctx ranges around the C-ABI's work entry points (SURVEY §5 tracing): rocprofv3
// --marker-trace shows each lrt_* call on the host timeline above the kernels it launched.
struct RoctxRange {
#if LRT_ROCTX
    explicit RoctxRange(const char* name) { roctxRangePushA(name); }
    ~RoctxRange() { roctxRangePop(); }
#else
    explicit RoctxRange(const char*) {}
#endif
};

extern "C" {

const char* lrt_last_error(void) { return t_err.c_str(); }
const char* lrt_version(void) { return LRT_VERSION_STRING; }
const char* lrt_last_launch(void) {
    // a copy taken under the lock: render calls on other threads rewrite g_last_launch
    std::lock_guard<std::mutex> lk(g_mu);
    t_launch = g_last_launch;
    return t_launch.c_str();
}

int lrt_initialize(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ndev > 0) return LRT_OK;
    int dev = 0;
    LRT_HIP(hipGetDevice(&dev));
    g_cur = 0;
    const int rc = init_context(g_devs[0], dev);
    if (rc) {
        free_context(g_devs[0]);
        return rc;
    }
    g_ndev = 1;
    g_multi = Multi();
    return LRT_OK;
}

int lrt_initialize_devices(int n, const int* device_ids, int flags) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ndev > 0) return fail(LRT_E_STATE, "already initialised: call lrt_shutdown() first");
    if ((flags & ~LRT_DEV_PEER_COPY) != 0) return fail(LRT_E_INVALID, "unknown lrt_initialize_devices flags");
    int visible = 0;
    LRT_HIP(hipGetDeviceCount(&visible));
    std::vector<int> ids;
    if (n == 0 && !device_ids) {   // every visible device
        for (int i = 0; i < visible && i < kMaxDevices; ++i) ids.push_back(i);
    } else {
        if (n < 1 || n > kMaxDevices || !device_ids) return fail(LRT_E_INVALID, "need 1..16 device ids");
        ids.assign(device_ids, device_ids + n);
    }
    if (ids.empty()) return fail(LRT_E_INVALID, "no device");
    for (int id : ids)
        if (id < 0 || id >= visible) return fail(LRT_E_INVALID, "device id out of range");
    int prev = 0;
    LRT_HIP(hipGetDevice(&prev));
    int rc = LRT_OK;
    int k = 0;
    for (; k < (int)ids.size() && rc == LRT_OK; ++k) {
        g_cur = k;
        if (hipSetDevice(ids[k]) != hipSuccess) {
            rc = fail(LRT_E_HIP, "hipSetDevice");
            break;
        }
        rc = init_context(g_devs[k], ids[k]);
    }
    g_cur = 0;
    const int N = (int)ids.size();
    bool distinct = true;
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < i; ++j) distinct = distinct && ids[i] != ids[j];
    g_multi = Multi();
    if (const char* e = getenv("LRT_ROW_BLOCK")) g_multi.row_block = std::max(1, atoi(e));
    if (rc == LRT_OK && distinct && !(flags & LRT_DEV_PEER_COPY)) {
        // one communicator per device, all in this process (the single-thread multi-device
        // form of RCCL); the gather is issued as a group (render_host_multi)
        const ncclResult_t r = ncclCommInitAll(g_multi.comms, N, ids.data());
        if (r != ncclSuccess) rc = fail(LRT_E_HIP, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
        g_multi.rccl = r == ncclSuccess;
    } else if (rc == LRT_OK) {
        for (int i = 1; i < N; ++i)   // peer copies into device 0 (ignore "already enabled")
            if (ids[i] != ids[0]) {
                (void)hipSetDevice(ids[0]);
                (void)hipDeviceEnablePeerAccess(ids[i], 0);
                (void)hipGetLastError();
            }
    }
    (void)hipSetDevice(prev);
    if (rc) {
        for (int i = 0; i < k; ++i) {
            DeviceScope ds(i);
            free_context(g_devs[i]);
        }
        if (g_multi.rccl)
            for (int i = 0; i < N; ++i) (void)ncclCommDestroy(g_multi.comms[i]);
        g_multi = Multi();
        return rc;
    }
    g_ndev = N;
    g_multi.on = true;
    return LRT_OK;
}

int lrt_device_count(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_ndev;
}

int lrt_shutdown(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ndev == 0) return LRT_OK;
    for (auto& r : g_host_regs)
        if (r.p) (void)host_unregister(r.p);
    g_host_last = HostReg();
    if (g_multi.rccl)
        for (int k = 0; k < g_ndev; ++k) (void)ncclCommDestroy(g_multi.comms[k]);
    for (int k = 0; k < g_ndev; ++k) {
        DeviceScope ds(k);
        free_context(g_devs[k]);
    }
    g_ndev = 0;
    g_cur = 0;
    g_multi = Multi();
    return LRT_OK;
}

int lrt_host_unregister(void* p) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!p) return LRT_OK;
    if (g_host_last.p == p) g_host_last = HostReg();
    return host_unregister(p);
}

int lrt_draw_test(float time, int frameCount, int screenWidth, int screenHeight, float* backbuffer,
                  int* outRayCount) {
    RoctxRange rr_("lrt_draw_test");
    (void)time;   // unused by the reference too (JobData::time, parallel.cpp:244)
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);   // context 0's device (device 0 of lrt_initialize_devices)
    lrt_render_desc d;
    memset(&d, 0, sizeof(d));
    int rc = camera_default(screenWidth, screenHeight, &d.camera);
    if (rc) return rc;
    d.width = screenWidth;
    d.height = screenHeight;
    d.x0 = 0;
    d.x_count = screenWidth;
    d.y0 = 0;
    d.row_count = screenHeight;
    d.row_block = screenHeight;
    d.row_period = 1;
    d.row_phase = 0;
    d.frame0 = frameCount;
    d.frames = 1;
    d.max_depth = LRT_REFERENCE_MAX_DEPTH;
    long long rays = 0;
    rc = render_host(&d, backbuffer, &rays, nullptr, true);
    if (rc) return rc;
    if (outRayCount) *outRayCount = (int)rays;
    return LRT_OK;
}

int lrt_camera_make(lrt_float3 lookFrom, lrt_float3 lookAt, lrt_float3 vup, float vfov, float aspect,
                    float aperture, float focusDist, lrt_camera* out) {
    return camera_make(lookFrom, lookAt, vup, vfov, aspect, aperture, focusDist, out);
}

int lrt_camera_default(int width, int height, lrt_camera* out) { return camera_default(width, height, out); }

int lrt_set_scene(const lrt_sphere* spheres, const lrt_material* materials, int count) {
    RoctxRange rr_("lrt_set_scene");
    std::lock_guard<std::mutex> lk(g_mu);
    if (!ctx().ready) return fail(LRT_E_STATE, "lrt_initialize() has not been called");
    for (int k = 0; k < g_ndev; ++k) {   // every device in use holds the scene
        DeviceScope ds(k);
        LRT_HIP(hipStreamSynchronize(ctx().stream));
        LRT_HIP(hipDeviceSynchronize());
        if (int rc = upload_scene(ctx(), spheres, materials, count)) return rc;
    }
    return LRT_OK;
}

int lrt_default_scene(lrt_sphere* spheres, lrt_material* materials, int capacity, int* count) {
    if (count) *count = 9;
    if (capacity < 9 || !spheres || !materials) return fail(LRT_E_INVALID, "need capacity >= 9");
    memcpy(spheres, kDefaultSpheres, sizeof(kDefaultSpheres));
    memcpy(materials, kDefaultMats, sizeof(kDefaultMats));
    return LRT_OK;
}

int lrt_render_device(const lrt_render_desc* desc, float* d_backbuffer, unsigned long long* d_rays, void* stream) {
    RoctxRange rr_("lrt_render_device");
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);   // context 0's device (device 0 of lrt_initialize_devices)
    return render_device(desc, d_backbuffer, d_rays, nullptr, (hipStream_t)stream);
}

int lrt_render_device_to_frame(const lrt_render_desc* desc, float* d_backbuffer, unsigned long long* d_rays,
                               float* d_frame, void* stream) {
    RoctxRange rr_("lrt_render_device_to_frame");
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);
    if (!d_frame) return fail(LRT_E_INVALID, "d_frame is NULL");
    return render_device(desc, d_backbuffer, d_rays, nullptr, (hipStream_t)stream, nullptr, d_frame);
}

int lrt_ipc_alloc(size_t bytes, void** d_ptr, void* handle) {
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);
    if (!d_ptr || !handle || bytes == 0) return fail(LRT_E_INVALID, "invalid ipc alloc arguments");
    *d_ptr = nullptr;
    LRT_HIP(hipMalloc(d_ptr, bytes));   // its own allocation: the handle maps exactly this buffer
    LRT_HIP(hipMemset(*d_ptr, 0, bytes));
    hipIpcMemHandle_t h;
    const hipError_t e = hipIpcGetMemHandle(&h, *d_ptr);
    if (e != hipSuccess) {
        (void)hipFree(*d_ptr);
        *d_ptr = nullptr;
        return hip_fail(e, "hipIpcGetMemHandle");
    }
    static_assert(sizeof(h) <= LRT_IPC_HANDLE_BYTES, "IPC handle size");
    memcpy(handle, &h, sizeof(h));
    return LRT_OK;
}

int lrt_ipc_free(void* d_ptr) {
    if (!d_ptr) return LRT_OK;
    LRT_HIP(hipFree(d_ptr));
    return LRT_OK;
}

int lrt_ipc_open(const void* handle, void** d_ptr) {
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);
    if (!handle || !d_ptr) return fail(LRT_E_INVALID, "invalid ipc open arguments");
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    LRT_HIP(hipIpcOpenMemHandle(d_ptr, h, hipIpcMemLazyEnablePeerAccess));
    return LRT_OK;
}

int lrt_ipc_close(void* d_ptr) {
    if (!d_ptr) return LRT_OK;
    LRT_HIP(hipIpcCloseMemHandle(d_ptr));
    return LRT_OK;
}

int lrt_render_device_ex(const lrt_render_desc* desc, float* d_backbuffer, unsigned long long* d_rays,
                         const lrt_features* d_features, void* stream) {
    RoctxRange rr_("lrt_render_device_ex");
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);   // context 0's device (device 0 of lrt_initialize_devices)
    return render_device(desc, d_backbuffer, d_rays, d_features, (hipStream_t)stream);
}

int lrt_render_host_ex(const lrt_render_desc* desc, float* backbuffer, long long* out_rays,
                       const lrt_features* features) {
    RoctxRange rr_("lrt_render_host_ex");
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);   // context 0's device (device 0 of lrt_initialize_devices)
    return render_host(desc, backbuffer, out_rays, features);
}

int lrt_render_host(const lrt_render_desc* desc, float* backbuffer, long long* out_rays) {
    RoctxRange rr_("lrt_render_host");
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);   // context 0's device (device 0 of lrt_initialize_devices)
    return render_host(desc, backbuffer, out_rays);
}

int lrt_stream_create(int reserved_cus, void** out) {
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);
    if (!ctx().ready) return fail(LRT_E_STATE, "lrt_initialize() has not been called");
    if (!out) return fail(LRT_E_INVALID, "stream out is NULL");
    const int n = ctx().num_cus;
    if (reserved_cus < 0 || reserved_cus >= n) return fail(LRT_E_INVALID, "reserved_cus must be in [0, CU count)");
    // the last reserved_cus logical CUs stay free; hipExtStreamCreateWithCUMask takes one
    // bit per CU, 32 per word
    std::vector<uint32_t> mask((size_t)(n + 31) / 32, 0u);
    // Logical CU c sits on XCD c % 8 (measured: reserving CUs 31, 63, ... -- all on one XCD
    // -- slows a full-chip render 20-70 %, because workgroups are dealt to XCDs round-robin),
    // so the last reserved_cus logical CUs spread the reservation evenly over the XCDs.
    int kept = 0;
    for (int c = 0; c < n - reserved_cus; ++c) {
        mask[c / 32] |= 1u << (c % 32);
        ++kept;
    }
    hipStream_t st = nullptr;
    LRT_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
    ctx().masked_streams.emplace_back(st, kept);
    *out = st;
    return LRT_OK;
}

int lrt_host_alloc(size_t bytes, void** out) {
    if (!out) return fail(LRT_E_INVALID, "out is NULL");
    *out = nullptr;
    if (bytes == 0) return fail(LRT_E_INVALID, "bytes must be > 0");
    if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) {
        *out = nullptr;
        return fail(LRT_E_NOMEM, "hipHostMalloc failed");
    }
    return LRT_OK;
}

int lrt_host_free(void* p) {
    if (!p) return LRT_OK;
    LRT_HIP(hipHostFree(p));
    return LRT_OK;
}

int lrt_stream_destroy(void* stream) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto& v = ctx().masked_streams;
    for (size_t i = 0; i < v.size(); ++i)
        if (v[i].first == (hipStream_t)stream) {
            (void)hipStreamSynchronize(v[i].first);
            LRT_HIP(hipStreamDestroy(v[i].first));
            v.erase(v.begin() + (long)i);
            return LRT_OK;
        }
    return fail(LRT_E_INVALID, "not a stream from lrt_stream_create");
}

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

// Diagnostic (host only, no GPU): build the BVH of the given scene and trace n rays
// (o.xyz, d.xyz; d normalised as the Ray ctor does) with the device traversal code.
// out[0..4]: mean nodes visited, mean spheres tested, max nodes, max spheres, fraction of
// rays whose (id, t) differs from the linear scan (must be 0).
int lrt_bvh_stats(const lrt_sphere* spheres, int count, const float* rays, int n, double* out) {
    if (!spheres || count < 2 || !rays || !out || n < 1) return fail(LRT_E_INVALID, "invalid arguments");
    std::vector<float4> sph(count);
    for (int i = 0; i < count; ++i) {
        const float r = spheres[i].radius;
        sph[i] = make_float4(spheres[i].center.x, spheres[i].center.y, spheres[i].center.z, r * r);
    }
    BvhHost H;
    build_bvh_host(spheres, count, sph, H);
    BvhView bv;
    bv.nodes = H.nodes.data();
    bv.lsph = H.lsph.data();
    bv.lid = H.lid.data();
    bv.margin = H.margin;
    bv.on = 1;
    bv.nnodes = (int)(H.nodes.size() / 8);
    bv.big0 = H.big0;
    bv.nbig = H.nbig;
    double sn = 0, ss = 0, mn = 0, ms = 0, bad = 0, msp = 0;
    unsigned short stk[kBvhStackLevels];
    for (int i = 0; i < n; ++i) {
        const Ray r = make_ray(f3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]),
                               f3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]));
        BvhStats st;
        float t1, t2;
        const int a = ClosestHitBVH(r.orig, r.dir, bv, t1, stk, 1, &st);
        const int b = ClosestHit(r.orig, r.dir, sph.data(), count, t2);
        if (a != b || memcmp(&t1, &t2, 4) != 0) bad += 1;
        // the bounded shadow-ray traversal: true for the scan's winner, and for any other
        // sphere exactly when it is the winner
        if (b >= 0 && !ShadowReachesLightBVH(r.orig, r.dir, b, sph[b], bv, stk, 1, false, &st)) bad += 1;
        const int other = (int)(((unsigned)i * 7919u) % (unsigned)count);
        if (ShadowReachesLightBVH(r.orig, r.dir, other, sph[other], bv, stk, 1, false, &st) != (b == other)) bad += 1;
        // the two-query loop (pool kernel): this ray as the shadow ray towards `other` (and
        // towards the winner), the next ray's direction from the same origin as the bounce ray
        {
            const int i2 = (i + 1) % n;
            const Ray r2 = make_ray(r.orig, f3(rays[6 * i2 + 3], rays[6 * i2 + 4], rays[6 * i2 + 5]));
            float t3, t4;
            const int c2 = ClosestHitBVH(r2.orig, r2.dir, bv, t3, stk, 1);
            for (int li : {other, b}) {
                if (li < 0) continue;
                bool lit = true;
                const int c3 = ClosestHitDualBVH4(r.orig, r2.dir, true, r.dir, li, sph[li], bv, t4, lit, stk, 1, &st);
                if (c3 != c2 || memcmp(&t3, &t4, 4) != 0 || lit != (b == li)) bad += 1;
            }
            bool lit = true;
            const int c4 = ClosestHitDualBVH4(r.orig, r2.dir, false, r.dir, 0, sph[0], bv, t4, lit, stk, 1, &st);
            if (c4 != c2 || memcmp(&t3, &t4, 4) != 0 || lit) bad += 1;
        }
        sn += st.nodes;
        ss += st.spheres;
        mn = std::max(mn, (double)st.nodes);
        msp = std::max(msp, (double)st.max_sp);
        ms = std::max(ms, (double)st.spheres);
    }
    out[0] = sn / n;
    out[1] = ss / n;
    out[2] = mn;
    out[3] = ms;
    out[4] = bad / n;
    out[5] = msp;                    // deepest stack entry any traversal wrote
    out[6] = (double)H.stack_levels; // the entries the LDS stack holds for this scene
    return LRT_OK;
}

int lrt_scatter_eval(const lrt_sphere* spheres, const lrt_material* materials, int count, const int* ids,
                     const float* rays, const float* recs, const uint32_t* seeds, int n, float* out, int* ret,
                     int* counted, uint32_t* state, int on_device) {
    if (!ids || !rays || !recs || !seeds || !out || !ret || !counted || !state || n < 0)
        return fail(LRT_E_INVALID, "scatter probe: null argument");
    std::vector<float4> sph, mats;
    std::vector<int> lights;
    if (const int e = pack_scene(spheres, materials, count, sph, mats, lights)) return e;
    for (int i = 0; i < n; ++i)
        if (ids[i] < 0 || ids[i] >= count) return fail(LRT_E_INVALID, "scatter probe: material id out of range");
    if (n == 0) return LRT_OK;
    const bool bvh = count > kBvhMinSpheres;
    BvhHost B;
    if (bvh) build_bvh_host(spheres, count, sph, B);
    SceneView sc{};
    sc.count = count;
    sc.nlights = (int)lights.size();
    if (lights.empty()) lights.push_back(0);   // never read (nlights = 0): keeps the copy non-empty
    sc.pow = libm::pow_tables();   // host addresses: the probe kernel sets its own
    sc.rnlut = nullptr;
    sc.bv.margin = B.margin;
    sc.bv.on = bvh ? 1 : 0;
    sc.bv.nnodes = bvh ? (int)(B.nodes.size() / 8) : 0;
    sc.bv.big0 = B.big0;
    sc.bv.nbig = B.nbig;
    if (!on_device) {
        sc.sph = sph.data();
        sc.mats = mats.data();
        sc.lights = lights.data();
        sc.bv.nodes = B.nodes.data();
        sc.bv.lsph = B.lsph.data();
        sc.bv.lid = B.lid.data();
        unsigned short stk[kBvhStackLevels];
        sc.bstk = stk;
        sc.bstride = 1;
        for (int i = 0; i < n; ++i) {
            if (bvh) scatter_case<true>(sc, i, ids, rays, recs, seeds, out, ret, counted, state);
            else scatter_case<false>(sc, i, ids, rays, recs, seeds, out, ret, counted, state);
        }
        return LRT_OK;
    }
    // device: one thread per case over device copies of everything
    std::vector<void*> owned;
    auto up = [&](const void* src, size_t bytes) -> void* {   // a device copy (>= 16 B), owned
        void* d = nullptr;
        if (hipMalloc(&d, std::max<size_t>(bytes, 16)) != hipSuccess) return nullptr;
        owned.push_back(d);
        if (bytes && hipMemcpy(d, src, bytes, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
        return d;
    };
    auto release = [&]() {
        for (void* p : owned) (void)hipFree(p);
    };
    void* dd[10] = {up(sph.data(), sph.size() * sizeof(float4)), up(mats.data(), mats.size() * sizeof(float4)),
                    up(lights.data(), lights.size() * sizeof(int)),
                    up(B.nodes.data(), B.nodes.size() * sizeof(float4)),
                    up(B.lsph.data(), B.lsph.size() * sizeof(float4)), up(B.lid.data(), B.lid.size() * sizeof(int)),
                    up(ids, sizeof(int) * n), up(rays, sizeof(float) * 6 * n), up(recs, sizeof(float) * 7 * n),
                    up(seeds, sizeof(uint32_t) * n)};
    float* o_out = nullptr;
    int *o_ret = nullptr, *o_cnt = nullptr;
    uint32_t* o_st = nullptr;
    if (hipMalloc(&o_out, sizeof(float) * 12 * n) == hipSuccess) owned.push_back(o_out);
    if (hipMalloc(&o_ret, sizeof(int) * n) == hipSuccess) owned.push_back(o_ret);
    if (hipMalloc(&o_cnt, sizeof(int) * n) == hipSuccess) owned.push_back(o_cnt);
    if (hipMalloc(&o_st, sizeof(uint32_t) * n) == hipSuccess) owned.push_back(o_st);
    if (std::find(std::begin(dd), std::end(dd), nullptr) != std::end(dd) || !o_out || !o_ret ||
        !o_cnt || !o_st) {
        release();
        return fail(LRT_E_NOMEM, "scatter probe: device allocation failed");
    }
    sc.sph = (const float4*)dd[0];
    sc.mats = (const float4*)dd[1];
    sc.lights = (const int*)dd[2];
    sc.bv.nodes = (const float4*)dd[3];
    sc.bv.lsph = (const float4*)dd[4];
    sc.bv.lid = (const int*)dd[5];
    const unsigned blocks = (unsigned)((n + 63) / 64);
    if (bvh)
        scatter_probe_kernel<true><<<blocks, 64>>>(sc, (const int*)dd[6], (const float*)dd[7], (const float*)dd[8],
                                                   (const uint32_t*)dd[9], n, o_out, o_ret, o_cnt, o_st,
                                                   on_device == 2);
    else
        scatter_probe_kernel<false><<<blocks, 64>>>(sc, (const int*)dd[6], (const float*)dd[7], (const float*)dd[8],
                                                    (const uint32_t*)dd[9], n, o_out, o_ret, o_cnt, o_st, 0);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, o_out, sizeof(float) * 12 * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(ret, o_ret, sizeof(int) * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(counted, o_cnt, sizeof(int) * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(state, o_st, sizeof(uint32_t) * n, hipMemcpyDeviceToHost);
    release();
    if (e != hipSuccess) return fail(LRT_E_HIP, std::string("scatter probe: ") + hipGetErrorString(e));
    return LRT_OK;
}

int lrt_bvh_eval(const lrt_sphere* spheres, int count, const float* rays, int n, int* ids, float* ts, int mode) {
    if (!spheres || count < 2 || !rays || !ids || !ts || n < 0 || mode < 0 || mode > 2)
        return fail(LRT_E_INVALID, "bvh eval: invalid arguments");
    std::vector<float4> sph(count);
    for (int i = 0; i < count; ++i) {
        const float r = spheres[i].radius;
        sph[i] = make_float4(spheres[i].center.x, spheres[i].center.y, spheres[i].center.z, r * r);
    }
    BvhHost H;
    build_bvh_host(spheres, count, sph, H);
    BvhView bv;
    bv.margin = H.margin;
    bv.on = 1;
    bv.nnodes = (int)(H.nodes.size() / 8);
    bv.big0 = H.big0;
    bv.nbig = H.nbig;
    if (mode == 0) {
        bv.nodes = H.nodes.data();
        bv.lsph = H.lsph.data();
        bv.lid = H.lid.data();
        unsigned short stk[kBvhStackLevels];
        for (int i = 0; i < n; ++i) {
            const Ray r = make_ray(f3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]),
                                   f3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]));
            ids[i] = ClosestHitBVH(r.orig, r.dir, bv, ts[i], stk, 1);
        }
        return LRT_OK;
    }
    if (n == 0) return LRT_OK;
    void *d_nodes = nullptr, *d_lsph = nullptr, *d_lid = nullptr, *d_rays = nullptr, *d_ids = nullptr, *d_ts = nullptr;
    hipError_t e = hipMalloc(&d_nodes, sizeof(float4) * std::max<size_t>(H.nodes.size(), 8));
    if (e == hipSuccess) e = hipMalloc(&d_lsph, sizeof(float4) * H.lsph.size());
    if (e == hipSuccess) e = hipMalloc(&d_lid, sizeof(int) * H.lid.size());
    if (e == hipSuccess) e = hipMalloc(&d_rays, sizeof(float) * 6 * (size_t)n);
    if (e == hipSuccess) e = hipMalloc(&d_ids, sizeof(int) * (size_t)n);
    if (e == hipSuccess) e = hipMalloc(&d_ts, sizeof(float) * (size_t)n);
    if (e == hipSuccess && !H.nodes.empty())
        e = hipMemcpy(d_nodes, H.nodes.data(), sizeof(float4) * H.nodes.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_lsph, H.lsph.data(), sizeof(float4) * H.lsph.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_lid, H.lid.data(), sizeof(int) * H.lid.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_rays, rays, sizeof(float) * 6 * (size_t)n, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        bv.nodes = (const float4*)d_nodes;
        bv.lsph = (const float4*)d_lsph;
        bv.lid = (const int*)d_lid;
        bvh_probe_kernel<<<(unsigned)((n + 63) / 64), 64>>>(bv, (const float*)d_rays, n, (int*)d_ids, (float*)d_ts,
                                                          mode == 2);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(ids, d_ids, sizeof(int) * (size_t)n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(ts, d_ts, sizeof(float) * (size_t)n, hipMemcpyDeviceToHost);
    for (void* p : {d_nodes, d_lsph, d_lid, d_rays, d_ids, d_ts})
        if (p) (void)hipFree(p);
    if (e != hipSuccess) return fail(LRT_E_HIP, std::string("bvh eval: ") + hipGetErrorString(e));
    return LRT_OK;
}

int lrt_libm_eval_host(int kind, const float* in, float* out, long long n) {
    if (kind < 0 || kind > 7 || !in || !out || n < 0) return fail(LRT_E_INVALID, "invalid libm eval arguments");
    for (long long i = 0; i < n; ++i)
        out[i] = libm_eval(kind, in[i]);
    return LRT_OK;
}

int lrt_libm_eval_device(int kind, const float* d_in, float* d_out, long long n) {
    if (kind < 0 || kind > 7 || !d_in || !d_out || n < 0) return fail(LRT_E_INVALID, "invalid libm eval arguments");
    if (n == 0) return LRT_OK;
    libm_kernel<<<(unsigned)((n + 255) / 256), 256, 0, nullptr>>>(kind, d_in, d_out, n);
    LRT_HIP(hipGetLastError());
    LRT_HIP(hipDeviceSynchronize());
    return LRT_OK;
}

}  // extern "C"
