// v0: trace_kernel (the reference's per-pixel loop, TraceRowJob parallel.cpp:254-294) and its
// launch policy; instantiated per depth class by lrt_v0_d8.hip and lrt_v0_d64.hip.
//
// A pixel's S samples are spread over up to 16 adjacent lanes and lerped in frame order (so
// the progressive sequence of S DrawTest calls is reproduced bit for bit from the buffer's prev
// value); persistent single-wave workgroups are fed from 16 tile queues; the scene, the powf
// tables and the recursion stack live in LDS; each pixel is read once and written once per
// call; rays are counted per lane, reduced per wave, folded per queue.
#pragma once
#include "lrt_internal.h"

namespace lrt {

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
template <int MAXD, bool kLds, int kAcc, int kSplit, bool kFeat = false, bool kSamp = false, int kNS = 0>
__global__ __launch_bounds__(kBlock, kWavesPerEU) void trace_kernel(const KernelArgs a) {
    static_assert(kNS == 0 || (kLds && !kAcc), "a fixed sphere count is for the LDS linear scan");
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
    constexpr int kLutBytes = kAcc ? 0 : kRenormBytes;
    float* s_lut = kAcc ? nullptr : reinterpret_cast<float*>(s_pow + 64);
    if (!kAcc) renorm_lut_fill(s_lut, tid, kBlock);
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
    sc.gv = a.gv;
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
        // (a.lateFetch, few tasks per wave: the next task is reserved after this one's trace
        // instead, so that the waves done first take the last tasks -- lrt_pool.h; profiles/r5_af)
        unsigned long long fetched = 0;
        if (!a.lateFetch && lane == 0) fetched = atomicAdd(ctr, 1ull);
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
                col = Trace<MAXD, kAcc, kFeat, kTraceLdsLevels, kNS>(r, a.maxDepth, rays, rng, sc, smem + tid, kBlock, a.ovf + gtid,
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
        if (a.lateFetch && lane == 0) fetched = atomicAdd(ctr, 1ull);
        if (!kSamp && valid && sub == 0) {
            *px = acc;
            if (a.frame) a.frame[(size_t)y * a.width + x] = acc;   // the frame exchange, fused
        }
        if constexpr (kFeat) {
#pragma unroll
            for (int k = 0; k < 6; ++k)
                if (valid && a.feat[k]) a.feat[k][pix] = fb[k];
        }
        {
            const unsigned long long n = __shfl(fetched, 0, 64) + (unsigned long long)bq;
            i = n < (unsigned long long)nq ? (int)n : nq;
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
        a.wtrace[4 * w + 2] = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) |   // HW_ID
                              ((unsigned long long)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32);   // XCC_ID
        a.wtrace[4 * w + 3] = 0;
    }
#endif
    if (tid == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += s_rays[w];
        block_epilogue(a.tiles, a.rays, q, bq, t);
    }
}

constexpr int kMaxSplit = 16;   // lanes per pixel at most (32 / 64: no better, 4 % slower on config 4)


template <int MAXD, int kSplit, bool kFeat = false>
int launch_depth(KernelArgs a, bool lds, int xc, int rows, hipStream_t s) {
    constexpr int kTileRows = kBlockWavesY * (64 / kSplit / WaveCols(kSplit));
    constexpr int kTileX = WaveCols(kSplit) * kBlockWavesX;
    const long long ntiles = (long long)((xc + kTileX - 1) / kTileX) * ((rows + kTileRows - 1) / kTileRows);
    const int acc = a.gv.on ? kAccGrid : a.bv.on ? kAccBvh : kAccScan;
    const size_t stack = sizeof(float4) * kTraceLdsLevels * kBlock + kPowTableBytes + (acc ? 0 : kRenormBytes);
    const size_t scene = lds ? sizeof(float4) * (4 * (size_t)a.count + (size_t)(a.nlights + 3) / 4 + 1) : 0;
    a.bvh_stack_offset = (int)(stack + scene);
    // v0 sizes the LDS traversal stack to this scene's BVH depth (1000 spheres: ~9
    // levels, 1.2 KB instead of 3 KB per wave -- the difference between 13 and 16 waves/CU)
    const size_t bstk = acc == kAccBvh ? sizeof(unsigned short) * ctx().bvh_stack_levels * kBlock : 0;
    const size_t ldsb = stack + (lds ? scene : 0) + bstk;
    // the reference's own scene size (parallel.cpp:27) gets the unrolled-scan instances
    const bool fixed = lds && acc == kAccScan && a.count == kFixedSpheres;
    const void* kern = acc == kAccGrid ? (lds ? (const void*)trace_kernel<MAXD, true, kAccGrid, kSplit, kFeat>
                                              : (const void*)trace_kernel<MAXD, false, kAccGrid, kSplit, kFeat>)
                       : acc == kAccBvh ? (lds ? (const void*)trace_kernel<MAXD, true, kAccBvh, kSplit, kFeat>
                                               : (const void*)trace_kernel<MAXD, false, kAccBvh, kSplit, kFeat>)
                       : (fixed ? (const void*)trace_kernel<MAXD, true, kAccScan, kSplit, kFeat, false, kFixedSpheres>
                          : lds ? (const void*)trace_kernel<MAXD, true, kAccScan, kSplit, kFeat>
                                : (const void*)trace_kernel<MAXD, false, kAccScan, kSplit, kFeat>);
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
    // rounds on 4,096 waves).
    const int rounds = (a.frames + kSplit - 1) / kSplit;
    const size_t npix = (size_t)xc * rows;
    bool samp = false;
    if constexpr (!kFeat && kSplit == 1) samp = a.sampOnly && lds && acc == kAccScan;
    if constexpr (!kFeat && kSplit >= 4) {
        const long long slots = (long long)per_cu * cus;
        samp = lds && acc == kAccScan && rounds >= 2 && npix * (size_t)a.frames * sizeof(float4) <= (2ull << 30) &&
               ntiles < 16 * slots;
    }
    if (a.sampOnly && !samp) return fail(LRT_E_INVALID, "colours-only render: needs the LDS linear scan, one frame lane");
    const long long tasks = samp ? ntiles * rounds : ntiles;
    long long blocks = (long long)per_cu * cus;
    // block b serves queue b % kV0Queues: every queue that owns a task needs a block, even
    // on a CU-masked stream left with fewer slots than queues (those blocks start later)
    blocks = std::max(blocks, (long long)kV0Queues);
    if (blocks > tasks) blocks = tasks;
    const dim3 grid((unsigned)blocks);
    a.lateFetch = tasks < 6LL * blocks * (kBlock / 64) ? 1 : 0;   // few tasks per wave: reserve late
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
    kernel_timing(s, 0);
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
            e = launch_merge_samples(a.samp, a.out, a.lerp, (int)npix, a.frame0, a.frames, npix, a, 0, s);
            if (e != hipSuccess) return hip_fail(e, "merge_samples_kernel launch");
            e = hipFreeAsync(a.samp, s);
            if (e != hipSuccess) return hip_fail(e, "hipFreeAsync(sample planes)");
        }
    }
    if (samp) {
    } else if (acc == kAccGrid) {
        if (lds)
            trace_kernel<MAXD, true, kAccGrid, kSplit, kFeat><<<grid, kBlock, ldsb, s>>>(a);
        else
            trace_kernel<MAXD, false, kAccGrid, kSplit, kFeat><<<grid, kBlock, ldsb, s>>>(a);
    } else if (acc == kAccBvh) {
        if (lds)
            trace_kernel<MAXD, true, kAccBvh, kSplit, kFeat><<<grid, kBlock, ldsb, s>>>(a);
        else
            trace_kernel<MAXD, false, kAccBvh, kSplit, kFeat><<<grid, kBlock, ldsb, s>>>(a);
    } else {
        if (fixed)
            trace_kernel<MAXD, true, false, kSplit, kFeat, false, kFixedSpheres><<<grid, kBlock, ldsb, s>>>(a);
        else if (lds)
            trace_kernel<MAXD, true, false, kSplit, kFeat><<<grid, kBlock, ldsb, s>>>(a);
        else
            trace_kernel<MAXD, false, false, kSplit, kFeat><<<grid, kBlock, ldsb, s>>>(a);
    }
    kernel_timing(s, 1);
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "trace_kernel launch");
    snprintf(g_last_launch, sizeof(g_last_launch),
             "kernel=trace_kernel maxd=%d lds=%d bvh=%d acc=%s split=%d samp=%d feat=%d ns=%d grid=%u tasks=%lld per_cu=%d",
             MAXD, lds ? 1 : 0, acc == kAccBvh ? 1 : 0, acc_name(acc), kSplit, samp ? 1 : 0, kFeat ? 1 : 0, fixed ? kFixedSpheres : 0,
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
    // kMaxSplit lanes per pixel. Fewer lanes per pixel than frames means several
    // rounds per wave task, i.e. fewer, longer tasks: with few pixels (one GPU's row shard
    // at 8 GPUs: 115,200 pixels at 32 spp) 7,200 tasks of 8 rounds on 4,096 waves left a
    // 1.7x tail (0.635 ms vs 0.365 for the same rays). Each lane replays its group's lerp
    // chain, so the merge costs kSplit steps per round: 16 measured best (shard of 8:
    // 0.437 ms, 32 lanes: 0.446; config 4 at 64 spp: 457 ms, 64 lanes: 478).
    int split = 1;
    while (split * 2 <= frames && split * 2 <= kMaxSplit) split *= 2;
    switch (split) {
        case 64: return launch_depth<MAXD, (kMaxSplit >= 64 ? 64 : 1)>(a, lds, xc, rows, s);
        case 32: return launch_depth<MAXD, (kMaxSplit >= 32 ? 32 : 1)>(a, lds, xc, rows, s);
        case 16: return launch_depth<MAXD, (kMaxSplit >= 16 ? 16 : 1)>(a, lds, xc, rows, s);
        case 8: return launch_depth<MAXD, (kMaxSplit >= 8 ? 8 : 1)>(a, lds, xc, rows, s);
        case 4: return launch_depth<MAXD, (kMaxSplit >= 4 ? 4 : 1)>(a, lds, xc, rows, s);
        case 2: return launch_depth<MAXD, (kMaxSplit >= 2 ? 2 : 1)>(a, lds, xc, rows, s);
        default: return launch_depth<MAXD, 1>(a, lds, xc, rows, s);
    }
}

}  // namespace lrt
