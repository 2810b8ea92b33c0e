// v5 (LRT_F_POOL): the v0 per-pixel loop with SAMPLE-POOL regeneration inside the wave.
//
// In v0 a wave task is a tile of pixels x frames, one pixel-sample per lane, and the bounce
// loop runs until the task's longest path ends. At 1000 spheres the closest-hit and shadow
// traversals dominate, and their wave executions carry few lanes: config 4 section counts
// (LRT_EXP_SECSTATS, profiles/r2_sec1) show ~6.7 bounce iterations per wave task while a
// path averages ~1.7 closest hits, so secondary closest-hit passes run at 20 lanes of 64
// and shadow passes at 10.
//
// Here a wave owns a tile of kPix pixels and works through a POOL of its pixel-samples,
// up to kPoolSamples per round (frame-major: sample k is frame fr0 + k / kPix of pixel
// k % kPix). A lane whose path ends folds its recursion stack (Trace's return value,
// parallel.cpp:214), stores the colour in the wave's slot k and takes the next sample
// index at once (ballot + mbcnt: no atomics). Every bounce iteration therefore traces
// (nearly) 64 paths until the pool runs dry. When the round's pool is done, lane j < kPix
// applies TraceRowJob's progressive lerp (parallel.cpp:262,280-286) to pixel j's colours
// in frame order -- the serial chain, so the result is bit-identical to the reference's
// frame-by-frame loop -- and the next round (or tile) starts.
//
// Same per-ray arithmetic, RNG streams (PixelSeed(x, y, f)), draw order, ray counting,
// Scatter and recursion fold as Trace (lrt_trace.h). The colour slots (12 B per sample of
// a round) live in global memory: LDS already holds the recursion stack.
#pragma once

namespace lrt {

enum : int { kPoolIdle = 0, kPoolTrace = 1, kPoolDone = 2, kPoolEnded = 3 };

template <int kPix>
struct PoolTile {   // tile shape: kPix pixels, as square as a power of two allows
    static constexpr int X = kPix >= 128 ? 16 : kPix >= 32 ? 8 : kPix >= 8 ? 4 : kPix >= 2 ? 2 : 1;
    static constexpr int Y = kPix / X;
    static_assert(X * Y == kPix && kPix <= 256, "kPix: a power of two up to 256");
};

// The kernel arguments a path start needs (camera, window), read where they are used through
// a pointer the compiler cannot hoist out of the loop (an empty asm launders it): held in
// SGPRs for the whole kernel, they pushed the traversal's own state into spills.
// (The kernel's only argument is the KernelArgs, at offset 0 of the kernarg segment; taking
// &a instead would copy the struct to scratch.)
#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(4))) KernelArgs* KArgPtr;
__device__ __forceinline__ KArgPtr opaque_args() {
    KArgPtr p = (KArgPtr)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return p;
}
#else   // (the host pass only parses the kernel)
typedef const KernelArgs* KArgPtr;
__device__ __forceinline__ KArgPtr opaque_args() { return nullptr; }
#endif

// The grid's spheres tested first by every query (the ground, the light: GridStart) are read
// from an LDS copy (at a.bvh_stack_offset: the grid has no traversal stack) instead of through
// L1/L2, and their uniform loads leave the walk's latency chain.
template <int kAcc, int kW>
__device__ __forceinline__ GridView pool_grid_view(float4* smem) {
    GridView g = opaque_args()->gv;
    {
        float4* b = reinterpret_cast<float4*>(reinterpret_cast<char*>(smem) + opaque_args()->bvh_stack_offset);
        g.bsph = b;
        g.bid = reinterpret_cast<const int*>(b + g.nbig);
    }
    if (kW > 1) {   // the block's copy of the cells and their spheres (pool_grid_lds)
        char* base = reinterpret_cast<char*>(smem) + opaque_args()->grid_lds_offset;
        const unsigned ncell = (unsigned)(g.nx * g.ny * g.nz), nref = g.cells_refs;
        g.rsph = reinterpret_cast<const float4*>(base);
        g.cells = reinterpret_cast<const uint2*>(base + 16 * nref);
        g.rid = reinterpret_cast<const int*>(base + 16 * nref + 8 * ncell);
    }
    return g;
}

// Blocks of kW > 1 waves (kPoolGridWaves, grid instances): the waves of a block share one
// LDS copy of the grid -- the cell ranges, the cell-ordered spheres and their indices
// (config 4: 1,044 cells and 1,742 references, 43 KB) -- so the walk's dependent loads are LDS
// reads (~50 cycles) instead of L1/L2 hits. Each wave keeps its own recursion stack (below).
constexpr int kPoolGridWaves = 16;
// Every instance keeps kTraceLdsLevels (8) recursion levels per lane in LDS. The grid
// instance's 16-wave blocks keep them PACKED -- planes of x, y and z floats and one of u16
// material ids, 14 B a level instead of a float4's 16 -- so that 16 stacks of 8 levels take the
// 112 KB that 7 float4 levels took and still fit beside the grid in the CU's 160 KB. (Round 4
// had 7 float4 levels there and the eighth in the global overflow stack, whose per-lane
// pointers also held registers.) Bytes per wave:
template <int kW>
constexpr int pool_stack_bytes() { return 64 * kTraceLdsLevels * (kW > 1 ? 14 : 16); }

template <int MAXD, bool kLds, int kAcc, int kPix, int kNS = 0, int kW = 1>
__global__ __launch_bounds__(64 * kW, kWavesPerEU) void pool_kernel(
    const KernelArgs a) {
    static_assert(kNS == 0 || (kLds && !kAcc), "a fixed sphere count is for the LDS linear scan");
    static_assert(kW == 1 || (kAcc == kAccGrid && !kLds), "multi-wave blocks: the grid instance");
    constexpr int kLv = kTraceLdsLevels;   // recursion stack levels in LDS
    constexpr bool kPacked = kW > 1;        // (pool_stack_bytes)
    // LDS as trace_kernel: [recursion stack kTraceLdsLevels x 64][powf tables][renormalize
    // table unless kAcc][spheres][materials][lights][bvh stack at a.bvh_stack_offset]
    extern __shared__ float4 smem[];
    const int lane = kW > 1 ? (int)(threadIdx.x & 63u) : (int)threadIdx.x;
    const int tid = threadIdx.x;   // fills of the block-shared LDS
    // this wave's place among all waves (kW > 1: several per block, each as a block of one)
    const int wave = kW > 1 ? (int)(threadIdx.x >> 6) : 0;
    const int wid = (int)blockIdx.x * kW + wave;
    const int nwaves = (int)gridDim.x * kW;
    (void)nwaves;
    double* s_pow = reinterpret_cast<double*>(reinterpret_cast<char*>(smem) + kW * pool_stack_bytes<kW>());
    {
        const libm::PowTables g = libm::pow_tables();
        for (int i = tid; i < 16; i += 64 * kW) {
            s_pow[i] = g.invc[i];
            s_pow[16 + i] = g.logc[i];
        }
        for (int i = tid; i < 32; i += 64 * kW) reinterpret_cast<uint64_t*>(s_pow + 32)[i] = g.exp2[i];
    }
    constexpr int kLutBytes = kAcc ? 0 : kRenormBytes;
    float* s_lut = kAcc ? nullptr : reinterpret_cast<float*>(s_pow + 64);
    if (!kAcc) renorm_lut_fill(s_lut, lane, 64);
    float4* s_sph = reinterpret_cast<float4*>(reinterpret_cast<char*>(smem) + kW * pool_stack_bytes<kW>() +
                                              kPowTableBytes + kLutBytes);
    float4* s_mat = s_sph + a.count;
    int* s_lights = reinterpret_cast<int*>(s_mat + 3 * a.count);
    if (kLds) {
        for (int i = lane; i < a.count; i += 64) s_sph[i] = a.sph[i];
        for (int i = lane; i < 3 * a.count; i += 64) s_mat[i] = a.mats[i];
        for (int i = lane; i < a.nlights; i += 64) s_lights[i] = a.lights[i];
    }
    if (kAcc == kAccGrid) {   // (pool_grid_view)
        float4* b = reinterpret_cast<float4*>(reinterpret_cast<char*>(smem) + a.bvh_stack_offset);
        for (int i = tid; i < a.gv.nbig; i += 64 * kW) {
            b[i] = a.gv.bsph[i];
            reinterpret_cast<int*>(b + a.gv.nbig)[i] = a.gv.bid[i];
        }
    }
    if (kW > 1) {   // the grid's LDS copy (pool_grid_view)
        char* base = reinterpret_cast<char*>(smem) + a.grid_lds_offset;
        const int ncell = a.gv.nx * a.gv.ny * a.gv.nz, nref = (int)a.gv.cells_refs;
        for (int i = tid; i < nref; i += 64 * kW) {
            reinterpret_cast<float4*>(base)[i] = a.gv.rsph[i];
            reinterpret_cast<int*>(base + 16 * nref + 8 * ncell)[i] = a.gv.rid[i];
        }
        for (int i = tid; i < ncell; i += 64 * kW) reinterpret_cast<uint2*>(base + 16 * nref)[i] = a.gv.cells[i];
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
    // (the grid's view is read from the kernel arguments where a walk starts, below: held in
    // SGPRs for the whole kernel its ~28 scalars spilled the loop's own state)
    sc.bstk = reinterpret_cast<unsigned short*>(reinterpret_cast<char*>(smem) + a.bvh_stack_offset) + lane;
    sc.bstride = 64;
#ifdef LRT_EXP_SECSTATS
    __shared__ unsigned long long s_sectime[kW][2 + 3 * kSecN];
    sc.secstats = a.wtrace;
    sc.sectime = s_sectime[wave];
    if (lane == 0) {
        for (int k = 0; k < 2 + 3 * kSecN; ++k) sc.sectime[k] = 0;
        sc.sectime[0] = kSecOther;
        sc.sectime[1] = __builtin_amdgcn_s_memtime();
    }
#endif
#ifdef LRT_EXP_WAVETRACE
    const unsigned long long wt0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long wc0 = __builtin_amdgcn_s_memtime();   // (LRT_EXP_WAVECLK: shader cycles)
    unsigned long long wlast = 0, wtiles = 0;   // the last task's start, the task count
#endif
    float4* const lstk = smem + wave * kLv * 64 + lane;   // this lane's recursion stack (LDS)
    // (packed: the x plane at lane, then y, z, and the u16 ids after the three float planes)
    float* const pstk = reinterpret_cast<float*>(reinterpret_cast<char*>(smem) + wave * pool_stack_bytes<kW>()) + lane;
    unsigned short* const pids = reinterpret_cast<unsigned short*>(pstk - lane + 3 * kLv * 64) + lane;
    const size_t gtid = (size_t)wid * 64 + lane;
    const size_t gthreads = (size_t)nwaves * 64;
    // Levels >= kLv (MAXD > 8) in the global overflow stack: a u16 per level (the
    // material id, bit 15 set when the level's matE + lightE is exactly +0, which then needs no
    // float4 at all -- the fold adds the literal +0 the stored value was, parallel.cpp:214) and
    // the float4 only for the others. Deep levels are mostly glass and metal chains, whose
    // events add nothing (round 3 stored a float4 per level).
    float4* const gstk = a.ovf + gtid;
    unsigned short* const gid =
        reinterpret_cast<unsigned short*>(a.ovf + gthreads * (size_t)(a.maxDepth - kLv)) + gtid;
    auto put = [&](int lvl, float4 v) {
        if (MAXD <= kLv || lvl < kLv) {
            if constexpr (kPacked) {
                pstk[lvl * 64] = v.x;
                pstk[(kLv + lvl) * 64] = v.y;
                pstk[(2 * kLv + lvl) * 64] = v.z;
                pids[lvl * 64] = (unsigned short)__float_as_int(v.w);
            } else {
                lstk[lvl * 64] = v;
            }
        } else {
            const size_t o = (size_t)(lvl - kLv) * gthreads;
            const bool z = (__float_as_uint(v.x) | __float_as_uint(v.y) | __float_as_uint(v.z)) == 0u;
            gid[o] = (unsigned short)(__float_as_int(v.w) | (z ? 0x8000 : 0));
            if (!z) gstk[o] = v;
        }
    };
    auto get = [&](int lvl) -> float4 {
        if (MAXD <= kLv || lvl < kLv) {
            if constexpr (kPacked)
                return make_float4(pstk[lvl * 64], pstk[(kLv + lvl) * 64], pstk[(2 * kLv + lvl) * 64],
                                   __int_as_float((int)pids[lvl * 64]));
            return lstk[lvl * 64];
        }
        const size_t o = (size_t)(lvl - kLv) * gthreads;
        const unsigned t = gid[o];
        if (t & 0x8000u) return make_float4(0.0f, 0.0f, 0.0f, __int_as_float((int)(t & 0x7fffu)));
        return gstk[o];
    };
    // this wave's colour slots: RGB, 12 B per sample (the 4th float was never read)
    float* const slots = a.colbuf + (size_t)wid * a.poolSlots * 3;

    constexpr int TX = PoolTile<kPix>::X, TY = PoolTile<kPix>::Y;
    constexpr int kLgPix = kPix >= 256 ? 8 : kPix >= 128 ? 7 : kPix >= 64 ? 6 : kPix >= 32 ? 5 : kPix >= 16 ? 4
                         : kPix >= 8 ? 3 : kPix >= 4 ? 2 : kPix >= 2 ? 1 : 0;
    constexpr int kLgTX = TX >= 16 ? 4 : TX >= 8 ? 3 : TX >= 4 ? 2 : TX >= 2 ? 1 : 0;
    static_assert((1 << kLgPix) == kPix && (1 << kLgTX) == TX, "tiles: powers of two");
    const int tilesX = (a.xc + TX - 1) / TX;
    const int ntiles = tilesX * ((a.rows + TY - 1) / TY);
    // Split tail (a.splitFrom; the depth-8 one-wave linear-scan instances, whose launches have
    // few tiles per wave): the queue's items from splitFrom on are the last -- lightest, in
    // heaviest-first order -- tiles' left and right halves, so that a launch alone ends at
    // half-tile granularity while its other pools keep the full tile's size (launch_pool).
    constexpr bool kSplit = kW == 1 && TX >= 2 && MAXD <= 8 && kAcc == kAccScan;
    const int splitFrom = kSplit ? (a.splitFrom < ntiles ? a.splitFrom : ntiles) : ntiles;
    const int nitems = ntiles + (ntiles - splitFrom);
    const float invWidth = 1.0f / (float)a.width;     // parallel.cpp:260
    const float invHeight = 1.0f / (float)a.height;   // parallel.cpp:261
    const int fend = a.frame0 + a.frames;
    const unsigned long long below = (1ull << lane) - 1ull;   // lanes before this one
    int rays = 0;
    // tile queues, as v0: block b serves queue b % kV0Queues (XCD-local counters)
    // (kW > 1: the block's waves share its queue, so that a queue's counters stay in one XCD)
    const int q = blockIdx.x % kV0Queues;
    const int bq = (((int)gridDim.x - q + kV0Queues - 1) / kV0Queues) * kW;   // waves serving queue q
    const int nq = (nitems - q + kV0Queues - 1) / kV0Queues;
    unsigned long long* ctr = a.tiles + q * kCtrStride;
    // late tile reservation and issue priority by occupancy (below): the depth-8 one-wave instances
    constexpr bool kLate = kW == 1 && MAXD <= 8;
    for (int i = (int)(blockIdx.x / kV0Queues) * kW + wave; i < nq;) {
        const int task = q + kV0Queues * i;
        // a whole tile, or (task >= splitFrom) one half of a tail tile
        const int h = task - splitFrom;
        const bool half = kSplit && h >= 0;
        const int ord = half ? splitFrom + (h >> 1) : task;
        const int tile = a.perm ? a.perm[ord] : ord;   // heaviest-first order (tile_order)
        const unsigned long long tt0 = a.tcost ? __builtin_amdgcn_s_memrealtime() : 0ull;
#ifdef LRT_EXP_WAVETRACE
        wlast = __builtin_amdgcn_s_memrealtime();
        ++wtiles;
#endif
        // the pool: 2^lgP pixels in rows of 2^lgW from (tx0, ty0)
        const int lgW = half ? kLgTX - 1 : kLgTX;
        const int lgP = half ? kLgPix - 1 : kLgPix;
        const int tx0 = (tile % tilesX) * TX + (half ? (h & 1) << lgW : 0), ty0 = (tile / tilesX) * TY;
        const int roundFrames = kPoolSamples >> lgP;
        // The next tile is reserved (queue atomic) at this tile's start, which hides the atomic's
        // latency behind the whole tile -- or, in launches of few tiles per wave (a.lateFetch:
        // config 2 has 3.5), once this tile's last samples are handed out: a tile reserved at the
        // start of the one before it is held by a wave still a whole tile away from it, and at the
        // launch's end the queue's last tiles waited for such waves while others found the queue
        // empty (profiles/r5_m). Config 2 alone 0.272 -> 0.259 ms, two streams within noise
        // (profiles/r5_z); with many tiles per wave the exposed latency costs more than the tail
        // (configs 3-4: +1-2 %, r5_n); only the depth-8 one-wave instances carry the code (its
        // presence alone cost config 3's instance 0.9 %, r5_aa).
        unsigned long long fetched = 0;
        bool asked = !(kLate && a.lateFetch);
        if (asked && lane == 0) fetched = atomicAdd(ctr, 1ull);   // consumed after the tile
        for (int fr0 = a.frame0; fr0 < fend; fr0 += roundFrames) {
            const int nfr = fend - fr0 < roundFrames ? fend - fr0 : roundFrames;
            const int N = nfr << lgP;   // this round's pool
            int next = 0, state = kPoolIdle, k = 0, depth = 0;
            bool prevLambert = false;
            uint32_t rng = 1;
            Ray r;   // the ray to trace next (a camera ray, or the last scatter's bounce ray)
            r.orig = f3(0.0f, 0.0f, 0.0f);
            r.dir = f3(0.0f, 1.0f, 0.0f);
            // the last scatter event, pushed on the stack but not yet counted in `depth`: its
            // deferred shadow ray (the last light's, as TraceDual) is traced in the same
            // pass as the bounce ray; carry = its stack value should the light be reached
            bool pend = false;
            F3 carry = f3(0.0f, 0.0f, 0.0f);
            DeferredLight dl;
            dl.on = false;
            dl.li = -1;
            dl.l = f3(0.0f, 0.0f, 0.0f);
            dl.contrib = f3(0.0f, 0.0f, 0.0f);
            for (;;) {
                // ---- refill: ended paths are folded and their lanes take the pool's next
                // samples, together once a.regenMin lanes wait (or no path is left to trace),
                // so the fold and the camera rays run with more lanes than end per bounce ----
                const unsigned long long waitM = __ballot(state == kPoolIdle || state == kPoolEnded);
                if (waitM && (__popcll(waitM) >= a.regenMin || __ballot(state == kPoolTrace) == 0)) {
                    if (state == kPoolEnded) {   // :214 folded leaf-outwards into the sample's slot
                        sec_count(sc, kSecFold);
                        F3 T = carry;
                        for (int d = depth - 1; d >= 0; --d) {
                            const float4 s = get(d);
                            const float4 b = sc.mats[3 * __float_as_int(s.w) + 2];
                            T = f3(s.x, s.y, s.z) + f3(b.x, b.y, b.z) * T;
                        }
                        slots[3 * k] = T.x;
                        slots[3 * k + 1] = T.y;
                        slots[3 * k + 2] = T.z;
                        state = kPoolIdle;
                    }
                    const unsigned long long needM = waitM;
                    if (state == kPoolIdle) {
                        k = next + __popcll(needM & below);
                        state = kPoolDone;
                        if (k < N) {
                            const int j = k & ((1 << lgP) - 1), f = fr0 + (k >> lgP);
                            const int lx = tx0 + (j & ((1 << lgW) - 1)), ly = ty0 + (j >> lgW);
                            const KArgPtr pa = opaque_args();   // window and camera, read here
                            if (lx < pa->xc && ly < pa->rows) {   // TraceRowJob's per-pixel body (:270-279)
                                sec_count(sc, kSecCamera);
                                const int x = pa->x0 + lx;
                                const int rb = pa->rb;
                                const int y = pa->y0 + (ly / rb) * rb * pa->rp + pa->rph * rb + ly % rb;
                                rng = PixelSeed((uint32_t)x, (uint32_t)y, (uint32_t)f);
                                const float u = ((float)x + RandomFloat01(rng)) * invWidth;    // :272
                                const float v = ((float)y + RandomFloat01(rng)) * invHeight;   // :273
                                const CameraDev cam = pa->cam;
                                r = GetRay(cam, u, v, rng, sc.rnlut);
                                depth = 0;
                                prevLambert = false;
                                pend = false;
                                state = kPoolTrace;
                            } else {
                                state = kPoolIdle;   // outside the window: nothing to trace
                            }
                        }
                    }
                    next += __popcll(needM);
                    if constexpr (kLate) {
                        if (!asked && next >= N && fr0 + roundFrames >= fend) {   // the tile's last samples
                            if (lane == 0) fetched = atomicAdd(ctr, 1ull);
                            asked = true;
                        }
                    }
                }
                const unsigned long long traceM = __ballot(state == kPoolTrace);
                if (traceM == 0) {
                    if (__ballot(state == kPoolIdle || state == kPoolEnded) == 0) break;   // the pool is dry
                    continue;
                }
                // A wave tracing few paths (its pool draining) yields the SIMD's issue slots to the
                // fuller waves beside it: config 2 alone 0.2598 -> 0.2527 ms, two streams and
                // configs 3-4 within noise (profiles/r5_al); the depth-8 one-wave instances only
                if constexpr (kLate) {
                    if (__popcll(traceM) < 24) __builtin_amdgcn_s_setprio(0);
                    else __builtin_amdgcn_s_setprio(1);
                }
                // (no packet traversal here: without its code the instance keeps its traversal
                // state in fewer registers, config 4: 222.4 -> 209.8 ms/step, profiles/r2_q2)
                constexpr bool coherent = false;
                sec_enter(sc, kSecOther, false);
                // ---- one bounce of every traced path: Trace's body (parallel.cpp:202-226) ----
                int nid = -1;
                float nt = 0.0f;
                bool shade = false, fin = false;
                F3 leaf = f3(0.0f, 0.0f, 0.0f);
                if (state == kPoolTrace) {
                    // HitWorld of r (:204-205) and the pending shadow ray (:122-123) in one pass
                    sec_count(sc, coherent ? kSecHit0 : kSecHit);
                    ++rays;
                    bool lit = false;
                    const bool hasS = pend && dl.on;
                    if constexpr (kAcc == kAccGrid) {
                        const float4 ls = hasS ? sc.sph[dl.li] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                        const GridView gv = pool_grid_view<kAcc, kW>(smem);
                        nid = ClosestHitDualGrid<(kW > 1 ? 1 : 0)>(r.orig, r.dir, hasS, dl.l, dl.li, ls, gv, nt, lit);
                    } else if constexpr (kAcc == kAccBvh) {
                        if (coherent) {
                            nid = ClosestHitBVH(r.orig, r.dir, sc.bv, nt, sc.bstk, sc.bstride, nullptr, true);
                        } else {
                            const float4 ls = hasS ? sc.sph[dl.li] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                            nid = ClosestHitDualBVH4(r.orig, r.dir, hasS, dl.l, dl.li, ls, sc.bv, nt, lit, sc.bstk,
                                                     sc.bstride);
                        }
                    } else {
                        int sid;
                        DualClosestHit<kNS>(r.orig, r.dir, hasS, dl.l, sc, nid, nt, sid);
                        lit = hasS && sid == dl.li;
                    }
                    if (pend) {   // the scatter event that produced r (:214), with its light if reached
                        if (lit) put(depth, make_float4(carry.x, carry.y, carry.z, __int_as_float(dl.id)));
                        ++depth;
                        pend = false;
                    }
                    if (nid < 0) {   // sky (:223-225)
                        const float t = 0.5f * (r.dir.y + 1.0f);
                        leaf = ((1.0f - t) * f3(1.0f, 1.0f, 1.0f) + t * f3(0.5f, 0.7f, 1.0f)) * 0.3f;
                        fin = true;
                    } else {
                        shade = true;
                    }
                }
                if (shade) {   // HitWorld's winner (maths.cpp:74-76,86-88), then Scatter (:210-212)
                    const float4 sp4 = sc.sph[nid];
                    Hit rec;
                    rec.pos = point_at(r, nt);
                    rec.normal = normalize(rec.pos - f3(sp4.x, sp4.y, sp4.z));
                    rec.t = nt;
                    const Material mat = load_material(sc.mats, nid);
                    F3 matE = mat.emissive;
                    fin = true;
                    leaf = matE;
                    if (depth < a.maxDepth) {
                        F3 lightE;
                        dl.on = false;
                        if constexpr (kAcc == kAccGrid) sc.gv = pool_grid_view<kAcc, kW>(smem);   // other lights' shadow rays
                        const F3 X = ScatterDir<kAcc, kNS>(mat, nid, r, rec, lightE, rays, rng, sc, &dl, coherent);
                        sec_count(sc, kSecPost);
                        const F3 dir = renormalize(normalize(X), sc.rnlut);   // Ray(rec.pos, normalize(X))
                        if ((mat.type != 1) | (dot(dir, rec.normal) > 0.0f)) {    // Metal absorbs (:147)
                            if (a.ndl && prevLambert) matE = f3(0.0f, 0.0f, 0.0f);
                            prevLambert = mat.type == 0;
                            const F3 e = matE + lightE;
                            put(depth, make_float4(e.x, e.y, e.z, __int_as_float(nid)));
                            if (dl.on) carry = matE + (lightE + dl.contrib);   // TraceDual's order
                            dl.id = nid;
                            pend = true;
                            r.orig = rec.pos;
                            r.dir = dir;
                            fin = false;
                        }
                    }
                }
                if (fin) {   // the path's leaf colour waits for the fold at the next refill
                    carry = leaf;
                    state = kPoolEnded;
                }
            }
            // ---- the round's colours in frame order, one lane per pixel (:262,282) ---------
            // Lane j owns pixels j, j + 64, ... of the tile. Its address and previous value are
            // taken here, not held in registers through the bounce loop (fewer live VGPRs in
            // the traversal); a later round re-reads what this one wrote.
            sec_enter(sc, kSecOther, false);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            const KArgPtr pa = opaque_args();   // output window, lerp table, frame: read here
            const int xc = pa->xc, rows = pa->rows;
            float4* const out = pa->out;
            const float* const lerp = pa->lerp;
            float4* const frame = pa->frame;
            for (int j0 = 0; j0 < (1 << lgP); j0 += 64) {   // pools above 64 pixels: several per lane
                const int j = j0 + lane;
                const int mx = tx0 + (j & ((1 << lgW) - 1)), my = ty0 + (j >> lgW);
                if (j < (1 << lgP) && mx < xc && my < rows) {
                    float4* const mpx = out + (size_t)my * xc + mx;
                    float4 acc = *mpx;
                    F3 c3 = f3(acc.x, acc.y, acc.z);
                    int t = 0;
                    // four frames at a time: their colours and factors are read together (one
                    // memory latency per four frames instead of one per frame), then chained in
                    // frame order (config 2 -0.9 %, config 3 -1.0 %, profiles/r6_an)
                    for (; t + 4 <= nfr; t += 4) {
                        F3 c[4];
                        float lf[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const float* const cp = slots + 3 * (((t + u) << lgP) + j);
                            c[u] = f3(cp[0], cp[1], cp[2]);
                            const int f = fr0 + t + u;
                            lf[u] = f < kLerpTable ? lerp[f] : (float)f / (float)(f + 1);
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u) c3 = c3 * lf[u] + c[u] * (1.0f - lf[u]);
                    }
                    for (; t < nfr; ++t) {
                        const float* const cp = slots + 3 * ((t << lgP) + j);
                        const F3 c = f3(cp[0], cp[1], cp[2]);
                        const int f = fr0 + t;
                        const float lerpFac = f < kLerpTable ? lerp[f] : (float)f / (float)(f + 1);
                        c3 = c3 * lerpFac + f3(c.x, c.y, c.z) * (1.0f - lerpFac);
                    }
                    acc.x = c3.x;
                    acc.y = c3.y;
                    acc.z = c3.z;
                    *mpx = acc;   // alpha as read
                    if (frame) {   // the exchange, fused: the pixel at its global row (GlobalRow)
                        const int rb = pa->rb;
                        const int gy = pa->y0 + (my / rb) * rb * pa->rp + pa->rph * rb + my % rb;
                        frame[(size_t)gy * pa->width + pa->x0 + mx] = acc;
                    }
                }
            }
            // the next round overwrites the slots: every read above completes first
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
        // recording launch: the tile's cost = its wall time (the rays it traced ordered config 2
        // worse: 0.300 against 0.276 ms alone, profiles/r5_p)
        if (a.tcost && lane == 0) a.tcost[tile] = (unsigned)(__builtin_amdgcn_s_memrealtime() - tt0);
        if constexpr (kLate)
            if (!asked && lane == 0) fetched = atomicAdd(ctr, 1ull);   // (a tile whose pool never ran dry)
        const unsigned long long n = __shfl(fetched, 0, 64) + (unsigned long long)bq;
        i = n < (unsigned long long)nq ? (int)n : nq;
    }
#ifdef LRT_EXP_SECSTATS
    sec_enter(sc, kSecOther, false);
    if (lane == 0)
        for (int k = 0; k < kSecN; ++k) {
            unsigned long long* g = sc.secstats + 3 * (k + kSecN * (wid & 15));
            atomicAdd(g, sc.sectime[2 + kSecN + k]);
            atomicAdd(g + 1, sc.sectime[2 + 2 * kSecN + k]);
            atomicAdd(g + 2, sc.sectime[2 + k]);
        }
#endif
#ifdef LRT_EXP_WAVETRACE
    if (lane == 0) {
        a.wtrace[4 * wid + 0] = wt0;
        a.wtrace[4 * wid + 1] = __builtin_amdgcn_s_memrealtime();
        a.wtrace[4 * wid + 2] = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) |   // HW_ID
                                ((unsigned long long)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32) |  // XCC_ID
                                (wtiles << 40);
#ifdef LRT_EXP_WAVECLK
        a.wtrace[4 * wid + 3] = __builtin_amdgcn_s_memtime() - wc0;   // the wave's life in shader cycles
#else
        a.wtrace[4 * wid + 3] = wlast;
#endif
    }
#endif
    const unsigned long long total = wave_sum((unsigned long long)rays);
    if (lane == 0) block_epilogue(a.tiles, a.rays, q, bq, total);
}

}  // namespace lrt
