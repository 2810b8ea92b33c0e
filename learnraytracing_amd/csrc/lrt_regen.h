// v3: the v0 per-pixel loop with PATH REGENERATION inside the wave.
//
// v0 gives every lane one pixel-sample; a wave then runs as long as its longest path.
// Path lengths are very uneven (default scene, D = 8: counted rays per pixel-sample are
// 2-17, mean 3.8), so only ~38 % of the lane-iterations of the bounce loop do work
// (oracle path lengths on a 256x128 crop, 8x2-pixel x 4-frame waves) -- the same 36.5 %
// lane utilisation rocprof measures (profiles/r1_v5).
//
// Here a lane owns one PIXEL at a time and traces its frames one after another
// (frame0, frame0 + 1, ...), lerping each finished sample into the pixel's running value
// exactly as TraceRowJob does (parallel.cpp:262,280-286), so the result is bit-identical
// to the serial loop. When a lane's path ends it waits; once `regenMin` lanes of the
// wave have ended (or nothing else is left to do) they are regenerated together: fold of
// the recursion stack, lerp, next frame's camera ray (GetRay, maths.h:205-215) or, after
// the pixel's last frame, store and the next pixel. Pixels come from the wave's stream of
// 8x8-pixel tiles (the v0 tile queues, one atomic per 64 pixels), handed to the waiting
// lanes by ballot + mbcnt -- no per-pixel atomics. Each loop iteration then runs one
// closest-hit pass for every lane holding a ray (camera rays and bounce rays together, the
// bounce ray sharing its pass with the last light's deferred shadow ray as in TraceDual)
// and one shading step.
//
// Same per-ray arithmetic, RNG streams (PixelSeed(x, y, f)), draw order, ray counting and
// recursion fold as Trace/TraceDual in lrt_trace.h.
#pragma once

namespace lrt {

#ifndef LRT_V3_WAVES_PER_EU
#define LRT_V3_WAVES_PER_EU 4
#endif

// Lane states at the top of an iteration.
enum : int { kV3Trace = 0, kV3Ended = 1, kV3Dead = 2 };

// Stage powf tables, spheres, materials and lights into LDS and describe the scene
// (the same layout as trace_kernel: [stack kTraceLdsLevels x 64][powf tables][spheres]
// [materials][lights][bvh stack]).
template <bool kLds>
__device__ __forceinline__ SceneView stage_scene(const KernelArgs& a, float4* smem, int tid, int block) {
    double* s_pow = reinterpret_cast<double*>(smem + kTraceLdsLevels * block);
    {
        const libm::PowTables g = libm::pow_tables();
        for (int i = tid; i < 16; i += block) {
            s_pow[i] = g.invc[i];
            s_pow[16 + i] = g.logc[i];
        }
        for (int i = tid; i < 32; i += block) reinterpret_cast<uint64_t*>(s_pow + 32)[i] = g.exp2[i];
    }
    float* s_lut = reinterpret_cast<float*>(s_pow + 64);   // renormalize() table
    renorm_lut_fill(s_lut, tid, block);
    float4* s_sph = smem + kTraceLdsLevels * block + (kPowTableBytes + kRenormBytes) / 16;
    float4* s_mat = s_sph + a.count;
    int* s_lights = reinterpret_cast<int*>(s_mat + 3 * a.count);
    if (kLds) {
        for (int i = tid; i < a.count; i += block) s_sph[i] = a.sph[i];
        for (int i = tid; i < 3 * a.count; i += block) s_mat[i] = a.mats[i];
        for (int i = tid; i < a.nlights; i += block) s_lights[i] = a.lights[i];
    }
    __syncthreads();
    SceneView sc;
    sc.pow.invc = s_pow;
    sc.pow.logc = s_pow + 16;
    sc.pow.exp2 = reinterpret_cast<const uint64_t*>(s_pow + 32);
    sc.rnlut = s_lut;
    sc.sph = kLds ? s_sph : a.sph;
    sc.gsph = a.sph;
    sc.mats = kLds ? s_mat : a.mats;
    sc.lights = kLds ? s_lights : a.lights;
    sc.count = a.count;
    sc.nlights = a.nlights;
    sc.bv = a.bv;
    sc.bstk = reinterpret_cast<unsigned short*>(reinterpret_cast<char*>(smem) + a.bvh_stack_offset) + tid;
    sc.bstride = block;
    return sc;
}

template <int MAXD, bool kLds, bool kBvh, int kSplit>
__global__ __launch_bounds__(64, LRT_V3_WAVES_PER_EU) void regen_kernel(const KernelArgs a) {
    extern __shared__ float4 smem[];
    const int lane = threadIdx.x;
    SceneView sc = stage_scene<kLds>(a, smem, lane, 64);
#ifdef LRT_EXP_SECSTATS
    __shared__ unsigned long long s_sectime[2 + 3 * kSecN];
    sc.secstats = a.wtrace;
    sc.sectime = s_sectime;
    if (lane == 0) {
        for (int k = 0; k < 2 + 3 * kSecN; ++k) sc.sectime[k] = 0;
        sc.sectime[0] = kSecOther;
        sc.sectime[1] = __builtin_amdgcn_s_memtime();
    }
#endif
    float4* const lstk = smem + lane;                       // this lane's recursion stack (LDS)
    const size_t gtid = (size_t)blockIdx.x * 64 + lane;
    const size_t gthreads = (size_t)gridDim.x * 64;
    float4* const gstk = a.ovf + gtid;                      // levels >= kTraceLdsLevels (MAXD > 8)
    auto put = [&](int lvl, float4 v) {
        if (MAXD <= kTraceLdsLevels || lvl < kTraceLdsLevels) lstk[lvl * 64] = v;
        else gstk[(size_t)(lvl - kTraceLdsLevels) * gthreads] = v;
    };
    auto get = [&](int lvl) -> float4 {
        if (MAXD <= kTraceLdsLevels || lvl < kTraceLdsLevels) return lstk[lvl * 64];
        return gstk[(size_t)(lvl - kTraceLdsLevels) * gthreads];
    };

    // pixel groups: kSplit adjacent lanes own one pixel and trace its frames f0 + sub in
    // parallel (v0's split); a tile is 8 x (8 / kSplit) pixels = one wave's worth of lanes
    constexpr int kTilePix = 64 / kSplit;
    constexpr int kTileRows = 8 / kSplit;
    constexpr unsigned long long kGroupBits = (1ull << kSplit) - 1ull;
    const int sub = lane % kSplit;
    const int g0 = lane - sub;                         // first lane of this lane's group
    const int tilesX = (a.xc + 7) / 8;
    const int ntiles = tilesX * ((a.rows + kTileRows - 1) / kTileRows);
    const float invWidth = 1.0f / (float)a.width;     // parallel.cpp:260
    const float invHeight = 1.0f / (float)a.height;   // parallel.cpp:261
    const int fend = a.frame0 + a.frames;
    const int q = blockIdx.x % kV0Queues;
    const int bq = ((int)gridDim.x - q + kV0Queues - 1) / kV0Queues;   // blocks serving queue q
    const int nq = (ntiles - q + kV0Queues - 1) / kV0Queues;            // tiles owned by queue q
    unsigned long long* const ctr = a.tiles + q * kCtrStride;

    // The wave's pixel stream: tile `cur` covers stream positions [base, base + kTilePix),
    // tile `nxt` the next kTilePix; `cursor` is the next position to hand out (a round of
    // hand-outs takes at most kTilePix positions, so it never reaches past nxt). The first
    // two tiles are static (queue rounds 0 and 1); later ones come from the queue's
    // counter, fetched when the stream moves on and read when they are needed.
    int cur = blockIdx.x / kV0Queues;
    int nxt = cur + bq;
    bool nxtKnown = true;
    unsigned long long fetched = 0;
    int base = 0, cursor = 0;
    bool poolDone = cur >= nq;

    int rays = 0;
    int state = kV3Ended;
    bool haveLeaf = false;          // the ended path has a colour for this round
    int f0 = fend;                  // the group's current round of frames f0 .. f0 + kSplit - 1
    int lx = 0, ly = 0;             // the group's pixel (window coordinates)
    F3 acc = f3(0.0f, 0.0f, 0.0f);  // the pixel's running value (channels 0-2), in every lane of the group
    uint32_t rng = 0;
    Ray r;                          // the ray to trace / the ray that reached rec
    r.orig = f3(0.0f, 0.0f, 0.0f);
    r.dir = f3(0.0f, 1.0f, 0.0f);
    // carry: the ended path's leaf colour (Ended lanes) or the pending event's lit sum
    // (Trace lanes with pend) -- a lane never needs both
    F3 carry = f3(0.0f, 0.0f, 0.0f);
    int id = 0, depth = 0;
    bool prevLambert = false;
    // scatter event waiting for its closest-hit pass (the deferred shadow ray's result)
    bool pend = false;
    DeferredLight dl;
    dl.on = false;
    dl.li = -1;
    dl.l = f3(0.0f, 0.0f, 0.0f);
    dl.contrib = f3(0.0f, 0.0f, 0.0f);

    for (;;) {
        // ---- regeneration of the groups whose lanes have all ended -------------------
        const unsigned long long endedM = __ballot(state == kV3Ended);
        const bool ready = state == kV3Ended && ((endedM >> g0) & kGroupBits) == kGroupBits;
        const unsigned long long readyM = __ballot(ready);
        const unsigned long long traceM = __ballot(state == kV3Trace);
        if (readyM && (__popcll(readyM) >= a.regenMin || poolDone || traceM == 0)) {
            bool need = false;
            if (ready) {
                sec_count(sc, kSecFold);
                F3 T = carry;
                if (haveLeaf) {   // Trace's return value (parallel.cpp:214) folded leaf-outwards
                    for (int d = depth - 1; d >= 0; --d) {
                        const float4 s = get(d);
                        const float4 b = sc.mats[3 * __float_as_int(s.w) + 2];
                        T = f3(s.x, s.y, s.z) + f3(b.x, b.y, b.z) * T;
                    }
                }
                haveLeaf = false;
                if (f0 < fend) {
                    // the round's colours in frame order (parallel.cpp:262,282), every lane of
                    // the group computing the same running value
#pragma unroll
                    for (int j = 0; j < kSplit; ++j) {
                        F3 c = T;
                        if (kSplit > 1) c = f3(__shfl(T.x, g0 + j, 64), __shfl(T.y, g0 + j, 64), __shfl(T.z, g0 + j, 64));
                        const int fj = f0 + j;
                        if (fj < fend) {
                            const float lerpFac = (float)fj / (float)(fj + 1);
                            acc = acc * lerpFac + c * (1.0f - lerpFac);
                        }
                    }
                    f0 += kSplit;
                    if (f0 >= fend && sub == 0) {   // :283-285, alpha untouched
                        float* o = reinterpret_cast<float*>(a.out + (size_t)ly * a.xc + lx);
                        o[0] = acc.x;
                        o[1] = acc.y;
                        o[2] = acc.z;
                    }
                }
                need = f0 >= fend;
            }
            // groups whose pixel is complete take the next pixels of the wave's stream
            for (;;) {
                const unsigned long long needM = __ballot(need && sub == 0);   // one bit per group
                if (needM == 0) break;
                if (poolDone) {
                    if (need) state = kV3Dead;
                    break;
                }
                const int n = __popcll(needM);
                if (!nxtKnown && cursor + n - base > kTilePix) {   // positions in nxt are handed out
                    nxt = (int)__builtin_amdgcn_readlane((int)fetched, 0) + 2 * bq;
                    nxtKnown = true;
                }
                if (need) {
                    const int rank = __popcll(needM & ((1ull << g0) - 1ull));   // groups before this one
                    const int k = cursor + rank - base;   // < 2 * kTilePix
                    const int ti = k < kTilePix ? cur : nxt;
                    const int j = k % kTilePix;
                    if (ti < nq) {
                        const int tile = q + kV0Queues * ti;
                        const int nx = (tile % tilesX) * 8 + (j & 7);
                        const int ny = (tile / tilesX) * kTileRows + (j >> 3);
                        if (nx < a.xc && ny < a.rows) {
                            lx = nx;
                            ly = ny;
                            f0 = a.frame0;
                            const float4 prev = a.out[(size_t)ly * a.xc + lx];
                            acc = f3(prev.x, prev.y, prev.z);
                            need = false;
                        }
                    }
                }
                cursor += n;
                if (cursor - base >= kTilePix) {   // the stream moves on to nxt; fetch its successor
                    if (!nxtKnown) {
                        nxt = (int)__builtin_amdgcn_readlane((int)fetched, 0) + 2 * bq;
                        nxtKnown = true;
                    }
                    base += kTilePix;
                    cur = nxt;
                    poolDone = cur >= nq;
                    if (!poolDone) {
                        if (lane == 0) fetched = atomicAdd(ctr, 1ull);
                        nxtKnown = false;
                    }
                }
            }
            sec_enter(sc, kSecOther, false);
            if (ready && state == kV3Ended) {   // the group's next round: TraceRowJob's per-pixel body
                const int f = f0 + sub;
                if (f < fend) {
                    sec_count(sc, kSecCamera);
                    const int px = a.x0 + lx;
                    const int py = a.y0 + (ly / a.rb) * a.rb * a.rp + a.rph * a.rb + ly % a.rb;
                    rng = PixelSeed((uint32_t)px, (uint32_t)py, (uint32_t)f);
                    const float u = ((float)px + RandomFloat01(rng)) * invWidth;          // :272
                    const float v = ((float)py + RandomFloat01(rng)) * invHeight;         // :273
                    r = GetRay(a.cam, u, v, rng, sc.rnlut);
                    depth = 0;
                    prevLambert = false;
                    pend = false;
                    state = kV3Trace;
                }   // else: no frame for this lane this round; it waits (Ended, no leaf)
            }
        }
        if (__ballot(state == kV3Trace) == 0) {
            if (__ballot(state == kV3Ended) == 0) break;   // every lane dead: done
            continue;
        }

        // ---- closest hit of every lane's ray (HitWorld, parallel.cpp:204) -----------
        sec_enter(sc, kSecOther, false);
        if (state == kV3Trace) {
            sec_count(sc, kSecHit);
            ++rays;
            int nid;
            float nt;
            if constexpr (kBvh) {
                nid = ClosestHitBVH(r.orig, r.dir, sc.bv, nt, sc.bstk, sc.bstride);
            } else {
                int sid;
                DualClosestHit(r.orig, r.dir, pend && dl.on, dl.l, sc, nid, nt, sid);
                if (pend && dl.on && sid == dl.li) {   // the light is reached (:123-132)
                    float* slot = reinterpret_cast<float*>(
                        (MAXD <= kTraceLdsLevels || depth < kTraceLdsLevels) ? lstk + depth * 64
                                                                             : gstk + (size_t)(depth - kTraceLdsLevels) * gthreads);
                    slot[0] = carry.x;
                    slot[1] = carry.y;
                    slot[2] = carry.z;
                }
            }
            if (pend) {   // the scatter event that produced r is on the stack (:214)
                ++depth;
                pend = false;
            }
            if (nid >= 0) {   // HitWorld's winner: pos (maths.cpp:74,86); the normal follows below
                r.orig = point_at(r, nt);
                id = nid;
            } else {          // sky (parallel.cpp:223-225)
                const float t = 0.5f * (r.dir.y + 1.0f);
                carry = ((1.0f - t) * f3(1.0f, 1.0f, 1.0f) + t * f3(0.5f, 0.7f, 1.0f)) * 0.3f;
                haveLeaf = true;
                state = kV3Ended;
            }
        }

        // ---- shading: Scatter (parallel.cpp:78-196) of every lane that hit ----------
        if (state == kV3Trace) {
            const float4 s = sc.sph[id];
            const F3 nrm = normalize(r.orig - f3(s.x, s.y, s.z));   // maths.cpp:75,87
            const Material mat = load_material(sc.mats, id);
            F3 matE = mat.emissive;
            bool cont = false;
            if (depth < a.maxDepth) {   // :212
                Hit rec;
                rec.pos = r.orig;
                rec.normal = nrm;
                rec.t = 0.0f;
                F3 lightE;
                dl.on = false;
                const F3 X = ScatterDir<kBvh>(mat, id, r, rec, lightE, rays, rng, sc, kBvh ? nullptr : &dl);
                sec_count(sc, kSecPost);
                const F3 dir = renormalize(normalize(X), sc.rnlut);
                if (mat.type != 1 || dot(dir, nrm) > 0.0f) {   // Metal absorbs (:147)
                    if (a.ndl && prevLambert) matE = f3(0.0f, 0.0f, 0.0f);
                    prevLambert = mat.type == 0;
                    // push matE + lightE (:214) for an unlit deferred light; carry the sum
                    // with the light's contribution, stored if the shadow ray reaches it
                    const F3 e = matE + lightE;
                    put(depth, make_float4(e.x, e.y, e.z, __int_as_float(id)));
                    if (dl.on) carry = matE + (lightE + dl.contrib);
                    pend = true;
                    r.dir = dir;   // r.orig is rec.pos already
                    cont = true;
                }
            }
            if (!cont) {
                carry = matE;
                haveLeaf = true;
                state = kV3Ended;
            }
        }
    }
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
    // one ray-count atomic per block (same-address atomics serialise in one L2 channel)
    const unsigned long long total = wave_sum((unsigned long long)rays);
    if (lane == 0) block_epilogue(a.tiles, a.rays, q, bq, total);
}

}  // namespace lrt
