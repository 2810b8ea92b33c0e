// v2 megakernel: persistent waves, path regeneration, PHASE-SCHEDULED sections.
//
// Measured on v0/v1 (profiles/r1_v0, tools/gpu_counters.sh): with one pixel per lane
// (v0) or a per-lane state machine that runs every shading section each iteration (v1),
// only ~30 % of the lanes are active per VALU instruction (SQ_THREAD_CYCLES_VALU /
// (SQ_ACTIVE_INST_VALU * 64)): camera generation, Lambert setup, light sampling,
// metal/dielectric scattering and path finishing each run for the few lanes that need
// them. Here each lane is still a state machine, but in every iteration the wave
// counts (ballot) how many lanes wait in each phase and runs ONLY the phase with the
// most lanes:
//
//   TRACE   one ray query (HitWorld) for every lane holding a ray; classifies the hit
//   LIGHT   Lambert scatter (parallel.cpp:81-92) or the shadow-ray result
//           (parallel.cpp:123-132), then the next light's shadow ray or, when no light
//           is left, the push of matE + lightE and the bounce ray
//   SPEC    Metal (parallel.cpp:137-148) and Dielectric (parallel.cpp:149-193)
//   CAMERA  path finish (fold of the recursion, progressive lerp), pixel hand-over
//           from the work queue, and the next sample's camera ray (parallel.cpp:270-286)
//
// The arithmetic, RNG order and ray counting are those of lrt_paths.h/lrt_trace.h (the
// reference's), so results are bit-identical whatever the schedule.
#pragma once
#include "lrt_paths.h"

namespace lrt {

enum : int { sPix = 0, sCam, sTrace, sLam, sMet, sDie, sShadow, sLight, sFin, sDead };
enum : int { kSecTrace = 0, kSecLight, kSecSpec, kSecCam, kSecCount };

// Share of the work chunks dealt statically (round-robin over the persistent waves);
// the rest is handed out by the atomic queue to balance the tail. A contended
// returning atomic takes microseconds and, because vmcnt retires in order, every later
// VMEM wait of the wave waits for it too -- so the queue is only used at the end.
constexpr int kStaticPercent = 85;

// kPix > 0 (static mode): each lane owns kPix pixels for the whole launch (a block covers
// 16 columns x 16*kPix rows; lane pixel j is 16*j rows below pixel 0). All prev values
// are read into LDS before the loop and all results written back after it, so the loop
// issues no global memory operation at all. kPix == 0: persistent waves fed by the work
// queue (static chunks, then atomics).
#ifndef LRT_WAVES_PER_EU
#define LRT_WAVES_PER_EU 1
#endif
template <int kLdsLevels, bool kLdsScene, bool kOverflow, int kPix, bool kBvh>
__global__ __launch_bounds__(kPathBlock, LRT_WAVES_PER_EU) void paths2_kernel(const PathArgs a) {
    constexpr bool kStaticPixel = kPix > 0;
    extern __shared__ float4 smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    PathStack<kLdsLevels> stk;
    stk.lds = smem;
    stk.overflow = a.overflow;
    stk.tid = tid;
    // linear block id: the static-pixel mode launches a 2-D grid
    stk.gtid = ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * kPathBlock + tid;
    stk.gthreads = (size_t)gridDim.x * gridDim.y * kPathBlock;
    // powf tables (Dielectric's schlick) live in LDS
    double* s_pow = reinterpret_cast<double*>(smem + kLdsLevels * kPathBlock);
    {
        const libm::PowTables g = libm::pow_tables();
        if (tid < 16) {
            s_pow[tid] = g.invc[tid];
            s_pow[16 + tid] = g.logc[tid];
        }
        if (tid < 32) reinterpret_cast<uint64_t*>(s_pow + 32)[tid] = g.exp2[tid];
    }
    libm::PowTables powT;
    powT.invc = s_pow;
    powT.logc = s_pow + 16;
    powT.exp2 = reinterpret_cast<const uint64_t*>(s_pow + 32);
    const float4* sph = a.sph;
    const float4* mats = a.mats;
    const int* lights = a.lights;
    if (kLdsScene) {
        float4* s_sph = smem + kLdsLevels * kPathBlock + kPowTableBytes / 16;
        float4* s_mat = s_sph + a.count;
        int* s_lights = reinterpret_cast<int*>(s_mat + 3 * a.count);
        for (int i = tid; i < a.count; i += kPathBlock) s_sph[i] = a.sph[i];
        for (int i = tid; i < 3 * a.count; i += kPathBlock) s_mat[i] = a.mats[i];
        for (int i = tid; i < a.nlights; i += kPathBlock) s_lights[i] = a.lights[i];
        sph = s_sph;
        mats = s_mat;
        lights = s_lights;
    }
    __syncthreads();
    const float invWidth = 1.0f / (float)a.width;     // parallel.cpp:260
    const float invHeight = 1.0f / (float)a.height;   // parallel.cpp:261
    const int fend = a.frame0 + a.frames;
    unsigned short* bstk = reinterpret_cast<unsigned short*>(reinterpret_cast<char*>(smem) + a.bvh_stack_offset) + tid;

    auto push = [&](int level, F3 E, int id) {
        const float4 v = make_float4(E.x, E.y, E.z, __int_as_float(id));
        if (!kOverflow || level < kLdsLevels)
            stk.lds[level * kPathBlock + tid] = v;
        else
            stk.overflow[(size_t)(level - kLdsLevels) * stk.gthreads + stk.gtid] = v;
    };
    auto get = [&](int level) -> float4 {
        if (!kOverflow || level < kLdsLevels) return stk.lds[level * kPathBlock + tid];
        return stk.overflow[(size_t)(level - kLdsLevels) * stk.gthreads + stk.gtid];
    };

    // work chunks of kChunk pixels: wave wv takes chunks wv, wv + nw, ... for nStatic
    // rounds, then chunks from the queue
    const int nw = gridDim.x * (kPathBlock / 64);
    const int wv = blockIdx.x * (kPathBlock / 64) + (tid >> 6);
    const int nchunks = (a.nitems + kChunk - 1) / kChunk;
    const int nStatic = (int)(((long long)nchunks * kStaticPercent / 100) / nw);
    int round = 0;
    int qcur = 0, qend = 0;   // wave-uniform cursor in the current chunk
    int state = sPix, pix = 0, f = 0, x = 0, y = 0, depth = 0, rays = 0;
    int self = 0, k = 0, lid = 0, id = -1;
    bool shadowRay = false;
    uint32_t rng = 0;
    float t = 0.0f, w = 0.0f;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    F3 o = f3(0.f, 0.f, 0.f), d = o, sd = o, nl = o, lightE = o, leaf = o;
    // static mode: LDS slots [kPix][kPathBlock] for the lane's pixels
    float4* s_pix = smem + kLdsLevels * kPathBlock + kPowTableBytes / 16 +
                    (kLdsScene ? 4 * a.count + (a.nlights + 3) / 4 + 1 : 0);
    const int slx = blockIdx.x * 16 + ((tid >> 6) & 1) * 8 + (lane & 7);
    const int sly0 = blockIdx.y * 16 * (kPix > 0 ? kPix : 1) + ((tid >> 6) >> 1) * 8 + (lane >> 3);
    int pj = 0;   // index of the lane's current pixel
    auto set_pixel = [&](int j) -> bool {   // static mode: make pixel j current
        const int ly = sly0 + 16 * j;
        if (slx >= a.xc || ly >= a.rows) return false;
        x = a.x0 + slx;
        y = a.y0 + (ly / a.rb) * a.rb * a.rp + a.rph * a.rb + ly % a.rb;
        pix = ly * a.xc + slx;
        acc = s_pix[j * kPathBlock + tid];
        f = a.frame0;
        return true;
    };
    if (kStaticPixel) {
#pragma unroll
        for (int j = 0; j < (kPix > 0 ? kPix : 1); ++j) {
            const int ly = sly0 + 16 * j;
            if (slx < a.xc && ly < a.rows) s_pix[j * kPathBlock + tid] = a.out[ly * a.xc + slx];
        }
        state = set_pixel(0) ? sCam : sDead;
    }

#ifdef LRT_EXP_STAMPS
    // diagnostic build: [sec][cycles, executions, lanes] + schedule overhead, per wave
    unsigned long long stc[kSecCount + 1] = {}, stn[kSecCount + 1] = {}, stl[kSecCount + 1] = {};
#endif
    for (;;) {
#ifdef LRT_EXP_STAMPS
        const unsigned long long ts0 = __builtin_amdgcn_s_memtime();
#endif
        // ---- schedule: the phase with the most lanes -----------------------------------
        const int nTrace = __popcll(__ballot(state == sTrace));
        const int nLight = __popcll(__ballot(state == sLam || state == sShadow || state == sLight));
        const int nSpec = __popcll(__ballot(state == sMet || state == sDie));
        const int nCam = __popcll(__ballot(state == sFin || state == sCam || state == sPix));
        if (nTrace + nLight + nSpec + nCam == 0) break;   // every lane dead
        int sec = kSecTrace, best = nTrace;
        if (nLight > best) { sec = kSecLight; best = nLight; }
        if (nCam > best) { sec = kSecCam; best = nCam; }
        if (nSpec > best) { sec = kSecSpec; best = nSpec; }
#ifdef LRT_EXP_STAMPS
        const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
        stc[kSecCount] += ts1 - ts0;
        stn[kSecCount] += 1;
#endif

        if (sec == kSecTrace) {
            // ---- TRACE: the ray query, then classification -----------------------------
            if (state == sTrace) {
                id = kBvh ? ClosestHitBVH(o, d, a.bv, t, bstk, kPathBlock) : ClosestHit(o, d, sph, a.count, t);
                if (shadowRay) {
                    state = sShadow;
                } else if (id < 0) {                                             // sky :221-226
                    const float tt = 0.5f * (d.y + 1.0f);
                    leaf = ((1.0f - tt) * f3(1.0f, 1.0f, 1.0f) + tt * f3(0.5f, 0.7f, 1.0f)) * 0.3f;
                    state = sFin;
                } else if (depth >= a.maxDepth) {                                // :212, :218
                    const float4 e = mats[3 * id + 1];
                    leaf = f3(e.x, e.y, e.z);
                    state = sFin;
                } else {
                    const int type = __float_as_int(mats[3 * id + 0].w);
                    state = type == 0 ? sLam : type == 1 ? sMet : sDie;
                }
            }
        } else if (sec == kSecLight) {
            // ---- LIGHT: Lambert scatter (:87-92) / shadow result (:123-132), then the
            //      next light's shadow ray or, when none is left, the bounce ray ----------
            if (state == sLam) {
                const F3 pos = o + d * t;
                const float4 s = sph[id];
                const F3 normal = normalize(pos - f3(s.x, s.y, s.z));
                const F3 target = pos + normal + RandomUnitVector(rng);
                sd = normalize(normalize(target - pos));
                nl = dot(normal, d) < 0.0f ? normal : -normal;                   // :129
                lightE = f3(0.0f, 0.0f, 0.0f);
                self = id;
                o = pos;
                k = 0;
                state = sLight;
            } else if (state == sShadow) {
                if (id == lid) {                                                 // :123
                    const float4 e = mats[3 * lid + 1];
                    const float4 alb = mats[3 * self + 0];
                    lightE = lightE + (f3(alb.x, alb.y, alb.z) * f3(e.x, e.y, e.z)) * w;   // :131
                }
                ++k;
                state = sLight;
            }
            if (state == sLight) {
                while (k < a.nlights && lights[k] == self) ++k;                 // :96-99
                if (k < a.nlights) {
                    lid = lights[k];
                    const float4 s = sph[lid];
                    const F3 c = f3(s.x, s.y, s.z);
                    const F3 sw = normalize(c - o);
                    const F3 su = normalize(cross(__builtin_fabsf(sw.x) > 0.01f ? f3(0.0f, 1.0f, 0.0f)
                                                                                : f3(1.0f, 0.0f, 0.0f), sw));
                    const F3 sv = cross(sw, su);
                    const float len = length(o - c);
                    const float cosAMax = __builtin_sqrtf(1.0f - s.w / (len * len));      // :109
                    const float eps1 = RandomFloat01(rng);
                    const float eps2 = RandomFloat01(rng);
                    const float cosA = 1.0f - eps1 + eps1 * cosAMax;
                    const float sinA = __builtin_sqrtf(1.0f - cosA * cosA);
                    const float phi = 2.0f * kPI * eps2;
                    float sphi, cphi;
                    libm::sincosf(phi, &sphi, &cphi);
                    F3 l = su * cphi * sinA + sv * sphi * sinA + sw * cosA;             // :116
                    l = normalize_member(l);                                             // :117
                    d = normalize(l);                                                    // Ray(rec.pos, l)
                    const float omega = 2.0f * kPI * (1.0f - cosAMax);                   // :126
                    const float dd = dot(l, nl);
                    w = ((0.0f < dd) ? dd : 0.0f) * omega / kPI;                         // :131
                    shadowRay = true;
                    ++rays;                                                              // :122
                } else {
                    const float4 e = mats[3 * self + 1];
                    push(depth, f3(e.x, e.y, e.z) + lightE, self);                       // :214
                    d = sd;
                    ++depth;
                    shadowRay = false;
                    ++rays;                                                              // :204
                }
                state = sTrace;
            }
        } else if (sec == kSecSpec) {
            // ---- SPEC: Metal (:137-148) and Dielectric (:149-193) -----------------------
            if (state == sMet || state == sDie) {
                const F3 pos = o + d * t;
                const float4 s = sph[id];
                const F3 normal = normalize(pos - f3(s.x, s.y, s.z));
                const float4 me = mats[3 * id + 1];
                const F3 matE = f3(me.x, me.y, me.z);
                F3 nd;
                bool keep = true;
                if (state == sMet) {
                    const F3 refl = reflect(d, normal);
                    nd = normalize(normalize(refl + me.w * RandomInUnitSphere(rng)));
                    keep = dot(nd, normal) > 0.0f;
                } else {
                    const float ri = mats[3 * id + 2].w;
                    F3 outwardN;
                    const F3 rdir = d;
                    const F3 refl = reflect(rdir, normal);
                    float nint, cosine, reflProb;
                    F3 refr = f3(0.0f, 0.0f, 0.0f);
                    if (dot(rdir, normal) > 0.0f) {
                        outwardN = -normal;
                        nint = ri;
                        cosine = dot(rdir, normal);
                    } else {
                        outwardN = normal;
                        nint = 1.0f / ri;
                        cosine = -dot(rdir, normal);
                    }
                    if (refract(rdir, outwardN, nint, refr))
                        reflProb = schlick(cosine, ri, powT);
                    else
                        reflProb = 1.0f;
                    nd = RandomFloat01(rng) < reflProb ? normalize(normalize(refl)) : normalize(normalize(refr));
                }
                if (keep) {
                    push(depth, matE + f3(0.0f, 0.0f, 0.0f), id);
                    o = pos;
                    d = nd;
                    ++depth;
                    ++rays;                                                      // :204
                    shadowRay = false;
                    state = sTrace;
                } else {
                    leaf = matE;                                                 // absorbed
                    state = sFin;
                }
            }
        } else {
            // ---- CAMERA: finish paths, hand over pixels, start samples ----------------
            if (state == sFin) {
                F3 T = leaf;                                       // fold, parallel.cpp:214
                for (int l = depth - 1; l >= 0; --l) {
                    const float4 e = get(l);
                    const float4 b = mats[3 * __float_as_int(e.w) + 2];
                    T = f3(e.x, e.y, e.z) + f3(b.x, b.y, b.z) * T;
                }
                const float lerpFac = (float)f / (float)(f + 1);                 // :262
                const F3 prev = f3(acc.x, acc.y, acc.z);
                const F3 col = prev * lerpFac + T * (1.0f - lerpFac);            // :282
                acc.x = col.x;
                acc.y = col.y;
                acc.z = col.z;
                ++f;
                if (f < fend) {
                    state = sCam;
                } else if (kStaticPixel) {
                    s_pix[pj * kPathBlock + tid] = acc;            // written back after the loop
                    ++pj;
                    state = (pj < kPix && set_pixel(pj)) ? sCam : sDead;
                } else {
                    a.out[pix] = acc;                              // alpha preserved
                    state = sPix;
                }
            }
            unsigned long long m = kStaticPixel ? 0ull : __ballot(state == sPix);
            while (m) {
                if (qcur >= qend) {                                // next chunk of this wave
                    int c;
                    if (round < nStatic) {
                        c = wv + round * nw;
                    } else {
                        int base = 0;
                        if (lane == 0) base = (int)atomicAdd(a.queue, 1u);
                        c = nStatic * nw + __shfl(base, 0, 64);
                    }
                    ++round;
                    if (c >= nchunks) {
                        qcur = qend = a.nitems;
                        break;
                    }
                    qcur = c * kChunk;
                    qend = min(qcur + kChunk, a.nitems);
                }
                const int avail = qend - qcur;
                const int rank = __popcll(m & ((1ull << lane) - 1ull));
                if (((m >> lane) & 1ull) && rank < avail) {
                    const int q = qcur + rank;
                    int lx, ly;
                    ItemToPixel(q, a.xc, a.rows, lx, ly);
                    x = a.x0 + lx;
                    y = a.y0 + (ly / a.rb) * a.rb * a.rp + a.rph * a.rb + ly % a.rb;
                    pix = ly * a.xc + lx;
                    acc = a.out[pix];
                    f = a.frame0;
                    state = sCam;
                }
                qcur += min(__popcll(m), avail);
                m = __ballot(state == sPix);
            }
            if (state == sPix) state = sDead;   // no work left
            if (state == sCam) {
                rng = PixelSeed((uint32_t)x, (uint32_t)y, (uint32_t)f);
                const float u = ((float)x + RandomFloat01(rng)) * invWidth;      // :272
                const float v = ((float)y + RandomFloat01(rng)) * invHeight;     // :273
                const Ray r = GetRay(a.cam, u, v, rng);
                o = r.orig;
                d = r.dir;
                depth = 0;
                shadowRay = false;
                ++rays;                                                          // :204
                state = sTrace;
            }
        }
#ifdef LRT_EXP_STAMPS
        {
            const unsigned long long ts2 = __builtin_amdgcn_s_memtime();
#pragma unroll
            for (int s2 = 0; s2 < kSecCount; ++s2)
                if (s2 == sec) {
                    stc[s2] += ts2 - ts1;
                    stn[s2] += 1;
                    stl[s2] += best;
                }
        }
#endif
    }
    if (kStaticPixel && a.frames > 0) {
#pragma unroll
        for (int j = 0; j < (kPix > 0 ? kPix : 1); ++j) {
            const int ly = sly0 + 16 * j;
            if (slx < a.xc && ly < a.rows) a.out[ly * a.xc + slx] = s_pix[j * kPathBlock + tid];
        }
    }
#ifdef LRT_EXP_STAMPS
    if (lane == 0 && a.stamps) {
#pragma unroll
        for (int s2 = 0; s2 <= kSecCount; ++s2) {
            atomicAdd(&a.stamps[3 * s2 + 0], stc[s2]);
            atomicAdd(&a.stamps[3 * s2 + 1], stn[s2]);
            atomicAdd(&a.stamps[3 * s2 + 2], stl[s2]);
        }
    }
#endif
    unsigned long long total = (unsigned long long)rays;
    for (int off = 32; off > 0; off >>= 1) total += __shfl_xor(total, off, 64);
    if (lane == 0 && total) atomicAdd(a.rays, total);
}

}  // namespace lrt
