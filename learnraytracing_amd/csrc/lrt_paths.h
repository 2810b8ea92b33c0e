// v1 megakernel: persistent waves with path regeneration.
//
// The reference traces one pixel per loop iteration of TraceRowJob (parallel.cpp:265-292)
// and recurses inside Trace (parallel.cpp:200-227). On a 64-wide wave, one pixel per
// lane for the whole path wastes most lanes: paths take 1 to 17+ rays
// and the wave runs until its slowest lane is done. Here every lane is a small state
// machine and EVERY loop iteration performs exactly one ray query (HitWorld) per live
// lane -- camera ray, bounce ray or one shadow ray of the Lambert light loop
// (parallel.cpp:93-133) -- followed by the state update for that ray:
//
//   kNeed   : the lane has no ray in flight: it starts the next sample of its pixel, or
//             stores the finished pixel and takes a new one from the wave's work queue
//   kBounce : a camera/bounce ray is in flight (Trace's HitWorld, parallel.cpp:205)
//   kShadow : shadow ray k of the light loop is in flight (parallel.cpp:123)
//   kDead   : the queue is empty
//
// RNG draws happen in exactly the reference order (jitter u, v; lens disk; then per
// bounce: Lambert unit vector, then eps1/eps2 per light, each light's draws after the
// previous light's shadow ray; Metal unit sphere; Dielectric one draw), rays are counted
// exactly where the reference counts them, and the recursion's result
// matE + lightE + att * Trace(...) is folded from the leaf outwards over a per-lane
// stack (LDS for the first kLdsLevels levels, a global overflow array beyond), so the
// output is bit-identical to the reference for any work distribution.
//
// Pixels are handed out in chunks of 64 (one atomicAdd per chunk per wave) in a
// banded 8x8-tile order, so the lanes of a wave trace neighbouring pixels.
#pragma once
#include "lrt_trace.h"

namespace lrt {

constexpr int kPathBlock = 256;
constexpr int kChunk = 64;
enum : int { kNeed = 0, kBounce = 1, kShadow = 2, kDead = 3 };

struct PathArgs {
    CameraDev cam;
    const float4* sph;
    const float4* mats;
    const int* lights;
    int count, nlights;
    int width, height;
    int x0, xc, y0, rows;
    int rb, rp, rph;
    int frame0, frames, maxDepth;
    int nitems;                 // xc * rows
    float4* out;
    unsigned long long* rays;
    unsigned int* queue;        // zeroed before every launch
    float4* overflow;           // stack levels >= kLdsLevels: [level - kLdsLevels][global thread]
    unsigned long long* stamps; // diagnostic builds only (-DLRT_EXP_STAMPS): per-section cycles
    BvhView bv;                 // bv.on: closest hit by BVH traversal (v2)
    int bvh_stack_offset;       // byte offset of the BVH traversal stacks in dynamic LDS
};

// Closest hit over all spheres: HitWorld's loop (parallel.cpp:54-73) with HitSphere's
// test (maths.cpp:51-94); returns the id (or -1) and t. Ties keep the lowest index.
LRT_DEV int ClosestHit(const F3& o, const F3& d, const float4* sph, int count, float& tOut) {
    float closestT = kMaxT;
    int id = -1;
    float4 next = sph[0];
    for (int i = 0; i < count; ++i) {
        const float4 s = next;
        if (i + 1 < count) next = sph[i + 1];   // issue the next sphere's read before this test
        const F3 rs = f3(s.x, s.y, s.z) - o;
        const float rsProj = dot(rs, d);
        const float ifHit = dot(rs, rs) - rsProj * rsProj - s.w;
        if (ifHit < 0.0f) {
            const float halfCut = __builtin_sqrtf(-ifHit);
            float t = rsProj - halfCut;
            if (t > kMinT && t < closestT) {
                closestT = t;
                id = i;
            } else {
                t = rsProj + halfCut;
                if (t > kMinT && t < closestT) {
                    closestT = t;
                    id = i;
                }
            }
        }
    }
    tOut = closestT;
    return id;
}

// Dense pixel order for the work queue: bands of 8 rows, 8-column groups inside a
// band, column-fastest inside a group (partial bands/groups at the edges, no holes).
__device__ __forceinline__ void ItemToPixel(int q, int xc, int rows, int& lx, int& ly) {
    const int band = q / (8 * xc);
    const int bh = min(8, rows - band * 8);
    const int r = q - band * 8 * xc;
    const int g = r / (8 * bh);
    const int gw = min(8, xc - g * 8);
    const int w = r - g * 8 * bh;
    lx = g * 8 + w % gw;
    ly = band * 8 + w / gw;
}

template <int kLdsLevels>
struct PathStack {
    float4* lds;            // [kLdsLevels][kPathBlock]
    float4* overflow;       // [level - kLdsLevels][gthreads]
    int tid;
    size_t gtid, gthreads;
    __device__ __forceinline__ void put(int level, float4 v) const {
        if (level < kLdsLevels)
            lds[level * kPathBlock + tid] = v;
        else
            overflow[(size_t)(level - kLdsLevels) * gthreads + gtid] = v;
    }
    __device__ __forceinline__ float4 get(int level) const {
        if (level < kLdsLevels) return lds[level * kPathBlock + tid];
        return overflow[(size_t)(level - kLdsLevels) * gthreads + gtid];
    }
};

// LDS carve-up of paths_kernel: [stack kLdsLevels x 256][spheres N][materials 3N][lights]
// (kLdsScene; otherwise only the stack is in LDS and the scene is read from global).
constexpr int kPowTableBytes = 16 * 8 + 16 * 8 + 32 * 8;   // powf tables (lrt_libm.h), staged by v2

__host__ __device__ inline size_t paths_lds_bytes(int lds_levels, bool lds_scene, int count, int nlights,
                                                   int pix = 0, bool bvh = false) {
    size_t b = sizeof(float4) * (size_t)lds_levels * kPathBlock + kPowTableBytes;
    if (lds_scene) b += sizeof(float4) * (4 * (size_t)count + (size_t)(nlights + 3) / 4 + 1);
    b += sizeof(float4) * (size_t)pix * kPathBlock;   // static-mode pixel slots (v2)
    if (bvh) b += sizeof(unsigned short) * (size_t)kBvhStackLevels * kPathBlock;   // last
    return b;
}

template <int kLdsLevels, bool kLdsScene>
__global__ __launch_bounds__(kPathBlock) void paths_kernel(const PathArgs a) {
    extern __shared__ float4 smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    PathStack<kLdsLevels> stk;
    stk.lds = smem;
    stk.overflow = a.overflow;
    stk.tid = tid;
    stk.gtid = (size_t)blockIdx.x * kPathBlock + tid;
    stk.gthreads = (size_t)gridDim.x * kPathBlock;
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
        __syncthreads();
        sph = s_sph;
        mats = s_mat;
        lights = s_lights;
    }
    const float invWidth = 1.0f / (float)a.width;     // parallel.cpp:260
    const float invHeight = 1.0f / (float)a.height;   // parallel.cpp:261
    const int fend = a.frame0 + a.frames;

    int qcur = 0, qend = 0;          // wave-uniform chunk cursor
    int q = -1, f = 0, x = 0, y = 0, kind = kNeed, depth = 0, rays = 0;
    int self = 0, k = 0, lid = 0;
    uint32_t rng = 0;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    F3 o = f3(0.f, 0.f, 0.f), d = o, sd = o, nl = o, lightE = o;
    float w = 0.0f;

    // The light loop of Scatter (parallel.cpp:93-133) one shadow ray at a time: find the
    // next emissive sphere other than the surface itself, draw eps1/eps2, aim the shadow
    // ray; when no light is left, push (matE + lightE, self) and continue the path along
    // the scattered direction.
    auto next_light = [&]() {
        while (k < a.nlights && lights[k] == self) ++k;
        if (k < a.nlights) {
            lid = lights[k];
            const float4 s = sph[lid];
            const F3 c = f3(s.x, s.y, s.z);
            const F3 sw = normalize(c - o);
            const F3 su = normalize(cross(__builtin_fabsf(sw.x) > 0.01f ? f3(0.0f, 1.0f, 0.0f) : f3(1.0f, 0.0f, 0.0f), sw));
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
            kind = kShadow;
            ++rays;                                                              // :122
        } else {
            const float4 e = mats[3 * self + 1];
            const F3 E = f3(e.x, e.y, e.z) + lightE;                             // matE + lightE (:214)
            stk.put(depth, make_float4(E.x, E.y, E.z, __int_as_float(self)));
            d = sd;
            ++depth;
            kind = kBounce;
            ++rays;                                                              // :204
        }
    };

    int pix = 0;   // local pixel offset ly * xc + lx
    for (;;) {
        // ---- (A) pixel hand-over (every lane reaches this point) ----------------------
        if (kind == kNeed && q >= 0 && f >= fend) {
            a.out[pix] = acc;      // one 16-byte store per finished pixel, alpha preserved
            q = -1;
        }
        const bool needPix = (kind == kNeed) && (q < 0);
        unsigned long long m = __ballot(needPix);
        while (m) {
            if (qcur >= qend) {                 // wave-uniform: grab the next chunk
                int base = 0;
                if (lane == 0) base = (int)atomicAdd(a.queue, (unsigned)kChunk);
                base = __shfl(base, 0, 64);
                if (base >= a.nitems) {
                    qcur = qend = a.nitems;
                    break;
                }
                qcur = base;
                qend = min(base + kChunk, a.nitems);
            }
            const int avail = qend - qcur;
            const int rank = __popcll(m & ((1ull << lane) - 1ull));
            if (((m >> lane) & 1ull) && rank < avail) q = qcur + rank;
            qcur += min(__popcll(m), avail);
            m = __ballot(needPix && q < 0);
        }
        if (needPix) {
            if (q < 0) {
                kind = kDead;
            } else {
                int lx, ly;
                ItemToPixel(q, a.xc, a.rows, lx, ly);
                x = a.x0 + lx;
                y = a.y0 + (ly / a.rb) * a.rb * a.rp + a.rph * a.rb + ly % a.rb;
                pix = ly * a.xc + lx;
                acc = a.out[pix];
                f = a.frame0;
            }
        }
        if (__ballot(kind != kDead) == 0ull) break;

        // ---- (B) camera ray of sample f (TraceRowJob body, parallel.cpp:270-276) ------
        if (kind == kNeed) {
            rng = PixelSeed((uint32_t)x, (uint32_t)y, (uint32_t)f);
            const float u = ((float)x + RandomFloat01(rng)) * invWidth;          // :272
            const float v = ((float)y + RandomFloat01(rng)) * invHeight;         // :273
            const Ray r = GetRay(a.cam, u, v, rng);
            o = r.orig;
            d = r.dir;
            depth = 0;
            kind = kBounce;
            ++rays;                                                              // :204
        }

        // ---- (C) the one ray query of this iteration -----------------------------------
        float t = kMaxT;
        int id = -1;
        if (kind != kDead) id = ClosestHit(o, d, sph, a.count, t);

        // ---- (D) state update -------------------------------------------------------
        bool wantLight = false;
        if (kind == kShadow) {
            if (id == lid) {                                                     // :123
                const float4 e = mats[3 * lid + 1];
                const float4 alb = mats[3 * self + 0];
                lightE = lightE + (f3(alb.x, alb.y, alb.z) * f3(e.x, e.y, e.z)) * w;   // :131
            }
            ++k;
            wantLight = true;
        } else if (kind == kBounce) {
            bool finish = false;
            F3 leaf;
            if (id < 0) {                                                        // sky, :221-226
                const float tt = 0.5f * (d.y + 1.0f);
                leaf = ((1.0f - tt) * f3(1.0f, 1.0f, 1.0f) + tt * f3(0.5f, 0.7f, 1.0f)) * 0.3f;
                finish = true;
            } else {
                const F3 pos = o + d * t;                                        // Ray::pointAt
                const float4 s = sph[id];
                const F3 normal = normalize(pos - f3(s.x, s.y, s.z));            // maths.cpp:74
                const Material mat = load_material(mats, id);
                if (depth < a.maxDepth) {                                        // :212
                    if (mat.type == 0) {                                         // Lambert :81-92
                        const F3 target = pos + normal + RandomUnitVector(rng);
                        sd = normalize(normalize(target - pos));
                        nl = dot(normal, d) < 0.0f ? normal : -normal;           // :129
                        lightE = f3(0.0f, 0.0f, 0.0f);
                        self = id;
                        o = pos;
                        k = 0;
                        wantLight = true;
                    } else if (mat.type == 1) {                                  // Metal :137-148
                        const F3 refl = reflect(d, normal);
                        const F3 nd = normalize(normalize(refl + mat.roughness * RandomInUnitSphere(rng)));
                        if (dot(nd, normal) > 0.0f) {
                            const F3 E = mat.emissive + f3(0.0f, 0.0f, 0.0f);
                            stk.put(depth, make_float4(E.x, E.y, E.z, __int_as_float(id)));
                            o = pos;
                            d = nd;
                            ++depth;
                            ++rays;
                        } else {
                            leaf = mat.emissive;
                            finish = true;
                        }
                    } else {                                                     // Dielectric :149-193
                        F3 outwardN;
                        const F3 rdir = d;
                        const F3 refl = reflect(rdir, normal);
                        float nint, cosine, reflProb;
                        F3 refr = f3(0.0f, 0.0f, 0.0f);
                        if (dot(rdir, normal) > 0.0f) {
                            outwardN = -normal;
                            nint = mat.ri;
                            cosine = dot(rdir, normal);
                        } else {
                            outwardN = normal;
                            nint = 1.0f / mat.ri;
                            cosine = -dot(rdir, normal);
                        }
                        if (refract(rdir, outwardN, nint, refr))
                            reflProb = schlick(cosine, mat.ri);
                        else
                            reflProb = 1.0f;
                        const F3 nd = RandomFloat01(rng) < reflProb ? normalize(normalize(refl))
                                                                    : normalize(normalize(refr));
                        const F3 E = mat.emissive + f3(0.0f, 0.0f, 0.0f);
                        stk.put(depth, make_float4(E.x, E.y, E.z, __int_as_float(id)));
                        o = pos;
                        d = nd;
                        ++depth;
                        ++rays;
                    }
                } else {
                    leaf = mat.emissive;                                         // :218
                    finish = true;
                }
            }
            if (finish) {
                // fold matE + lightE + att * T from the leaf outwards (parallel.cpp:214)
                F3 T = leaf;
                for (int l = depth - 1; l >= 0; --l) {
                    const float4 e = stk.get(l);
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
                kind = kNeed;
            }
        }
        if (wantLight) next_light();   // the one call site: shadow follow-up or new Lambert hit
    }
    unsigned long long total = (unsigned long long)rays;
    for (int off = 32; off > 0; off >>= 1) total += __shfl_xor(total, off, 64);
    if (lane == 0 && total) atomicAdd(a.rays, total);
}

}  // namespace lrt
