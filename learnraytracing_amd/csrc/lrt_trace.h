// Device restatement of the reference hot path (src/cpu/maths.{h,cpp}, parallel.cpp),
// written for one work-item per pixel on gfx950.
//
// Parity rules are kept literally: left-to-right RNG draw order,
// XorShift32 13/17/15, rejection tests, double normalisation, member vs free
// normalize, the reference's association order in every expression, glibc-exact
// transcendentals (lrt_libm.h), IEEE sqrt/div, and the build uses
// -ffp-contract=off so no a*b+c is fused. The recursive Trace() is flattened into a
// loop that pushes (matE + lightE, material) per scatter event and then folds the
// stack from the leaf outwards, which evaluates exactly the reference's
// `matE + lightE + attenuation * Trace(...)` (parallel.cpp:214) in the same order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lrt_libm.h"

namespace lrt {

#define LRT_DEV __host__ __device__ __forceinline__

constexpr float kPI = 3.1415926f;     // maths.h:5
constexpr float kMinT = 0.001f;       // parallel.cpp:9
constexpr float kMaxT = 1.0e7f;       // parallel.cpp:10

struct float3_ { float x, y, z; };    // maths.h:10-61 (own type: no vendor operators)
using F3 = float3_;

LRT_DEV F3 f3(float x, float y, float z) { F3 r; r.x = x; r.y = y; r.z = z; return r; }
LRT_DEV F3 operator+(F3 a, F3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }   // maths.h:63
LRT_DEV F3 operator-(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }   // maths.h:67
LRT_DEV F3 operator*(F3 a, F3 b) { return f3(a.x * b.x, a.y * b.y, a.z * b.z); }   // maths.h:71
LRT_DEV F3 operator*(F3 a, float b) { return f3(a.x * b, a.y * b, a.z * b); }      // maths.h:75
LRT_DEV F3 operator*(float a, F3 b) { return f3(a * b.x, a * b.y, a * b.z); }      // maths.h:79
LRT_DEV F3 operator-(F3 a) { return f3(-a.x, -a.y, -a.z); }                        // maths.h:27
LRT_DEV float dot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }        // maths.h:83
LRT_DEV F3 cross(F3 a, F3 b) {                                                      // maths.h:87-92
    return f3(a.y * b.z - a.z * b.y, -(a.x * b.z - a.z * b.x), a.x * b.y - a.y * b.x);
}
// Correctly rounded sqrt and reciprocal (the IEEE results the reference's sqrtf and 1/x
// give) in fewer instructions than LLVM's generic expansions, which also handle operands
// the path almost never produces:
//  * sqrt: v_sqrt_f32 is faithful (within 1 ulp); one residual check of each neighbour,
//    fma(-s', s, x), picks the correctly rounded root. This is LLVM's own sequence minus
//    the denormal scaling and the 0/inf class fix-up, and equals __builtin_sqrtf for
//    every float >= 2^-104 (checked exhaustively on gfx950: tools/fpexact.hip).
//  * reciprocal: v_rcp_f32 plus two Newton steps in fma, equal to 1.0f / x for every
//    float with |x| in [2^-125, 2^125] (exhaustive, tools/fpexact.hip).
// Operands outside those ranges (or NaN) send the whole wave through the generic
// sequence: a wave-uniform branch, essentially never taken. Host builds (the BVH
// diagnostics) use the plain operations.
LRT_DEV float sqrt_rn(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __int_as_float(__float_as_int(s) - 1);
    const float su = __int_as_float(__float_as_int(s) + 1);
    const float rd = __builtin_fmaf(-sd, s, x);
    const float ru = __builtin_fmaf(-su, s, x);
    s = rd <= 0.0f ? sd : s;
    s = ru > 0.0f ? su : s;
    if (__builtin_expect(__ballot(!(x >= 0x1p-96f)) != 0, 0)) s = __builtin_sqrtf(x);
    return s;
#else
    return __builtin_sqrtf(x);
#endif
}
LRT_DEV float rcp_rn(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    float r = __builtin_amdgcn_rcpf(x);
    float e = __builtin_fmaf(-x, r, 1.0f);
    r = __builtin_fmaf(e, r, r);
    e = __builtin_fmaf(-x, r, 1.0f);
    r = __builtin_fmaf(e, r, r);
    const float ax = __builtin_fabsf(x);
    if (__builtin_expect(__ballot(!(ax >= 0x1p-125f && ax <= 0x1p125f)) != 0, 0)) r = 1.0f / x;
    return r;
#else
    return 1.0f / x;
#endif
}
LRT_DEV float length(F3 v) { return sqrt_rn(v.x * v.x + v.y * v.y + v.z * v.z); } // maths.h:15
LRT_DEV F3 normalize(F3 v) { float k = rcp_rn(length(v)); return f3(v.x * k, v.y * k, v.z * k); } // maths.h:93
// normalize() of a vector that is already unit length to a few ulps (the reference
// normalises twice: every Ray ctor normalises its direction again, maths.h:133-137).
// Its |y|^2 lies within kRenormR ulps of 1, so 1/sqrt(|y|^2) comes from a table of
// rcp_rn(sqrt_rn(d)) for those d, filled with the very same operations (renorm_lut_fill):
// same bits as normalize(y) with ~12 fewer instructions. Any other |y|^2 computes.
constexpr int kRenormR = 64;
constexpr int kRenormBytes = ((2 * kRenormR + 1) * 4 + 15) / 16 * 16;
LRT_DEV void renorm_lut_fill(float* lut, int tid, int block) {
    for (int j = tid; j <= 2 * kRenormR; j += block) {
        const float d = libm::u2f((uint32_t)(0x3f800000 + j - kRenormR));
        lut[j] = rcp_rn(sqrt_rn(d));
    }
}
constexpr int kPowTableBytes = 16 * 8 + 16 * 8 + 32 * 8;   // powf tables (lrt_libm.h) staged in LDS
LRT_DEV F3 normalize_member(F3 v) { float l = length(v); return f3(v.x / l, v.y / l, v.z / l); } // maths.h:19
LRT_DEV F3 reflect(F3 v, F3 n) { return v + 2.0f * (-dot(v, n) * n); }             // maths.h:100-103
LRT_DEV bool refract(F3 v, F3 n, float nint, F3& out) {                             // maths.h:106-118
    float dt = dot(v, n);
    float discr = 1.0f - nint * nint * (1.0f - dt * dt);
    if (discr > 0) {
        out = nint * (v - n * dt) - n * sqrt_rn(discr);
        return true;
    }
    return false;
}
LRT_DEV float schlick(float cosine, float ri, const libm::PowTables& T) {          // maths.h:122-127
    float r0 = (1.0f - ri) / (1.0f + ri);
    r0 = r0 * r0;
    return r0 + (1.0f - r0) * libm::powf5(1.0f - cosine, T);
}
LRT_DEV float schlick(float cosine, float ri) { return schlick(cosine, ri, libm::pow_tables()); }

struct Ray {                                                                        // maths.h:130-145
    F3 orig, dir;
};
LRT_DEV Ray make_ray(F3 o, F3 d) { Ray r; r.orig = o; r.dir = normalize(d); return r; }
LRT_DEV F3 renormalize(F3 y, const float* lut) {
    if (!lut) return normalize(y);
    const float d = y.x * y.x + y.y * y.y + y.z * y.z;   // length()'s sum, same order
    const int j = libm::f2u_i(d) - 0x3f800000 + kRenormR;
    float k;
    if ((unsigned)j <= 2u * kRenormR) k = lut[j];
    else k = rcp_rn(sqrt_rn(d));
    return f3(y.x * k, y.y * k, y.z * k);
}
LRT_DEV F3 point_at(const Ray& r, float t) { return r.orig + r.dir * t; }

struct Hit { F3 pos, normal; float t; };                                            // maths.h:148-153

// ---- RNG: maths.cpp:7-49 with the state in a register (one stream per pixel-sample)
LRT_DEV uint32_t XorShift32(uint32_t& s) {
    uint32_t x = s;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 15;
    s = x;
    return x;
}
LRT_DEV float RandomFloat01(uint32_t& s) { return (float)(XorShift32(s) & 0xFFFFFF) * (1.0f / 16777216.0f); }
LRT_DEV F3 RandomInUnitDisk(uint32_t& s) {
    F3 p;
    do {
        float a = RandomFloat01(s);
        float b = RandomFloat01(s);
        p = 2.0f * f3(a, b, 0.0f) - f3(1.0f, 1.0f, 0.0f);
    } while (dot(p, p) >= 1.0f);
    return p;
}
LRT_DEV F3 RandomUnitVector(uint32_t& s) {
    float z = RandomFloat01(s) * 2.0f - 1.0f;
    float a = RandomFloat01(s) * 2.0f * kPI;
    float r = sqrt_rn(1.0f - z * z);
    float sa, ca;
    libm::sincosf(a, &sa, &ca);   // bit-identical to separate cosf(a), sinf(a)
    float x = r * ca;
    float y = r * sa;
    return f3(x, y, z);
}
LRT_DEV F3 RandomInUnitSphere(uint32_t& s) {
    F3 p;
    do {
        float a = RandomFloat01(s);
        float b = RandomFloat01(s);
        float c = RandomFloat01(s);
        p = 2.0f * f3(a, b, c) - f3(1.0f, 1.0f, 1.0f);
        // the reference tests p.length() >= 1.0 (maths.cpp:47). With s = x*x + y*y + z*z
        // summed in the same order, the correctly rounded sqrt(s) >= 1 iff s >= 1:
        // sqrt(1 - 2^-24) = 1 - 2^-25 - 2^-51 rounds down to 1 - 2^-24, and sqrt is
        // monotonic, so the sqrt can go
    } while (p.x * p.x + p.y * p.y + p.z * p.z >= 1.0f);
    return p;
}

// ---- scene as the kernel sees it -------------------------------------------------
// Sphere: float4(center.xyz, radius*radius). The reference only ever uses the radius
// squared (maths.cpp:59, parallel.cpp:109), so r*r is folded once on the host.
// Material: three float4 rows: (albedo.xyz, type), (emissive.xyz, roughness),
// (attenuation.xyz, ri) where attenuation = albedo (Lambert, Metal) or 1 (Dielectric,
// parallel.cpp:90,144,192).
struct Material {
    F3 albedo;
    int type;
    int id;   // the table index: the reference's `&mat == &smat` self test (parallel.cpp:98)
    F3 emissive;
    float roughness;
    F3 att;
    float ri;
};
LRT_DEV Material load_material(const float4* __restrict__ mats, int id) {
    float4 a = mats[3 * id + 0];
    float4 e = mats[3 * id + 1];
    float4 b = mats[3 * id + 2];
    Material m;
    m.albedo = f3(a.x, a.y, a.z);
    m.type = libm::f2u_i(a.w);
    m.id = id;
    m.emissive = f3(e.x, e.y, e.z);
    m.roughness = e.w;
    m.att = f3(b.x, b.y, b.z);
    m.ri = b.w;
    return m;
}

}  // namespace lrt
#include "lrt_bvh.h"
#include "lrt_grid.h"
namespace lrt {

// The closest-hit structure a kernel instance is compiled for (template parameter kAcc): the
// reference's linear scan, the 4-wide BVH (lrt_bvh.h) or the uniform grid (lrt_grid.h). All
// three return the scan's bits.
enum : int { kAccScan = 0, kAccBvh = 1, kAccGrid = 2 };

struct SceneView {
    const float4* sph;                 // LDS or global
    const float4* __restrict__ mats;   // global (per-lane gather, L1/L2 resident)
    const int* __restrict__ lights;    // emissive sphere ids in index order
    int count;
    int nlights;
    BvhView bv;                        // the BVH (kAcc == kAccBvh)
    GridView gv;                       // the uniform grid (kAcc == kAccGrid)
    unsigned short* bstk;              // this lane's BVH traversal stack (LDS)
    int bstride;
    libm::PowTables pow;               // powf tables for Dielectric's schlick (LDS copy)
    const float* rnlut;                // renormalize() table (LDS), null: plain normalize
#ifdef LRT_EXP_SECSTATS
    unsigned long long* secstats;      // diagnostic: per section {wave executions, active lanes, cycles}
    unsigned long long* sectime;       // this wave's LDS bookkeeping
#endif
};

// Diagnostic builds only (LRT_EXP_SECSTATS): per section, how many times a wave enters
// it, how many lanes are active then, and the shader cycles spent in it until the next
// section switch (s_memtime, bookkept in LDS by the first active lane so divergence
// cannot desynchronise it). sec_count enters and counts; sec_enter only switches time.
enum { kSecHit, kSecLambert, kSecShadow, kSecMetal, kSecDiel, kSecPost, kSecFold, kSecCamera, kSecOther, kSecHit0,
       kSecShadow0, kSecN };   // *0: a path's first closest hit / first shadow rays (coherent)
LRT_DEV void sec_enter(const SceneView& sc, int sec, bool count) {
#if defined(LRT_EXP_SECSTATS) && defined(__HIP_DEVICE_COMPILE__)
    const unsigned long long m = __ballot(1);
    if ((int)__lane_id() == __ffsll((long long)m) - 1) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        // LDS, this wave: [0] section, [1] since, [2 + s] cycles, [2 + kSecN + s] entries,
        // [2 + 2 kSecN + s] active lanes -- no global atomics in the loop (they would sit
        // in vmcnt and be charged to whichever section waits next)
        unsigned long long* w = sc.sectime;
        const int cur = (int)w[0];
        w[2 + cur] += now - w[1];
        w[0] = (unsigned long long)sec;
        w[1] = now;
        if (count) {
            w[2 + kSecN + sec] += 1;
            w[2 + 2 * kSecN + sec] += (unsigned long long)__popcll(m);
        }
    }
#else
    (void)sc;
    (void)sec;
    (void)count;
#endif
}
LRT_DEV void sec_count(const SceneView& sc, int sec) { sec_enter(sc, sec, true); }

// HitSphere's root selection against the running closestT (maths.cpp:61-90): the first
// root if it lies in (tMin, closestT), else the second. (A branchless form -- sqrt for every
// lane, selects -- measured slower: the divergent branch around the sqrt is cheap when no
// lane takes it.)
// Inside, the reference's if / else-if is taken as selects over both roots, its && as bitwise
// ands: each short-circuit was a divergent region of its own, whose exec bookkeeping (scalar
// instructions, a branch) cost more than the second root's add (the grid walk: profiles/r4_y).
LRT_DEV void SphereRoots(float rsProj, float ifHit, float tMin, float& closestT, int& id, int i) {
    if (ifHit < 0.0f) {
        const float halfCut = sqrt_rn(-ifHit);
        const float t1 = rsProj - halfCut, t2 = rsProj + halfCut;
        const bool ok1 = (t1 > tMin) & (t1 < closestT);
        const bool ok2 = (t2 > tMin) & (t2 < closestT);
        id = (ok1 | ok2) ? i : id;
        closestT = ok1 ? t1 : ok2 ? t2 : closestT;
    }
}

// HitWorld + HitSphere (parallel.cpp:54-73, maths.cpp:51-94). The per-sphere test
// is the reference's; hit position and normal are computed once for the winner
// (they are pure functions of (ray, t, sphere), so this is bit-identical to the
// reference overwriting them on every closer hit).
// kNS > 0: the scene has exactly kNS spheres (the reference's kSphereCount is a compile-time
// 9, parallel.cpp:27): the scan is fully unrolled with constant LDS offsets.
template <int kAcc = 0, int kNS = 0>
LRT_DEV int ClosestHitSV(const Ray& r, float tMin, float tMax, const SceneView& sc, float& tOut,
                         bool coherent = false) {
    if constexpr (kAcc == kAccGrid)   // tMin/tMax = kMinT/kMaxT
        return ClosestHitGrid(r.orig, r.dir, sc.gv, tOut);
    if constexpr (kAcc == kAccBvh)
        return ClosestHitBVH(r.orig, r.dir, sc.bv, tOut, sc.bstk, sc.bstride, nullptr, coherent);
    float closestT = tMax;
    int id = -1;
    auto test = [&](int i, const float4& s) {
        F3 rs = f3(s.x, s.y, s.z) - r.orig;
        float rsProj = dot(rs, r.dir);
        float ifHit = dot(rs, rs) - rsProj * rsProj - s.w;
        SphereRoots(rsProj, ifHit, tMin, closestT, id, i);
    };
    if constexpr (kNS > 0) {
        float4 next = sc.sph[0];   // one sphere ahead (as DualClosestHit)
#pragma unroll
        for (int i = 0; i < kNS; ++i) {
            const float4 s = next;
            if (i + 1 < kNS) next = sc.sph[i + 1];
            test(i, s);
        }
    } else {
        float4 next = sc.sph[0];   // one sphere ahead
        for (int i = 0; i < sc.count; ++i) {
            const float4 s = next;
            if (i + 1 < sc.count) next = sc.sph[i + 1];
            test(i, s);
        }
    }
    tOut = closestT;
    return id;
}
// The plain scan over a sphere array (host diagnostics: lrt_bvh_stats checks the BVH
// against it). Same per-sphere arithmetic and strict-< replacement as HitWorld.
LRT_DEV int ClosestHit(const F3& o, const F3& d, const float4* sph, int count, float& tOut) {
    float closestT = kMaxT;
    int id = -1;
    for (int i = 0; i < count; ++i) {
        const float4 s = sph[i];
        const F3 rs = f3(s.x, s.y, s.z) - o;
        const float rsProj = dot(rs, d);
        const float ifHit = dot(rs, rs) - rsProj * rsProj - s.w;
        SphereRoots(rsProj, ifHit, kMinT, closestT, id, i);
    }
    tOut = closestT;
    return id;
}

template <int kAcc = 0, int kNS = 0>
LRT_DEV bool HitWorld(const Ray& r, float tMin, float tMax, const SceneView& sc, Hit& outHit, int& outID,
                      bool coherent = false) {
    float closestT;
    sec_count(sc, coherent ? kSecHit0 : kSecHit);
    const int id = ClosestHitSV<kAcc, kNS>(r, tMin, tMax, sc, closestT, coherent);
    if (id < 0) return false;
    float4 s = sc.sph[id];
    outHit.pos = point_at(r, closestT);
    outHit.normal = normalize(outHit.pos - f3(s.x, s.y, s.z));
    outHit.t = closestT;
    outID = id;
    return true;
}

// Scatter (parallel.cpp:78-196). The reference's `&mat == &smat` self test is the
// comparison of table indices (matId). lightE accumulates in the same order.
// Every material ends in `Ray(rec.pos, normalize(X))`, i.e. dir = normalize(normalize(X))
// (the Ray ctor normalises again, maths.h:133-137), so ScatterDir returns X and the
// caller forms the ray once for whichever materials the wave's lanes hold; Metal's
// absorption test (:147) is applied there too. The attenuation is the material's
// `att` row (albedo or 1), read back by the fold.
// The last light sample of a Lambert scatter, left for the caller to trace together with
// the next bounce ray (TraceDual): its direction, light index and the contribution
// (mat.albedo * emissive) * (max(0, l.nl) * omega / pi) it adds if the shadow ray's
// closest hit is that light (parallel.cpp:122-132; a pure function of values known
// before the shadow test, so precomputing it changes no bits).
struct DeferredLight {
    F3 l, contrib;   // l: the shadow ray's direction
    int li;
    bool on;
    int id;          // the scattering sphere (pool kernel: its stack entry's material)
};

template <int kAcc = 0, int kNS = 0>
LRT_DEV F3 ScatterDir(const Material& mat, int matId, const Ray& r_in, const Hit& rec, F3& outLightE,
                      int& inoutRayCount, uint32_t& rng, const SceneView& sc, DeferredLight* defer = nullptr,
                      bool coherent = false) {
    outLightE = f3(0.0f, 0.0f, 0.0f);
    if (mat.type == 0) {  // Lambert :81-136
        sec_count(sc, kSecLambert);
        // the first light's index and sphere, read before RandomUnitVector: their two dependent
        // LDS reads are in flight across it instead of waited for at the light loop's start
        // (config 2 -0.3 % / -0.7 % on two streams / one, config 3 -0.5 %: profiles/r6_ao)
        const int i0 = sc.nlights > 0 ? sc.lights[0] : 0;
        const float4 s0 = sc.sph[i0];
        F3 target = rec.pos + rec.normal + RandomUnitVector(rng);
        const F3 X = target - rec.pos;
        for (int k = 0; k < sc.nlights; ++k) {
            int i = k == 0 ? i0 : sc.lights[k];
            if (i == matId) continue;  // :98
            float4 s = k == 0 ? s0 : sc.sph[i];
            F3 c = f3(s.x, s.y, s.z);
            // sw = normalize(c - pos) and len = length(pos - c) (:103,:108): pos - c is
            // -(c - pos) exactly, so both lengths are the same float -- computed once
            const F3 cp = c - rec.pos;
            const float len = length(cp);
            const float kinv = rcp_rn(len);
            F3 sw = f3(cp.x * kinv, cp.y * kinv, cp.z * kinv);
            F3 su = normalize(cross(__builtin_fabsf(sw.x) > 0.01f ? f3(0.0f, 1.0f, 0.0f) : f3(1.0f, 0.0f, 0.0f), sw));
            F3 sv = cross(sw, su);
            float cosAMax = sqrt_rn(1.0f - s.w / (len * len));                    // :109
            float eps1 = RandomFloat01(rng);
            float eps2 = RandomFloat01(rng);
            float cosA = 1.0f - eps1 + eps1 * cosAMax;
            float sinA = sqrt_rn(1.0f - cosA * cosA);
            float phi = 2.0f * kPI * eps2;
            float sphi, cphi;
            libm::sincosf(phi, &sphi, &cphi);   // bit-identical to cosf(phi), sinf(phi)
            F3 l = su * cphi * sinA + sv * sphi * sinA + sw * cosA;                         // :116
            l = normalize_member(l);                                                      // :117
            float tLight;
            ++inoutRayCount;                                                              // :122
            if (defer && k == sc.nlights - 1) {   // the last light: traced with the bounce ray
                float omega = 2.0f * kPI * (1.0f - cosAMax);
                F3 rdir = r_in.dir;
                F3 nl = dot(rec.normal, rdir) < 0.0f ? rec.normal : -rec.normal;
                float d = dot(l, nl);
                float mx = (0.0f < d) ? d : 0.0f;   // std::max(0.0f, d)
                const float4 e = sc.mats[3 * i + 1];
                defer->l = renormalize(l, sc.rnlut);   // the shadow Ray's ctor normalises again (maths.h:133-137)
                defer->contrib = (mat.albedo * f3(e.x, e.y, e.z)) * (mx * omega / kPI);
                defer->li = i;
                defer->on = true;
                continue;
            }
            sec_count(sc, coherent ? kSecShadow0 : kSecShadow);
            bool lit;
            if constexpr (kAcc == kAccGrid) {
                lit = ShadowReachesLightGrid(rec.pos, renormalize(l, sc.rnlut), i, s, sc.gv);
            } else if constexpr (kAcc == kAccBvh) {
                Ray sr;
                sr.orig = rec.pos;
                sr.dir = renormalize(l, sc.rnlut);
                lit = ShadowReachesLightBVH(sr.orig, sr.dir, i, s, sc.bv, sc.bstk, sc.bstride, coherent);
            } else {
                Ray sr;
                sr.orig = rec.pos;
                sr.dir = renormalize(l, sc.rnlut);
                lit = ClosestHitSV<kAcc, kNS>(sr, kMinT, kMaxT, sc, tLight) == i;
            }
            sec_enter(sc, kSecLambert, false);
            if (lit) {   // HitWorld && hitID == i
                float omega = 2.0f * kPI * (1.0f - cosAMax);
                F3 rdir = r_in.dir;
                F3 nl = dot(rec.normal, rdir) < 0.0f ? rec.normal : -rec.normal;
                float d = dot(l, nl);
                float mx = (0.0f < d) ? d : 0.0f;   // std::max(0.0f, d)
                const float4 e = sc.mats[3 * i + 1];
                outLightE = outLightE + (mat.albedo * f3(e.x, e.y, e.z)) * (mx * omega / kPI);
            }
        }
        return X;
    } else if (mat.type == 1) {  // Metal :137-148
        sec_count(sc, kSecMetal);
        F3 refl = reflect(r_in.dir, rec.normal);
        return refl + mat.roughness * RandomInUnitSphere(rng);
    }
    // Dielectric :149-193 (validate() admits types 0-2 only)
    sec_count(sc, kSecDiel);
    F3 outwardN;
    F3 rdir = r_in.dir;
    F3 refl = reflect(rdir, rec.normal);
    float nint;
    F3 refr = f3(0.0f, 0.0f, 0.0f);
    float reflProb;
    float cosine;
    if (dot(rdir, rec.normal) > 0.0f) {
        outwardN = -rec.normal;
        nint = mat.ri;
        cosine = dot(rdir, rec.normal);
    } else {
        outwardN = rec.normal;
        nint = rcp_rn(mat.ri);
        cosine = -dot(rdir, rec.normal);
    }
    if (refract(rdir, outwardN, nint, refr))
        reflProb = schlick(cosine, mat.ri, sc.pow);
    else
        reflProb = 1.0f;
    return RandomFloat01(rng) < reflProb ? refl : refr;
}

// Scatter in the reference's shape (parallel.cpp:78-196): the attenuation, the scattered
// Ray (its ctor normalises the direction again, maths.h:133-137), the explicit light
// samples in outLightE, shadow rays counted in inoutRayCount; returns false where the
// reference absorbs (Metal scattered below the surface, :147). The RNG state and the scene
// are explicit parameters, as in the reference's own per-stream variant
// (src/cpu/README.md:42, fragmentShader.fs.glsl:175-218). `mat.id` is the material's table
// index, the reference's `&mat` identity. coherent: the active lanes' shadow rays start
// together (packet traversal, lrt_bvh.h).
template <int kAcc = 0, int kNS = 0>
LRT_DEV bool Scatter(const Material& mat, const Ray& r_in, const Hit& rec, F3& attenuation, Ray& scattered,
                     F3& outLightE, int& inoutRayCount, uint32_t& rng, const SceneView& sc, bool coherent = false) {
    const F3 X = ScatterDir<kAcc, kNS>(mat, mat.id, r_in, rec, outLightE, inoutRayCount, rng, sc, nullptr, coherent);
    scattered.orig = rec.pos;
    scattered.dir = renormalize(normalize(X), sc.rnlut);   // Ray(rec.pos, normalize(X))
    attenuation = mat.att;                                  // albedo, or (1, 1, 1) for Dielectric (:192)
    return mat.type != 1 || dot(scattered.dir, rec.normal) > 0.0f;
}

// Trace (parallel.cpp:200-227) as a loop. Scatter events are pushed on a per-lane
// stack of (matE + lightE, material id); the fold T = E + att * T from the leaf
// outwards reproduces the recursion's rounding exactly. maxDepth scatter events at
// most (the reference's depth < kMaxDepth test); MAXD >= maxDepth.
// lstk: this lane's LDS stack (kLdsLev levels, stride lstride float4); levels beyond
// it (only when MAXD > kLdsLev) go to this lane's slice of a global overflow stack
// (gstk, stride gstride; L2-resident -- few paths get that deep).
constexpr int kTraceLdsLevels = 8;
template <int MAXD, bool kFeat, int kLdsLev, int kNS>
LRT_DEV F3 TraceDual(Ray r, int maxDepth, int& inoutRayCount, uint32_t& rng, const SceneView& sc,
                     float4* lstk, int lstride, float4* gstk, size_t gstride, int ndl, F3* feat);
// ndl (LRT_F_NO_DOUBLE_LIGHT): the GL loop's doMaterialE rule (fragmentShader.fs.glsl:430,
// 456-457) -- a scatter event reached through a Lambert bounce adds no emissive; the
// terminating hit always does. kFeat: feat[0..2] receive the first hit's normal,
// position and albedo (fragmentShader.fs.glsl:444-451; left untouched on a miss).
template <int MAXD, int kAcc = 0, bool kFeat = false, int kLdsLev = kTraceLdsLevels, int kNS = 0>
LRT_DEV F3 Trace(Ray r, int maxDepth, int& inoutRayCount, uint32_t& rng, const SceneView& sc,
                 float4* lstk, int lstride, float4* gstk, size_t gstride, int ndl = 0, F3* feat = nullptr) {
    if constexpr (!kAcc)
        return TraceDual<MAXD, kFeat, kLdsLev, kNS>(r, maxDepth, inoutRayCount, rng, sc, lstk, lstride, gstk, gstride,
                                               ndl, feat);
    auto put = [&](int lvl, float4 v) {
        if (MAXD <= kLdsLev || lvl < kLdsLev) lstk[lvl * lstride] = v;
        else gstk[(size_t)(lvl - kLdsLev) * gstride] = v;
    };
    auto get = [&](int lvl) -> float4 {
        if (MAXD <= kLdsLev || lvl < kLdsLev) return lstk[lvl * lstride];
        return gstk[(size_t)(lvl - kLdsLev) * gstride];
    };
    int depth = 0;
    bool prevLambert = false;
    F3 leaf;
    for (;;) {
        Hit rec;
        int id = 0;
        ++inoutRayCount;
        // the first rays of a wave's paths start together: packet traversal (lrt_bvh.h)
        const bool coherent = depth < kPacketDepth;
        if (!HitWorld<kAcc, kNS>(r, kMinT, kMaxT, sc, rec, id, coherent)) {
            float t = 0.5f * (r.dir.y + 1.0f);
            leaf = ((1.0f - t) * f3(1.0f, 1.0f, 1.0f) + t * f3(0.5f, 0.7f, 1.0f)) * 0.3f;
            break;
        }
        Material mat = load_material(sc.mats, id);
        F3 matE = mat.emissive;
        if (kFeat && depth == 0) {   // the first hit (depth 0 is only ever seen once)
            feat[0] = rec.normal;
            feat[1] = rec.pos;
            feat[2] = mat.albedo;
        }
        F3 lightE, attenuation;
        Ray scattered;
        // :212 -- the attenuation is the material's `att` row, which the fold reads back by id
        if (depth < maxDepth &&
            Scatter<kAcc, kNS>(mat, r, rec, attenuation, scattered, lightE, inoutRayCount, rng, sc, coherent)) {
            sec_count(sc, kSecPost);
            if (ndl && prevLambert) matE = f3(0.0f, 0.0f, 0.0f);
            prevLambert = mat.type == 0;
            F3 e = matE + lightE;
            put(depth, make_float4(e.x, e.y, e.z, __int_as_float(id)));
            ++depth;
            r = scattered;
            continue;
        }
        leaf = matE;
        break;
    }
    F3 T = leaf;
    sec_count(sc, kSecFold);
    for (int d = depth - 1; d >= 0; --d) {
        float4 s = get(d);
        float4 b = sc.mats[3 * __float_as_int(s.w) + 2];
        T = f3(s.x, s.y, s.z) + f3(b.x, b.y, b.z) * T;
    }
    sec_enter(sc, kSecOther, false);
    return T;
}

// One pass over the spheres for two rays from the same origin: the next bounce ray and
// (hasShadow) a light's shadow ray. rs = c - o and dot(rs, rs) are shared -- the very
// values HitSphere computes for each ray (maths.cpp:54-59) -- and each ray keeps its own
// shrinking closestT exactly as HitWorld does, so both results are bit-identical to two
// separate scans. Saves the shadow ray's separate, partly occupied pass.
template <int kNS = 0>
LRT_DEV void DualClosestHit(const F3& o, const F3& db, bool hasShadow, const F3& ds, const SceneView& sc,
                            int& idB, float& tB, int& idS) {
    float closestB = kMaxT, closestS = kMaxT;
    idB = -1;
    idS = -1;
    auto test = [&](int i, const float4& s) {
        const F3 rs = f3(s.x, s.y, s.z) - o;
        const float rr = dot(rs, rs);
        {
            const float rsProj = dot(rs, db);
            const float ifHit = rr - rsProj * rsProj - s.w;
            SphereRoots(rsProj, ifHit, kMinT, closestB, idB, i);
        }
        if (hasShadow) {
            const float rsProj = dot(rs, ds);
            const float ifHit = rr - rsProj * rsProj - s.w;
            SphereRoots(rsProj, ifHit, kMinT, closestS, idS, i);
        }
    };
    if constexpr (kNS > 0) {
        // one sphere ahead: the next sphere's LDS read is in flight across this one's test (read
        // at its use, each read's latency sat between two tests: config 2 -2.7 %, config 3 -2.3 %,
        // profiles/r6_ak)
        float4 next = sc.sph[0];
#pragma unroll
        for (int i = 0; i < kNS; ++i) {
            const float4 s = next;
            if (i + 1 < kNS) next = sc.sph[i + 1];
            test(i, s);
        }
    } else {
        float4 next = sc.sph[0];
        for (int i = 0; i < sc.count; ++i) {
            const float4 s = next;
            if (i + 1 < sc.count) next = sc.sph[i + 1];
            test(i, s);
        }
    }
    tB = closestB;
}

// Trace for the linear scan with the closest hit of each bounce ray found at the end of
// the previous iteration, in one pass with the last light's shadow ray (DualClosestHit).
// Same events, draws, ray counts and accumulation order as Trace.
template <int MAXD, bool kFeat = false, int kLdsLev = kTraceLdsLevels, int kNS = 0>
LRT_DEV F3 TraceDual(Ray r, int maxDepth, int& inoutRayCount, uint32_t& rng, const SceneView& sc,
                     float4* lstk, int lstride, float4* gstk, size_t gstride, int ndl, F3* feat) {
    auto put = [&](int lvl, float4 v) {
        if (MAXD <= kLdsLev || lvl < kLdsLev) lstk[lvl * lstride] = v;
        else gstk[(size_t)(lvl - kLdsLev) * gstride] = v;
    };
    auto get = [&](int lvl) -> float4 {
        if (MAXD <= kLdsLev || lvl < kLdsLev) return lstk[lvl * lstride];
        return gstk[(size_t)(lvl - kLdsLev) * gstride];
    };
    int depth = 0;
    bool prevLambert = false;
    F3 leaf;
    Hit rec;
    int id = 0;
    ++inoutRayCount;
    bool hit = HitWorld<false, kNS>(r, kMinT, kMaxT, sc, rec, id);
    for (;;) {
        if (!hit) {
            float t = 0.5f * (r.dir.y + 1.0f);
            leaf = ((1.0f - t) * f3(1.0f, 1.0f, 1.0f) + t * f3(0.5f, 0.7f, 1.0f)) * 0.3f;
            break;
        }
        Material mat = load_material(sc.mats, id);
        F3 matE = mat.emissive;
        if (kFeat && depth == 0) {
            feat[0] = rec.normal;
            feat[1] = rec.pos;
            feat[2] = mat.albedo;
        }
        if (depth < maxDepth) {   // :212
            F3 lightE;
            DeferredLight dl;
            dl.on = false;
            const F3 X = ScatterDir<false, kNS>(mat, id, r, rec, lightE, inoutRayCount, rng, sc, &dl);
            sec_count(sc, kSecPost);
            const F3 dir = renormalize(normalize(X), sc.rnlut);
            if (mat.type != 1 || dot(dir, rec.normal) > 0.0f) {   // Metal absorbs (:147)
                // the next Trace's HitWorld (:204) and the deferred shadow ray (:122-123)
                ++inoutRayCount;
                sec_count(sc, kSecHit);
                int nid, sid;
                float nt;
                DualClosestHit<kNS>(rec.pos, dir, dl.on, dl.l, sc, nid, nt, sid);
                if (dl.on && sid == dl.li) lightE = lightE + dl.contrib;
                sec_enter(sc, kSecPost, false);
                if (ndl && prevLambert) matE = f3(0.0f, 0.0f, 0.0f);
                prevLambert = mat.type == 0;
                F3 e = matE + lightE;
                put(depth, make_float4(e.x, e.y, e.z, __int_as_float(id)));
                ++depth;
                r.orig = rec.pos;
                r.dir = dir;
                hit = nid >= 0;
                if (hit) {   // HitWorld's winner data (maths.cpp:74-76,86-88)
                    const float4 s = sc.sph[nid];
                    rec.pos = point_at(r, nt);
                    rec.normal = normalize(rec.pos - f3(s.x, s.y, s.z));
                    rec.t = nt;
                    id = nid;
                }
                continue;
            }
        }
        leaf = matE;
        break;
    }
    F3 T = leaf;
    sec_count(sc, kSecFold);
    for (int d = depth - 1; d >= 0; --d) {
        float4 s = get(d);
        float4 b = sc.mats[3 * __float_as_int(s.w) + 2];
        T = f3(s.x, s.y, s.z) + f3(b.x, b.y, b.z) * T;
    }
    sec_enter(sc, kSecOther, false);
    return T;
}

struct CameraDev {   // maths.h:217-224
    F3 origin, a, u, r, llc, horiz, vert;
    float lensRadius;
};
LRT_DEV Ray GetRay(const CameraDev& c, float s, float t, uint32_t& rng, const float* lut = nullptr) {   // maths.h:205-215
    F3 rd = c.lensRadius * RandomInUnitDisk(rng);
    F3 offset = c.r * rd.x + c.u * rd.y;
    Ray r;
    r.orig = c.origin + offset;
    r.dir = renormalize(normalize(c.llc + s * c.horiz + t * c.vert - c.origin - offset), lut);
    return r;
}

LRT_DEV uint32_t PixelSeed(uint32_t x, uint32_t y, uint32_t f) { return (x * 1973u + y * 9277u + f * 26699u) | 1u; }

}  // namespace lrt
