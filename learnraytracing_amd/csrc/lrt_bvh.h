// Bit-exact BVH closest hit for N-sphere scenes (BASELINE configs 4-5).
//
// The reference scans every sphere in index order with a shrinking closestT
// (HitWorld, parallel.cpp:54-73; HitSphere, maths.cpp:51-94). For sphere i define
//     cand_i = t1 if t1 > tMin, else t2 if t2 > tMin, else +inf
// with t1 = proj - halfCut, t2 = proj + halfCut computed exactly as HitSphere does.
// cand_i does not depend on closestT, and sphere i replaces the running hit iff
// cand_i < closestT (strict). Hence the scan returns the lexicographic minimum of
// (cand_i, i) among spheres with cand_i < kMaxT: the smallest candidate, lowest index
// on ties. Any traversal order that evaluates the same per-sphere arithmetic and
// keeps (cand, index)-minimum returns the same id and t bit for bit, provided box
// culling never drops a sphere that could win. Boxes are padded and the cull test
// carries an absolute + relative margin far above float rounding (both set at build
// time from the scene's extent), so culling is conservative.
//
// Layout (global memory, L1/L2 resident): BVH2 nodes of 4 float4 holding both
// children's boxes. Child c: min.xyz + ref (int bits), max.xyz + count (int bits);
// count > 0: leaf of `count` spheres starting at `ref` in the leaf-ordered sphere
// array; count == 0: internal node `ref`; count < 0: empty. Leaf spheres are copies of
// the scene's float4(center, r^2) plus the original index (materials, ties, lights all
// keep using the original index).
//
// Included by lrt_trace.h (it uses F3, dot, kMinT, kMaxT defined there).
#pragma once
#include "lrt.h"   // LRT_MAX_SPHERES

namespace lrt {

constexpr int kBvhStackLevels = 24;   // builder guarantees depth <= 22

struct BvhView {
    const float4* nodes;    // 4 float4 per node, node 0 = root (none if nnodes == 0)
    const float4* lsph;     // leaf-ordered spheres, then the `big` spheres
    const int* lid;         // original index of each of those spheres
    float margin;           // absolute cull margin (scene-extent scaled)
    int on;                 // 0: linear scan
    int nnodes;
    int big0, nbig;         // spheres [big0, big0 + nbig) of lsph are tested before traversal:
                            // spheres far larger than the rest (the ground, r = 100) would make
                            // every ancestor box span the scene
};

LRT_DEV void SlabTest(const float4& mn, const float4& mx, const F3& o, const F3& inv, float& tn, float& tf) {
    const float tx0 = (mn.x - o.x) * inv.x, tx1 = (mx.x - o.x) * inv.x;
    const float ty0 = (mn.y - o.y) * inv.y, ty1 = (mx.y - o.y) * inv.y;
    const float tz0 = (mn.z - o.z) * inv.z, tz1 = (mx.z - o.z) * inv.z;
    // fminf/fmaxf drop a NaN operand (0 * inf on a slab plane): that axis then
    // constrains nothing, which only ever keeps a node (conservative)
    tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(tx0, tx1), __builtin_fminf(ty0, ty1)),
                         __builtin_fminf(tz0, tz1));
    tf = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(tx0, tx1), __builtin_fmaxf(ty0, ty1)),
                         __builtin_fmaxf(tz0, tz1));
}

// The 4-wide traversals' slab test: t = fma(plane, inv, -o * inv), one FMA per plane
// instead of a subtract and a multiply. Beyond the subtract-multiply form's rounding it
// errs by at most ulp(|o_k * inv_k|) per plane; MakeSlabRay bounds that once per ray
// and the culling margins add it, so culling stays conservative.
#ifndef LRT_BVH_FMA_SLAB
#define LRT_BVH_FMA_SLAB 1
#endif
LRT_DEV void SlabTestFma(const float4& mn, const float4& mx, const F3& inv, const F3& oi, float& tn, float& tf) {
    const float tx0 = __builtin_fmaf(mn.x, inv.x, -oi.x), tx1 = __builtin_fmaf(mx.x, inv.x, -oi.x);
    const float ty0 = __builtin_fmaf(mn.y, inv.y, -oi.y), ty1 = __builtin_fmaf(mx.y, inv.y, -oi.y);
    const float tz0 = __builtin_fmaf(mn.z, inv.z, -oi.z), tz1 = __builtin_fmaf(mx.z, inv.z, -oi.z);
    tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(tx0, tx1), __builtin_fminf(ty0, ty1)),
                         __builtin_fminf(tz0, tz1));
    tf = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(tx0, tx1), __builtin_fmaxf(ty0, ty1)),
                         __builtin_fmaxf(tz0, tz1));
}
// The FMA form is used only when no product can overflow: an infinite inv_k (a direction
// component of 0) makes plane * inv - o * inv an inf - inf = NaN, which the min/max would
// resolve to the wrong extreme. Such rays keep the subtract-multiply form. With finite
// products the extra margin is mo = 2^-22 * max_k |o_k * inv_k|, 4x the bound above.
struct SlabRay {
    F3 inv, oi;
    float mo;
    bool fma;
};
LRT_DEV SlabRay MakeSlabRay(const F3& o, const F3& d, float margin) {
    SlabRay r;
    r.inv = f3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    r.oi = f3(o.x * r.inv.x, o.y * r.inv.y, o.z * r.inv.z);
    const float mi = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(r.inv.x), __builtin_fabsf(r.inv.y)),
                                     __builtin_fabsf(r.inv.z));
    const float mo = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(o.x), __builtin_fabsf(o.y)), __builtin_fabsf(o.z));
    // margin = 1e-5 * extent + 1e-4 (build_bvh_host): every box coordinate is below 1e5 * margin
    const float bound = mi * (1.0e5f * margin + mo);
    r.fma = LRT_BVH_FMA_SLAB && bound < 1.0e30f;   // false for inf / NaN too
    r.mo = r.fma ? __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(r.oi.x), __builtin_fabsf(r.oi.y)),
                                   __builtin_fabsf(r.oi.z)) * 2.384185791015625e-07f
                 : 0.0f;
    return r;
}
LRT_DEV void SlabTest4(const float4& mn, const float4& mx, const F3& o, const SlabRay& sr, float& tn, float& tf) {
    if (sr.fma) SlabTestFma(mn, mx, sr.inv, sr.oi, tn, tf);
    else SlabTest(mn, mx, o, sr.inv, tn, tf);
}

struct BvhStats { int nodes = 0, spheres = 0; };   // host diagnostics (lrt_bvh_stats)

// LRT_BVH4 (default): the BVH2 collapsed to 4-wide nodes (8 float4: four children's boxes,
// same per-child encoding; empty slots have count -1). Half the levels, so fewer and
// fuller traversal iterations. A stack entry is (node << 4 | mask of the node's children
// still to visit), one entry per level. A popped entry descends into its first child
// without a second box test: every pushed child already passed the cull against a bound
// that has only shrunk since, so skipping the re-test is conservative.
#ifndef LRT_BVH4
#define LRT_BVH4 1
#endif
#ifndef LRT_BVH_CH_RETEST   // closest hit: re-test popped children against the shrunk bestT (A/B)
#define LRT_BVH_CH_RETEST 0
#endif
// A BVH4 stack entry is a u16 (node << 4 | mask): node indices must stay below 4096. The
// 4-wide node count is at most the BVH2's internal node count, < LRT_MAX_SPHERES.
static_assert(LRT_MAX_SPHERES <= 4096, "BVH4 stack entries hold 12-bit node indices");

// stk: this lane's traversal stack (kBvhStackLevels entries, stride `stride`).
LRT_DEV int ClosestHitBVH2(const F3& o, const F3& d, const BvhView& bv, float& tOut, unsigned short* stk,
                          int stride, BvhStats* st = nullptr) {
    const F3 inv = f3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    float bestT = kMaxT;
    int best = -1;
    int sp = 0, cur = 0;
    auto leaf = [&](int ref, int cnt) {
        if (st) st->spheres += cnt;
        for (int j = 0; j < cnt; ++j) {
            const float4 s = bv.lsph[ref + j];
            const F3 rs = f3(s.x, s.y, s.z) - o;                       // maths.cpp:54-59
            const float rsProj = dot(rs, d);
            const float ifHit = dot(rs, rs) - rsProj * rsProj - s.w;
            if (ifHit < 0.0f) {
                const float halfCut = sqrt_rn(-ifHit);
                const float t1 = rsProj - halfCut;
                const float t2 = rsProj + halfCut;
                const float cand = t1 > kMinT ? t1 : (t2 > kMinT ? t2 : __builtin_inff());
                const int id = bv.lid[ref + j];
                if (cand < bestT || (cand == bestT && best >= 0 && id < best)) {
                    bestT = cand;
                    best = id;
                }
            }
        }
    };
    leaf(bv.big0, bv.nbig);   // seeds bestT, which then culls the traversal
    if (bv.nnodes == 0) {
        tOut = bestT;
        return best;
    }
    for (;;) {
        const float4 a0 = bv.nodes[4 * cur + 0], a1 = bv.nodes[4 * cur + 1];
        const float4 b0 = bv.nodes[4 * cur + 2], b1 = bv.nodes[4 * cur + 3];
        if (st) st->nodes += 1;
        float tnA, tfA, tnB, tfB;
        SlabTest(a0, a1, o, inv, tnA, tfA);
        SlabTest(b0, b1, o, inv, tnB, tfB);
        // conservative margins: absolute (scene extent) + relative to the distances compared
        const float mb = bv.margin + 1e-5f * bestT;
        const float mA = bv.margin + 1e-5f * __builtin_fabsf(tfA);
        const float mB = bv.margin + 1e-5f * __builtin_fabsf(tfB);
        const int cntA = lrt::libm::f2u_i(a1.w), cntB = lrt::libm::f2u_i(b1.w);
        const bool hitA = cntA >= 0 && tnA <= tfA + mA && tnA <= bestT + mb && tfA >= kMinT - mA;
        const bool hitB = cntB >= 0 && tnB <= tfB + mB && tnB <= bestT + mb && tfB >= kMinT - mB;
        if (hitA && cntA > 0) leaf(lrt::libm::f2u_i(a0.w), cntA);
        if (hitB && cntB > 0) leaf(lrt::libm::f2u_i(b0.w), cntB);
        const bool goA = hitA && cntA == 0, goB = hitB && cntB == 0;
        if (goA && goB) {
            const bool aFirst = tnA <= tnB;
            stk[sp * stride] = (unsigned short)lrt::libm::f2u_i(aFirst ? b0.w : a0.w);
            ++sp;
            cur = lrt::libm::f2u_i(aFirst ? a0.w : b0.w);
        } else if (goA) {
            cur = lrt::libm::f2u_i(a0.w);
        } else if (goB) {
            cur = lrt::libm::f2u_i(b0.w);
        } else {
            if (sp == 0) break;
            --sp;
            cur = stk[sp * stride];
        }
    }
    tOut = bestT;
    return best;
}

// Light sampling's `HitWorld(shadow ray) && hitID == li` (parallel.cpp:122-123) through
// the BVH. (cand_li, li) must be the lexicographic minimum, so the light's own candidate
// is the bar from the start: boxes beyond it are culled (same conservative margins) and
// the first sphere that beats it -- cand_j < cand_li, or equal with j < li -- ends the
// traversal. Same per-sphere arithmetic as the scan, so the answer is bit-identical.
LRT_DEV float SphereCand(const F3& o, const F3& d, const float4& s) {   // maths.cpp:54-90
    const F3 rs = f3(s.x, s.y, s.z) - o;
    const float rsProj = dot(rs, d);
    const float ifHit = dot(rs, rs) - rsProj * rsProj - s.w;
    if (!(ifHit < 0.0f)) return __builtin_inff();
    const float halfCut = sqrt_rn(-ifHit);
    const float t1 = rsProj - halfCut;
    const float t2 = rsProj + halfCut;
    return t1 > kMinT ? t1 : (t2 > kMinT ? t2 : __builtin_inff());
}
LRT_DEV bool ShadowReachesLightBVH2(const F3& o, const F3& d, int li, const float4& lightSph, const BvhView& bv,
                                   unsigned short* stk, int stride) {
    const float candL = SphereCand(o, d, lightSph);
    if (!(candL < kMaxT)) return false;   // the light is not hit at all (closestT starts at kMaxT)
    auto beats = [&](float c, int id) { return c < candL || (c == candL && id < li); };
    for (int j = 0; j < bv.nbig; ++j)
        if (beats(SphereCand(o, d, bv.lsph[bv.big0 + j]), bv.lid[bv.big0 + j])) return false;
    if (bv.nnodes == 0) return true;
    const F3 inv = f3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const float mb = bv.margin + 1e-5f * candL;
    int sp = 0, cur = 0;
    for (;;) {
        const float4 a0 = bv.nodes[4 * cur + 0], a1 = bv.nodes[4 * cur + 1];
        const float4 b0 = bv.nodes[4 * cur + 2], b1 = bv.nodes[4 * cur + 3];
        float tnA, tfA, tnB, tfB;
        SlabTest(a0, a1, o, inv, tnA, tfA);
        SlabTest(b0, b1, o, inv, tnB, tfB);
        const float mA = bv.margin + 1e-5f * __builtin_fabsf(tfA);
        const float mB = bv.margin + 1e-5f * __builtin_fabsf(tfB);
        const int cntA = lrt::libm::f2u_i(a1.w), cntB = lrt::libm::f2u_i(b1.w);
        const bool hitA = cntA >= 0 && tnA <= tfA + mA && tnA <= candL + mb && tfA >= kMinT - mA;
        const bool hitB = cntB >= 0 && tnB <= tfB + mB && tnB <= candL + mb && tfB >= kMinT - mB;
        if (hitA && cntA > 0) {
            const int ref = lrt::libm::f2u_i(a0.w);
            for (int j = 0; j < cntA; ++j)
                if (beats(SphereCand(o, d, bv.lsph[ref + j]), bv.lid[ref + j])) return false;
        }
        if (hitB && cntB > 0) {
            const int ref = lrt::libm::f2u_i(b0.w);
            for (int j = 0; j < cntB; ++j)
                if (beats(SphereCand(o, d, bv.lsph[ref + j]), bv.lid[ref + j])) return false;
        }
        const bool goA = hitA && cntA == 0, goB = hitB && cntB == 0;
        if (goA && goB) {
            const bool aFirst = tnA <= tnB;
            stk[sp * stride] = (unsigned short)lrt::libm::f2u_i(aFirst ? b0.w : a0.w);
            ++sp;
            cur = lrt::libm::f2u_i(aFirst ? a0.w : b0.w);
        } else if (goA) {
            cur = lrt::libm::f2u_i(a0.w);
        } else if (goB) {
            cur = lrt::libm::f2u_i(b0.w);
        } else {
            if (sp == 0) break;
            --sp;
            cur = stk[sp * stride];
        }
    }
    return true;
}


// 4-wide ClosestHitBVH: same leaf arithmetic, (cand, id) minimum and conservative culling.
LRT_DEV int ClosestHitBVH4(const F3& o, const F3& d, const BvhView& bv, float& tOut, unsigned short* stk, int stride,
                           BvhStats* st = nullptr) {
    const SlabRay sr = MakeSlabRay(o, d, bv.margin);
    float bestT = kMaxT;
    int best = -1;
    auto leaf = [&](int ref, int cnt) {
        if (st) st->spheres += cnt;
        for (int j = 0; j < cnt; ++j) {
            const float4 s = bv.lsph[ref + j];
            const F3 rs = f3(s.x, s.y, s.z) - o;                       // maths.cpp:54-59
            const float rsProj = dot(rs, d);
            const float ifHit = dot(rs, rs) - rsProj * rsProj - s.w;
            if (ifHit < 0.0f) {
                const float halfCut = sqrt_rn(-ifHit);
                const float t1 = rsProj - halfCut;
                const float t2 = rsProj + halfCut;
                const float cand = t1 > kMinT ? t1 : (t2 > kMinT ? t2 : __builtin_inff());
                const int id = bv.lid[ref + j];
                if (cand < bestT || (cand == bestT && best >= 0 && id < best)) {
                    bestT = cand;
                    best = id;
                }
            }
        }
    };
    leaf(bv.big0, bv.nbig);
    if (bv.nnodes == 0) {
        tOut = bestT;
        return best;
    }
    int sp = 0, cur = 0, msk = 0xF;
    for (;;) {
        if (st) st->nodes += 1;
        const float mb = bv.margin + sr.mo + 1e-5f * bestT;
        const float mbase = bv.margin + sr.mo;
        int next = -1, rem = 0;
        float nearT = __builtin_inff();
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (!((msk >> c) & 1)) continue;
            const float4 lo = bv.nodes[8 * cur + 2 * c], hi = bv.nodes[8 * cur + 2 * c + 1];
            const int cnt = lrt::libm::f2u_i(hi.w);
            if (cnt < 0) continue;
            float tn, tf;
            SlabTest4(lo, hi, o, sr, tn, tf);
            const float m = __builtin_fmaf(1e-5f, __builtin_fabsf(tf), mbase);   // a margin: rounding is immaterial
            const float tfm = tf + m;   // (tn <= tf + m, tn <= bestT + mb, tf + m >= kMinT)
            if (!(tn <= __builtin_fminf(tfm, bestT + mb) && tfm >= kMinT)) continue;
            if (cnt > 0) {
                leaf(lrt::libm::f2u_i(lo.w), cnt);
            } else {
                rem |= 1 << c;
                if (tn < nearT) {
                    nearT = tn;
                    next = c;
                }
            }
        }
        if (next >= 0) {
            rem &= ~(1 << next);
            if (rem) {
                stk[sp * stride] = (unsigned short)((cur << 4) | rem);
                ++sp;
            }
            cur = lrt::libm::f2u_i(bv.nodes[8 * cur + 2 * next].w);
            msk = 0xF;
        } else {
            if (sp == 0) break;
            --sp;
            const int e = stk[sp * stride];
            cur = e >> 4;
            msk = e & 0xF;
#if !LRT_BVH_CH_RETEST
            const int c = __builtin_ctz(msk);
            msk &= msk - 1;
            if (msk) {
                stk[sp * stride] = (unsigned short)((cur << 4) | msk);
                ++sp;
            }
            cur = lrt::libm::f2u_i(bv.nodes[8 * cur + 2 * c].w);
            msk = 0xF;
#endif
        }
    }
    tOut = bestT;
    return best;
}

LRT_DEV bool ShadowReachesLightBVH4(const F3& o, const F3& d, int li, const float4& lightSph, const BvhView& bv,
                                    unsigned short* stk, int stride) {
    const float candL = SphereCand(o, d, lightSph);
    if (!(candL < kMaxT)) return false;   // the light is not hit at all (closestT starts at kMaxT)
    auto beats = [&](float c, int id) { return c < candL || (c == candL && id < li); };
    for (int j = 0; j < bv.nbig; ++j)
        if (beats(SphereCand(o, d, bv.lsph[bv.big0 + j]), bv.lid[bv.big0 + j])) return false;
    if (bv.nnodes == 0) return true;
    const SlabRay sr = MakeSlabRay(o, d, bv.margin);
    const float mb = bv.margin + sr.mo + 1e-5f * candL;
    const float mbase = bv.margin + sr.mo;
    int sp = 0, cur = 0, msk = 0xF;
    for (;;) {
        int next = -1, rem = 0;
        float nearT = __builtin_inff();
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (!((msk >> c) & 1)) continue;
            const float4 lo = bv.nodes[8 * cur + 2 * c], hi = bv.nodes[8 * cur + 2 * c + 1];
            const int cnt = lrt::libm::f2u_i(hi.w);
            if (cnt < 0) continue;
            float tn, tf;
            SlabTest4(lo, hi, o, sr, tn, tf);
            const float m = __builtin_fmaf(1e-5f, __builtin_fabsf(tf), mbase);   // a margin: rounding is immaterial
            const float tfm = tf + m;   // (tn <= tf + m, tn <= candL + mb, tf + m >= kMinT)
            if (!(tn <= __builtin_fminf(tfm, candL + mb) && tfm >= kMinT)) continue;
            if (cnt > 0) {
                const int ref = lrt::libm::f2u_i(lo.w);
                for (int j = 0; j < cnt; ++j)
                    if (beats(SphereCand(o, d, bv.lsph[ref + j]), bv.lid[ref + j])) return false;
            } else {
                rem |= 1 << c;
                if (tn < nearT) {
                    nearT = tn;
                    next = c;
                }
            }
        }
        if (next >= 0) {
            rem &= ~(1 << next);
            if (rem) {
                stk[sp * stride] = (unsigned short)((cur << 4) | rem);
                ++sp;
            }
            cur = lrt::libm::f2u_i(bv.nodes[8 * cur + 2 * next].w);
            msk = 0xF;
        } else {
            if (sp == 0) break;
            --sp;
            const int e = stk[sp * stride];
            cur = e >> 4;
            msk = e & 0xF;
            // candL does not shrink, so the popped children's boxes passed already: descend
            // into the first without testing again, push the rest back
            const int c = __builtin_ctz(msk);
            msk &= msk - 1;
            if (msk) {
                stk[sp * stride] = (unsigned short)((cur << 4) | msk);
                ++sp;
            }
            cur = lrt::libm::f2u_i(bv.nodes[8 * cur + 2 * c].w);
            msk = 0xF;
        }
    }
    return true;
}

// The layout the host built (build_bvh_host): 4-wide unless LRT_BVH4=0.
LRT_DEV int ClosestHitBVH(const F3& o, const F3& d, const BvhView& bv, float& tOut, unsigned short* stk, int stride,
                          BvhStats* st = nullptr) {
    return LRT_BVH4 ? ClosestHitBVH4(o, d, bv, tOut, stk, stride, st) : ClosestHitBVH2(o, d, bv, tOut, stk, stride, st);
}
LRT_DEV bool ShadowReachesLightBVH(const F3& o, const F3& d, int li, const float4& lightSph, const BvhView& bv,
                                   unsigned short* stk, int stride) {
    return LRT_BVH4 ? ShadowReachesLightBVH4(o, d, li, lightSph, bv, stk, stride)
                    : ShadowReachesLightBVH2(o, d, li, lightSph, bv, stk, stride);
}

}  // namespace lrt
