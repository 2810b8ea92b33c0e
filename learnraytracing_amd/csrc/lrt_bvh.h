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
    // Exactness reach: each box is padded by the reference's hit excursion
    // (hit_excursion, lrt_grid_build.h) for origins within sqrt(f2near) of every corner of the
    // tree spheres' centre box (clo, chi); a ray from anywhere else inflates every box it tests
    // by its own bound, hit_excursion(F + rmax, rmin) with F its farthest-corner distance
    // (MakeSlabRay).
    float clox, cloy, cloz, chix, chiy, chiz;
    float f2near, rmax, rmin;
};

// ei: per-axis inflation of the box in t (e |inv_k|, a far ray's hit excursion e; 0 for the
// others, which leaves every value as it was)
LRT_DEV void SlabTest(const float4& mn, const float4& mx, const F3& o, const F3& inv, const F3& ei, float& tn,
                      float& tf) {
    const float tx0 = (mn.x - o.x) * inv.x, tx1 = (mx.x - o.x) * inv.x;
    const float ty0 = (mn.y - o.y) * inv.y, ty1 = (mx.y - o.y) * inv.y;
    const float tz0 = (mn.z - o.z) * inv.z, tz1 = (mx.z - o.z) * inv.z;
    // fminf/fmaxf drop a NaN operand (0 * inf on a slab plane, inf - inf of an inflated
    // infinite slab): that axis then constrains nothing, which only ever keeps a node
    tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(tx0, tx1) - ei.x, __builtin_fminf(ty0, ty1) - ei.y),
                         __builtin_fminf(tz0, tz1) - ei.z);
    tf = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(tx0, tx1) + ei.x, __builtin_fmaxf(ty0, ty1) + ei.y),
                         __builtin_fmaxf(tz0, tz1) + ei.z);
}

// The 4-wide traversals' slab test: t = fma(plane, inv, -o * inv), one FMA per plane
// instead of a subtract and a multiply. Beyond the subtract-multiply form's rounding it
// errs by at most ulp(|o_k * inv_k|) per plane; MakeSlabRay bounds that once per ray
// and the culling margins add it, so culling stays conservative.
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
// Rays from beyond the BVH's near reach (f2near) take the subtract-multiply form with
// every box inflated by their own hit excursion (oi then holds e |inv_k|; 0 for the other
// rays of that form).
struct SlabRay {
    F3 inv, oi;
    float mo;
    bool fma;
};
// hit_excursion (lrt_grid_build.h) for any sphere of the tree from an origin whose farthest
// centre-box corner lies sqrt(f2) away, in float with a 2^-8 safety factor (its own rounding is
// ~1e-7 relative); inf when it overflows or the origin is not finite.
LRT_DEV float FarExcursion(float f2, const BvhView& bv) {
    const float D = sqrt_rn(f2) * 1.00000095367431640625f + bv.rmax;
    const float E = D * D * 1.9073486328125e-06f;   // 2^-19 D^2
    const float e = (E / (sqrt_rn(bv.rmin * bv.rmin + E) + bv.rmin) + D * 1.430511474609375e-06f) * 1.00390625f;
    return e < 3.0e38f ? e : __builtin_inff();
}
LRT_DEV SlabRay MakeSlabRay(const F3& o, const F3& d, const BvhView& bv) {
    SlabRay r;
    r.inv = f3(rcp_rn(d.x), rcp_rn(d.y), rcp_rn(d.z));   // = 1.0f / d (lrt_trace.h), shorter
    r.oi = f3(o.x * r.inv.x, o.y * r.inv.y, o.z * r.inv.z);
    const float mi = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(r.inv.x), __builtin_fabsf(r.inv.y)),
                                     __builtin_fabsf(r.inv.z));
    const float mo = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(o.x), __builtin_fabsf(o.y)), __builtin_fabsf(o.z));
    // margin = 1e-5 * extent + 1e-4 (build_bvh_host): every box coordinate is below 1e5 * margin
    const float bound = mi * (1.0e5f * bv.margin + mo);
    const float fx = __builtin_fmaxf(__builtin_fabsf(o.x - bv.clox), __builtin_fabsf(o.x - bv.chix));
    const float fy = __builtin_fmaxf(__builtin_fabsf(o.y - bv.cloy), __builtin_fabsf(o.y - bv.chiy));
    const float fz = __builtin_fmaxf(__builtin_fabsf(o.z - bv.cloz), __builtin_fabsf(o.z - bv.chiz));
    const float f2 = fx * fx + fy * fy + fz * fz;
    const bool near = f2 <= bv.f2near;   // false for NaN too
    r.fma = near & (bound < 1.0e30f);   // false for inf / NaN too
    r.mo = r.fma ? __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(r.oi.x), __builtin_fabsf(r.oi.y)),
                                   __builtin_fabsf(r.oi.z)) * 2.384185791015625e-07f
                 : 0.0f;
    if (!r.fma) {
        const float e = near ? 0.0f : FarExcursion(f2, bv);
        r.oi = e > 0.0f ? f3(e * __builtin_fabsf(r.inv.x), e * __builtin_fabsf(r.inv.y), e * __builtin_fabsf(r.inv.z))
                        : f3(0.0f, 0.0f, 0.0f);
    }
    return r;
}
LRT_DEV void SlabTest4(const float4& mn, const float4& mx, const F3& o, const SlabRay& sr, float& tn, float& tf) {
    if (sr.fma) SlabTestFma(mn, mx, sr.inv, sr.oi, tn, tf);
    else SlabTest(mn, mx, o, sr.inv, sr.oi, tn, tf);
}

// Host diagnostics (lrt_bvh_stats): node visits, sphere tests and the deepest traversal
// stack entry written, checked against the levels the LDS stack is sized to.
struct BvhStats { int nodes = 0, spheres = 0, max_sp = 0; };

// The BVH2 the host builds is collapsed to 4-wide nodes (8 float4: four children's boxes,
// per-child encoding as above; empty slots have count -1). A stack entry is a u16 (node << 4
// | mask of the node's children still to visit), one entry per level: a push happens only
// when descending from a node to an internal child, so the stack never holds more entries
// than the tree's depth (BvhHost::stack_levels, which sizes the LDS stack). A popped entry
// descends into its first child without a second box test: every pushed child already
// passed the cull against a bound that has only shrunk since, so skipping the re-test is
// conservative. Node indices must stay below 4096 (12 bits).
static_assert(LRT_MAX_SPHERES <= 4096, "BVH4 stack entries hold 12-bit node indices");

template <int kForm>   // 1: FMA slab form, 2: subtract-multiply form (MakeSlabRay chooses per ray)
LRT_DEV void SlabTestK(const float4& mn, const float4& mx, const F3& o, const SlabRay& sr, float& tn, float& tf) {
    if (kForm == 1) SlabTestFma(mn, mx, sr.inv, sr.oi, tn, tf);
    else SlabTest(mn, mx, o, sr.inv, sr.oi, tn, tf);
}

// Pushes (node, mask) as stack entry sp (host builds track the depth reached).
LRT_DEV void StackPush(unsigned short* stk, int stride, int& sp, int node, int mask, BvhStats* st) {
    stk[sp * stride] = (unsigned short)((node << 4) | mask);
    ++sp;
    if (st && sp > st->max_sp) st->max_sp = sp;
}

// 4-wide closest hit: the reference's per-sphere arithmetic, the (cand, id) minimum and
// conservative culling. The winner is kept as its position in lsph; the original index is
// read only on an exact tie and once at the end.
template <int kForm>
LRT_DEV int ClosestHitBVH4Impl(const F3& o, const F3& d, const SlabRay& sr, const BvhView& bv, float& tOut,
                               unsigned short* stk, int stride, BvhStats* st) {
    float bestT = kMaxT;
    int best = -1;
    auto test = [&](int pos, const float4& s) {
        const F3 rs = f3(s.x, s.y, s.z) - o;                       // maths.cpp:54-59
        const float rsProj = dot(rs, d);
        const float ifHit = dot(rs, rs) - rsProj * rsProj - s.w;
        if (ifHit < 0.0f) {
            const float halfCut = sqrt_rn(-ifHit);
            const float t1 = rsProj - halfCut;
            const float t2 = rsProj + halfCut;
            const float cand = t1 > kMinT ? t1 : (t2 > kMinT ? t2 : __builtin_inff());
            if (cand < bestT || (cand == bestT && best >= 0 && bv.lid[pos] < bv.lid[best])) {
                bestT = cand;
                best = pos;
            }
        }
    };
    auto leaf = [&](int ref, int cnt) {
        if (st) st->spheres += cnt;
        for (int j = 0; j < cnt; ++j) test(ref + j, bv.lsph[ref + j]);
    };
    leaf(bv.big0, bv.nbig);
    int sp = 0, cur = 0, msk = bv.nnodes == 0 ? 0 : 0xF;
    while (msk) {
        if (st) st->nodes += 1;
        const float mb = bv.margin + sr.mo + 1e-5f * bestT;
        const float mbase = bv.margin + sr.mo;
        int next = -1, rem = 0, nextRef = 0;
        float nearT = __builtin_inff();
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (!((msk >> c) & 1)) continue;
            const float4 lo = bv.nodes[8 * cur + 2 * c];
            const float4 hi = bv.nodes[8 * cur + 2 * c + 1];
            const int cnt = lrt::libm::f2u_i(hi.w);
            if (cnt < 0) continue;
            float tn, tf;
            SlabTestK<kForm>(lo, hi, o, sr, tn, tf);
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
                    nextRef = lrt::libm::f2u_i(lo.w);
                }
            }
        }
        if (next >= 0) {
            rem &= ~(1 << next);
            if (rem) StackPush(stk, stride, sp, cur, rem, st);
            cur = nextRef;
            msk = 0xF;
        } else {
            if (sp == 0) break;
            --sp;
            const int e = stk[sp * stride];
            cur = e >> 4;
            msk = e & 0xF;
            const int c = __builtin_ctz(msk);
            msk &= msk - 1;
            if (msk) StackPush(stk, stride, sp, cur, msk, st);
            cur = lrt::libm::f2u_i(bv.nodes[8 * cur + 2 * c].w);
            msk = 0xF;
        }
    }
    tOut = bestT;
    return best >= 0 ? bv.lid[best] : best;
}

LRT_DEV int ClosestHitBVH4(const F3& o, const F3& d, const BvhView& bv, float& tOut, unsigned short* stk, int stride,
                           BvhStats* st = nullptr) {
    const SlabRay sr = MakeSlabRay(o, d, bv);
    if (sr.fma) return ClosestHitBVH4Impl<1>(o, d, sr, bv, tOut, stk, stride, st);
    return ClosestHitBVH4Impl<2>(o, d, sr, bv, tOut, stk, stride, st);
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
template <int kForm>
LRT_DEV bool ShadowReachesLightBVH4Impl(const F3& o, const F3& d, int li, float candL, const SlabRay& sr,
                                        const BvhView& bv, unsigned short* stk, int stride, BvhStats* st) {
    // (cand, index) beats the light's (candL, li); the index is read only on an exact tie
    auto beats = [&](float c, int pos) { return c < candL || (c == candL && bv.lid[pos] < li); };
    for (int j = 0; j < bv.nbig; ++j)
        if (beats(SphereCand(o, d, bv.lsph[bv.big0 + j]), bv.big0 + j)) return false;
    if (bv.nnodes == 0) return true;
    const float mb = bv.margin + sr.mo + 1e-5f * candL;
    const float mbase = bv.margin + sr.mo;
    int sp = 0, cur = 0, msk = 0xF;
    for (;;) {
        int next = -1, rem = 0, nextRef = 0;
        float nearT = __builtin_inff();
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (!((msk >> c) & 1)) continue;
            const float4 lo = bv.nodes[8 * cur + 2 * c];
            const float4 hi = bv.nodes[8 * cur + 2 * c + 1];
            const int cnt = lrt::libm::f2u_i(hi.w);
            if (cnt < 0) continue;
            float tn, tf;
            SlabTestK<kForm>(lo, hi, o, sr, tn, tf);
            const float m = __builtin_fmaf(1e-5f, __builtin_fabsf(tf), mbase);   // a margin: rounding is immaterial
            const float tfm = tf + m;   // (tn <= tf + m, tn <= candL + mb, tf + m >= kMinT)
            if (!(tn <= __builtin_fminf(tfm, candL + mb) && tfm >= kMinT)) continue;
            if (cnt > 0) {
                const int ref = lrt::libm::f2u_i(lo.w);
                for (int j = 0; j < cnt; ++j)
                    if (beats(SphereCand(o, d, bv.lsph[ref + j]), ref + j)) return false;
            } else {
                rem |= 1 << c;
                if (tn < nearT) {
                    nearT = tn;
                    next = c;
                    nextRef = lrt::libm::f2u_i(lo.w);
                }
            }
        }
        if (next >= 0) {
            rem &= ~(1 << next);
            if (rem) StackPush(stk, stride, sp, cur, rem, st);
            cur = nextRef;
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
            if (msk) StackPush(stk, stride, sp, cur, msk, st);
            cur = lrt::libm::f2u_i(bv.nodes[8 * cur + 2 * c].w);
            msk = 0xF;
        }
    }
    return true;
}

LRT_DEV bool ShadowReachesLightBVH4(const F3& o, const F3& d, int li, const float4& lightSph, const BvhView& bv,
                                    unsigned short* stk, int stride, BvhStats* st = nullptr) {
    const float candL = SphereCand(o, d, lightSph);
    if (!(candL < kMaxT)) return false;   // the light is not hit at all (closestT starts at kMaxT)
    const SlabRay sr = MakeSlabRay(o, d, bv);
    if (sr.fma) return ShadowReachesLightBVH4Impl<1>(o, d, li, candL, sr, bv, stk, stride, st);
    return ShadowReachesLightBVH4Impl<2>(o, d, li, candL, sr, bv, stk, stride, st);
}


// Two queries from one origin (the pool kernel's bounce step, lrt_pool.h): first the
// deferred shadow ray of the last scatter's last light (ds, light li, when hasS), then the
// next bounce ray's closest hit (db). Until round 5 they shared ONE loop (a wave ran max over
// lanes of shadow + bounce visits), but each lane's handover then came at its own visit and
// restarted its query divergently; now every shadow query runs first and the handover is
// taken by all those lanes together (ClosestHitDualBVH4).
// The shadow query is the closest-hit query with its bound preset to the light's own
// candidate, (candL, li): a sphere that would replace it is exactly one that beats the
// light, `HitWorld(shadow ray) && hitID == li` is false (parallel.cpp:122-123), and the
// query ends there. Same per-sphere arithmetic, conservative culling and (cand, index)
// order as ClosestHitBVH4 / ShadowReachesLightBVH4, so both answers are bit-identical.
// The traversal is explicit per-lane state (TravQuery) advanced one node visit at a time
// (TravVisit). Shading the lanes whose queries had ended while the others' traversals
// went on (pool-kernel variants) was measured twice and dropped (profiles/r2_p2): with the
// queries in registers across the shading code 82 VGPRs spilled (config 4: 404-829 ms
// instead of 226); with the queries saved to memory between a traversal phase and a
// shading phase still 90 spilled (371-583 ms instead of 224).
// The spheres of all leaf children a lane hits in a node are tested in one loop after the box
// tests (a wave runs max over lanes of their sum), not one loop per child slot inside the
// box-test loop. Leaf positions must fit 12 bits and counts 1..16 (LRT_MAX_SPHERES <= 4096,
// leaves <= 16).
struct TravQuery {
    F3 o, d, db;   // origin, the current query's direction, the bounce ray's direction
    SlabRay sr;    // of d
    float bestT;
    int best;      // the current winner's position in lsph; -2: the light (index li); -1: none
    int li;
    int sp, cur, msk;   // traversal stack depth, node, children still to visit (0: query over)
    bool sh;            // on the shadow query
    bool lit;           // the shadow query's answer, once it is over
};

LRT_DEV void TravTest(TravQuery& q, const BvhView& bv, int pos, const float4& s) {
    const F3 rs = f3(s.x, s.y, s.z) - q.o;                       // maths.cpp:54-59
    const float rsProj = dot(rs, q.d);
    const float ifHit = dot(rs, rs) - rsProj * rsProj - s.w;
    if (ifHit < 0.0f) {
        const float halfCut = sqrt_rn(-ifHit);
        const float t1 = rsProj - halfCut;
        const float t2 = rsProj + halfCut;
        const float cand = t1 > kMinT ? t1 : (t2 > kMinT ? t2 : __builtin_inff());
        if (cand < q.bestT || (cand == q.bestT && q.best != -1 && bv.lid[pos] < (q.best >= 0 ? bv.lid[q.best] : q.li))) {
            q.bestT = cand;
            q.best = pos;
        }
    }
}

// Start the bounce query (d = db): the spheres kept out of the tree first, then the root.
LRT_DEV void TravStartBounce(TravQuery& q, const BvhView& bv) {
    q.sh = false;
    q.d = q.db;
    q.sr = MakeSlabRay(q.o, q.d, bv);
    q.bestT = kMaxT;
    q.best = -1;
    for (int j = 0; j < bv.nbig; ++j) TravTest(q, bv, bv.big0 + j, bv.lsph[bv.big0 + j]);
    q.sp = 0;
    q.cur = 0;
    q.msk = bv.nnodes == 0 ? 0 : 0xF;
}

LRT_DEV void TravInit(TravQuery& q, const F3& o, const F3& db, bool hasS, const F3& ds, int li,
                      const float4& lightSph, const BvhView& bv) {
    q.o = o;
    q.db = db;
    q.li = li;
    q.lit = false;
    const float candL = hasS ? SphereCand(o, ds, lightSph) : kMaxT;
    if (!(candL < kMaxT)) {   // no shadow ray, or the light is not hit at all: not lit
        TravStartBounce(q, bv);
        return;
    }
    q.sh = true;
    q.d = ds;
    q.sr = MakeSlabRay(o, ds, bv);
    q.bestT = candL;
    q.best = -2;
    for (int j = 0; j < bv.nbig; ++j) TravTest(q, bv, bv.big0 + j, bv.lsph[bv.big0 + j]);
    q.sp = 0;
    q.cur = 0;
    q.msk = bv.nnodes == 0 ? 0 : 0xF;
}

// Is the lane's current query over (its stack exhausted, or the light beaten)?
LRT_DEV bool TravOver(const TravQuery& q) { return (q.msk == 0) | (q.sh & (q.best != -2)); }
// One node visit of the lane's current query (not over).
LRT_DEV void TravVisit(TravQuery& q, const BvhView& bv, unsigned short* stk, int stride, BvhStats* st = nullptr) {
    const float mb = bv.margin + q.sr.mo + 1e-5f * q.bestT;
    const float mbase = bv.margin + q.sr.mo;
    int next = -1, rem = 0, nextRef = 0;
    float nearT = __builtin_inff();
    uint32_t lmask = 0, lpack0 = 0, lpack1 = 0;   // the node's leaves this lane hit
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if (!((q.msk >> c) & 1)) continue;
        const float4 lo = bv.nodes[8 * q.cur + 2 * c], hi = bv.nodes[8 * q.cur + 2 * c + 1];
        const int cnt = lrt::libm::f2u_i(hi.w);
        if (cnt < 0) continue;
        float tn, tf;
        SlabTest4(lo, hi, q.o, q.sr, tn, tf);
        const float m = __builtin_fmaf(1e-5f, __builtin_fabsf(tf), mbase);   // a margin
        const float tfm = tf + m;   // (tn <= tf + m, tn <= bestT + mb, tf + m >= kMinT)
        if (!(tn <= __builtin_fminf(tfm, q.bestT + mb) && tfm >= kMinT)) continue;
        if (cnt > 0) {
            const int ref = lrt::libm::f2u_i(lo.w);
            // leaf position (12 bits) and count - 1 (4 bits)
            const uint32_t e = (uint32_t)ref | ((uint32_t)(cnt - 1) << 12);
            if (c < 2) lpack0 |= e << (16 * c);
            else lpack1 |= e << (16 * (c - 2));
            lmask |= 1u << c;
        } else {
            rem |= 1 << c;
            if (tn < nearT) {
                nearT = tn;
                next = c;
                nextRef = lrt::libm::f2u_i(lo.w);
            }
        }
    }
    {   // one loop over the spheres of every leaf this lane hit
        int cs = lmask ? __builtin_ctz(lmask) : 0, jj = 0;
        while (lmask) {
            const uint32_t e = ((cs < 2 ? lpack0 >> (16 * cs) : lpack1 >> (16 * (cs - 2)))) & 0xFFFFu;
            const int pos = (int)(e & 4095u) + jj;
            TravTest(q, bv, pos, bv.lsph[pos]);
            if (++jj > (int)(e >> 12)) {
                lmask &= lmask - 1;
                jj = 0;
                cs = lmask ? __builtin_ctz(lmask) : 0;
            }
        }
    }
    if (next >= 0) {
        rem &= ~(1 << next);
        if (rem) StackPush(stk, stride, q.sp, q.cur, rem, st);
        q.cur = nextRef;
        q.msk = 0xF;
    } else if (q.sp == 0) {
        q.msk = 0;   // this query's traversal is complete
    } else {   // popped children descend without a second box test (as ClosestHitBVH4)
        --q.sp;
        const int e = stk[q.sp * stride];
        int cur = e >> 4, msk = e & 0xF;
        const int c = __builtin_ctz(msk);
        msk &= msk - 1;
        if (msk) StackPush(stk, stride, q.sp, cur, msk, st);
        q.cur = lrt::libm::f2u_i(bv.nodes[8 * cur + 2 * c].w);
        q.msk = 0xF;
    }
}

LRT_DEV int TravResult(const TravQuery& q, const BvhView& bv, float& tOut) {
    tOut = q.bestT;
    return q.best >= 0 ? bv.lid[q.best] : -1;
}

LRT_DEV int ClosestHitDualBVH4(const F3& o, const F3& db, bool hasS, const F3& ds, int li, const float4& lightSph,
                               const BvhView& bv, float& tOut, bool& lit, unsigned short* stk, int stride,
                               BvhStats* st = nullptr) {
    TravQuery q;
    TravInit(q, o, db, hasS, ds, li, lightSph, bv);
    // Every shadow query first, then the lanes that had one start their bounce query together,
    // then every bounce query: each lane's handover at its own node visit ran TravStartBounce
    // (the big spheres, the slab ray) divergently on almost every visit (as the grid's dual
    // walk, lrt_grid.h ClosestHitDualGrid). Same queries, same order per lane: same bits.
    if (q.sh) {
        while (!TravOver(q)) TravVisit(q, bv, stk, stride, st);
        q.lit = q.best == -2;   // nothing beat the light
        TravStartBounce(q, bv);
    }
    while (q.msk != 0) TravVisit(q, bv, stk, stride, st);
    lit = q.lit;
    return TravResult(q, bv, tOut);
}

// ---- packet (wave-coherent) traversal ----------------------------------------------
// For rays that start together and point the same way -- a wave's camera rays (its 64
// lanes are a few adjacent pixels' samples) and the shadow rays from their first hits --
// every active lane walks the SAME node sequence: a child is entered when any lane's box
// test passes (ballot), the near-first order follows the first active lane, and the stack
// is wave-uniform. Node and leaf-sphere data come through scalar loads (one per wave, in
// SGPRs), the loop control is scalar, and no lane waits on another's divergent path.
// Exactness is unchanged: a lane tests every sphere its own conservative culling keeps (a
// superset is harmless -- the (cand, index) minimum over more real spheres is the same),
// with the same per-sphere arithmetic. Device only; the caller checks that every active
// lane has the FMA slab form. kPacketDepth: scatter events below which a path's rays go this
// way (v0: a path's first rays).
constexpr int kPacketDepth = 1;
#if defined(__HIP_DEVICE_COMPILE__)
#define LRT_PACKET_AVAILABLE 1
typedef const __attribute__((address_space(4))) float4* CF4Ptr;
__device__ __forceinline__ int wave_first(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float wave_first(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

__device__ __forceinline__ int ClosestHitPacket(const F3& o, const F3& d, const SlabRay& sr, const BvhView& bv,
                                                float& tOut, unsigned short* stk, int stride) {
    const CF4Ptr nodes = (CF4Ptr)bv.nodes;
    const CF4Ptr lsph = (CF4Ptr)bv.lsph;
    float bestT = kMaxT;
    int best = -1;   // the winner's position in lsph
    auto test = [&](int pos, const float4& s) {
        const F3 rs = f3(s.x, s.y, s.z) - o;                       // maths.cpp:54-59
        const float rsProj = dot(rs, d);
        const float ifHit = dot(rs, rs) - rsProj * rsProj - s.w;
        if (ifHit < 0.0f) {
            const float halfCut = sqrt_rn(-ifHit);
            const float t1 = rsProj - halfCut;
            const float t2 = rsProj + halfCut;
            const float cand = t1 > kMinT ? t1 : (t2 > kMinT ? t2 : __builtin_inff());
            if (cand < bestT || (cand == bestT && best >= 0 && bv.lid[pos] < bv.lid[best])) {
                bestT = cand;
                best = pos;
            }
        }
    };
    for (int j = 0; j < bv.nbig; ++j) test(bv.big0 + j, lsph[bv.big0 + j]);
    int sp = 0, cur = 0, msk = bv.nnodes == 0 ? 0 : 0xF;
    while (msk) {
        const float mb = bv.margin + sr.mo + 1e-5f * bestT;
        const float mbase = bv.margin + sr.mo;
        int next = -1, rem = 0, nextRef = 0;
        float nearT = __builtin_inff();
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (!((msk >> c) & 1)) continue;
            const float4 lo = nodes[8 * cur + 2 * c], hi = nodes[8 * cur + 2 * c + 1];
            const int cnt = lrt::libm::f2u_i(hi.w);
            if (cnt < 0) continue;
            float tn, tf;
            SlabTestFma(lo, hi, sr.inv, sr.oi, tn, tf);
            const float m = __builtin_fmaf(1e-5f, __builtin_fabsf(tf), mbase);
            const float tfm = tf + m;
            const bool hit = tn <= __builtin_fminf(tfm, bestT + mb) && tfm >= kMinT;
            if (__ballot(hit) == 0) continue;
            const int ref = lrt::libm::f2u_i(lo.w);
            if (cnt > 0) {
                if (hit)
                    for (int j = 0; j < cnt; ++j) test(ref + j, lsph[ref + j]);
            } else {
                rem |= 1 << c;
                const float k = wave_first(hit ? tn : __builtin_inff());
                if (next < 0 || k < nearT) {
                    nearT = k;
                    next = c;
                    nextRef = ref;
                }
            }
        }
        if (next >= 0) {
            rem &= ~(1 << next);
            if (rem) {
                stk[sp * stride] = (unsigned short)((cur << 4) | rem);
                ++sp;
            }
            cur = nextRef;
            msk = 0xF;
        } else {
            if (sp == 0) break;
            --sp;
            const int e = wave_first((int)stk[sp * stride]);
            cur = e >> 4;
            msk = e & 0xF;   // re-tested against each lane's shrunk bestT
        }
    }
    tOut = bestT;
    return best >= 0 ? bv.lid[best] : -1;
}

__device__ __forceinline__ bool ShadowPacket(const F3& o, const F3& d, int li, float candL, const SlabRay& sr,
                                             const BvhView& bv, unsigned short* stk, int stride) {
    const CF4Ptr nodes = (CF4Ptr)bv.nodes;
    const CF4Ptr lsph = (CF4Ptr)bv.lsph;
    auto beats = [&](float c, int pos) { return c < candL || (c == candL && bv.lid[pos] < li); };
    bool alive = true;   // no sphere beats the light yet
    for (int j = 0; j < bv.nbig; ++j)
        if (beats(SphereCand(o, d, lsph[bv.big0 + j]), bv.big0 + j)) alive = false;
    const float mb = bv.margin + sr.mo + 1e-5f * candL;
    const float mbase = bv.margin + sr.mo;
    int sp = 0, cur = 0, msk = bv.nnodes == 0 ? 0 : 0xF;
    while (msk && __ballot(alive) != 0) {
        int next = -1, rem = 0, nextRef = 0;
        float nearT = __builtin_inff();
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (!((msk >> c) & 1)) continue;
            const float4 lo = nodes[8 * cur + 2 * c], hi = nodes[8 * cur + 2 * c + 1];
            const int cnt = lrt::libm::f2u_i(hi.w);
            if (cnt < 0) continue;
            float tn, tf;
            SlabTestFma(lo, hi, sr.inv, sr.oi, tn, tf);
            const float m = __builtin_fmaf(1e-5f, __builtin_fabsf(tf), mbase);
            const float tfm = tf + m;
            const bool hit = alive && tn <= __builtin_fminf(tfm, candL + mb) && tfm >= kMinT;
            if (__ballot(hit) == 0) continue;
            const int ref = lrt::libm::f2u_i(lo.w);
            if (cnt > 0) {
                if (hit)
                    for (int j = 0; j < cnt; ++j)
                        if (beats(SphereCand(o, d, lsph[ref + j]), ref + j)) alive = false;
            } else {
                rem |= 1 << c;
                const float k = wave_first(hit ? tn : __builtin_inff());
                if (next < 0 || k < nearT) {
                    nearT = k;
                    next = c;
                    nextRef = ref;
                }
            }
        }
        if (next >= 0) {
            rem &= ~(1 << next);
            if (rem) {
                stk[sp * stride] = (unsigned short)((cur << 4) | rem);
                ++sp;
            }
            cur = nextRef;
            msk = 0xF;
        } else {
            if (sp == 0) break;
            --sp;
            const int e = wave_first((int)stk[sp * stride]);
            cur = e >> 4;
            msk = e & 0xF;   // re-tested: lanes blocked since no longer count
        }
    }
    return alive;
}
#else
#define LRT_PACKET_AVAILABLE 0
#endif

// The 4-wide layout the host built (build_bvh_host). coherent: the
// caller's active lanes are rays that start together (packet traversal when every one of
// them takes the FMA slab form).
LRT_DEV int ClosestHitBVH(const F3& o, const F3& d, const BvhView& bv, float& tOut, unsigned short* stk, int stride,
                          BvhStats* st = nullptr, bool coherent = false) {
#if LRT_PACKET_AVAILABLE
    if (coherent) {
        const SlabRay sr = MakeSlabRay(o, d, bv);
        if (__ballot(!sr.fma) == 0) return ClosestHitPacket(o, d, sr, bv, tOut, stk, stride);
    }
#endif
    (void)coherent;
    return ClosestHitBVH4(o, d, bv, tOut, stk, stride, st);
}
LRT_DEV bool ShadowReachesLightBVH(const F3& o, const F3& d, int li, const float4& lightSph, const BvhView& bv,
                                   unsigned short* stk, int stride, bool coherent = false, BvhStats* st = nullptr) {
#if LRT_PACKET_AVAILABLE
    if (coherent) {
        const float candL = SphereCand(o, d, lightSph);
        const SlabRay sr = MakeSlabRay(o, d, bv);
        if (__ballot(!sr.fma) == 0) return candL < kMaxT && ShadowPacket(o, d, li, candL, sr, bv, stk, stride);
    }
#endif
    (void)coherent;
    return ShadowReachesLightBVH4(o, d, li, lightSph, bv, stk, stride, st);
}

}  // namespace lrt
