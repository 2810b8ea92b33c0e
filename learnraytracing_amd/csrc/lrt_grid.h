// Bit-exact uniform-grid closest hit (BASELINE configs 4-5).
//
// The same exactness argument as the BVH (lrt_bvh.h): for sphere i the reference's HitSphere
// arithmetic gives a candidate cand_i (first root if > tMin, else the second, else +inf)
// independent of closestT, and HitWorld's scan (parallel.cpp:54-73, maths.cpp:51-94) returns
// the lexicographic minimum of (cand_i, i). Any traversal that evaluates the same per-sphere
// arithmetic for every sphere that could win and keeps that minimum returns the same bits.
//
// The grid: a box over the scene's spheres split into n.x * n.y * n.z cells; each sphere is
// listed in every cell its bounding box, padded by `pad`, overlaps (CSR: cells[c] ..
// cells[c + 1] index cell-ordered copies of the spheres and their original indices). Spheres
// that would make the box or the cells large (the r = 100 ground, the light above the
// others) are tested first by every ray instead, as the BVH does with its `big` spheres.
// A ray walks the cells it crosses in order (3D DDA, Amanatides & Woo) from where it enters
// the box. The walk stops once the best candidate lies before the exit of the current cell:
// every ray point up to that exit lies within the DDA's rounding error of a visited cell, a
// sphere's hit point lies in its box, and the box was padded by more than that error -- so a
// sphere not yet tested has cand > the exit >= best and can neither win nor tie. Rays whose
// rounding bound (from |origin| and the box's extent) exceeds the padding's share scan every
// sphere instead (origins more than ~8 scene sizes away). No stack: the walk's state is a
// cell and three plane times, so the traversal holds fewer registers than the BVH's and no LDS.
//
// Walk and sphere tests share ONE loop (GridIter): an iteration advances to the next cell
// when the current cell's list is used up, then tests one sphere. A wave therefore runs max
// over lanes of (cells + spheres) iterations, not the sum of per-cell maxima.
#pragma once

namespace lrt {

// Exactness reach (lrt_grid_build.h): an origin within sqrt(f2near) of every corner
// of the grid's box: the walk alone is exact; otherwise, with dot(o, o) <= o2dda, the walk is
// exact up to tsafe from o, and a ray whose candidates could lie farther (GridFarClear) scans
// every sphere at the end unless its answer came first; beyond (or NaN): the scan. In memory,
// not in the view: read at each use (grid_reach), the values hold no registers across the walk
// (held in the view they added ~30 B of spills per lane to the pool kernel's grid instance).
struct GridReach {
    float f2near, o2dda;
    float tsafe;   // the walk finds every candidate up to tsafe from such an origin
    float conea;   // a reference hit point at t lies within conea + kConeB t of the box (plus
                   // GridFarClear's rounding slack)
    float lo[3], hi[3];   // the grid's box, as GridPlane gives it
};

struct GridView {
    const uint2* cells;      // per cell: [start, end) of its spheres in rsph / rid
    const float4* rsph;      // cell-ordered sphere copies: float4(center, r^2)
    const int* rid;          // their original indices
    const float4* bsph;      // spheres every ray tests first
    const int* bid;
    const float4* all;       // the scene in index order (the fallback scan)
    int nbig, count;
    int nx, ny, nz;
    float lox, loy, loz;     // the box's low corner
    float hx, hy, hz;        // cell size per axis
    float ihx, ihy, ihz;     // 1 / cell size
    float pad;               // insertion padding (absolute)
    const struct GridReach* reach;   // exactness reach (GridReach), read where used
    float ext;               // max |coordinate| of the box
    int on;
    unsigned cells_refs;     // entries of rsph / rid (the LDS copy's size, kPoolGridWaves blocks)
};

// The walk's reads of the cell ranges and the cell-ordered spheres. kL = 1: the pool kernel's
// block-shared LDS copy (kPoolGridWaves blocks): the view's pointers are generic addresses of
// that copy, read here as LDS (ds_read instead of flat loads). Any other reader of the same
// view (the other lights' shadow queries) goes through the generic pointers.
template <class T>
LRT_DEV T grid_ld(const T* p, unsigned i, std::integral_constant<int, 1>) {
#if defined(__HIP_DEVICE_COMPILE__)
    return ((const __attribute__((address_space(3))) T*)p)[i];
#else
    return p[i];   // (the host pass only parses the kernels)
#endif
}
template <class T>
LRT_DEV T grid_ld(const T* p, unsigned i, std::integral_constant<int, 0>) { return p[i]; }
#define LRT_GRID_LD(kL, p, i) grid_ld((p), (unsigned)(i), std::integral_constant<int, (kL)>())

// Host diagnostics (lrt_grid_stats): cell steps, sphere tests and fallback scans.
struct GridStats { int cells = 0, spheres = 0, fallback = 0; };

// One query's walk. best: the winner's original index; -1 none; -2 the light (shadow query).
struct GridQuery {
    F3 o, d, db;      // origin, this query's direction, the bounce query's direction (dual)
    F3 inv;           // 1 / d
    float tnx, tny, tnz;   // each axis' next plane crossing
    float bestT;
    int best, li;
    int cx, cy, cz;   // current cell
    unsigned j, jend; // the current cell's sphere range still to test
    int mode;         // 0 walking, 2 this query is over
    bool sh, lit, busy;
    bool far;         // the walk's answer is certain only up to tsafe (GridStart, GridFinish)
};

LRT_DEV float GridPlane(float lo, int c, float h) { return lo + (float)c * h; }

// (cand, index) order: does sphere `id` with candidate cand beat the query's best?
LRT_DEV bool GridBeats(const GridQuery& q, float cand, int id) {
    return (cand < q.bestT) | ((cand == q.bestT) & (q.best != -1) & (id < (q.best >= 0 ? q.best : q.li)));
}
LRT_DEV float GridCand(const F3& o, const F3& d, const float4& s) {   // maths.cpp:54-90
    const F3 rs = f3(s.x, s.y, s.z) - o;
    const float rsProj = dot(rs, d);
    const float ifHit = dot(rs, rs) - rsProj * rsProj - s.w;
    if (!(ifHit < 0.0f)) return __builtin_inff();
    const float halfCut = sqrt_rn(-ifHit);
    const float t1 = rsProj - halfCut;
    const float t2 = rsProj + halfCut;
    return t1 > kMinT ? t1 : (t2 > kMinT ? t2 : __builtin_inff());
}
LRT_DEV void GridTest(GridQuery& q, const float4& s, int id, bool on = true) {   // on: test at all
    const float cand = GridCand(q.o, q.d, s);
    const bool w = on & GridBeats(q, cand, id);   // selects, not a region
    q.bestT = w ? cand : q.bestT;
    q.best = w ? id : q.best;
}

LRT_DEV GridReach grid_reach(const GridView& g) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) GridReach* P;   // (uniform: scalar loads)
    const unsigned long long v = (unsigned long long)g.reach;
    unsigned long long u = ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(v >> 32)) << 32) |
                           (unsigned)__builtin_amdgcn_readfirstlane((unsigned)v);
    asm volatile("" : "+s"(u));   // loaded here, each time: not hoisted into the loop's registers
    return *(P)u;
#else
    return *g.reach;
#endif
}

// hit_excursion(D) <= c1 D (c1 = 2^-9.5 + 24 2^-24) with D <= 1.004 t + 3.02 rmax: the cone's
// slope, 1.004 c1 (1 + 2^-10) (lrt_grid_build.h checks it)
constexpr float kConeB = 0.00139f;

// For a ray from beyond the grid's near reach (but within o2dda) the walk finds every
// candidate up to tsafe (the padding is sized for them, lrt_grid_build.h). A candidate beyond
// lies within conea + kConeB t of the grid's box (conea also holds the rounding slack of the
// test below): a cone around the box. Is the ray outside it for every t >= tsafe? It is when,
// on some axis, it is beyond the cone's slab at tsafe and moves away from it at least as fast
// as the slab widens. No division, few registers (this runs in the pool kernel's loop, where
// the walk's state is live: the exact cone interval, 6 reciprocals, added ~56 B of spills).
LRT_DEV bool GridFarClear(const GridQuery& q, const GridView& g, const GridReach& R) {
    const float a = R.conea, b = kConeB, t = R.tsafe;
    // per axis: moving away from the far side at |d| - b >= 0 and beyond it at tsafe
    auto away = [&](float o, float d, float lo, float hi) {
        const float m = d > 0.0f ? o - hi : lo - o;
        const float e = __builtin_fabsf(d) - b;
        return (e >= 0.0f) & (m - a + t * e > 0.0f);
    };
    (void)g;
    return away(q.o.x, q.d.x, R.lo[0], R.hi[0]) | away(q.o.y, q.d.y, R.lo[1], R.hi[1]) | away(q.o.z, q.d.z, R.lo[2], R.hi[2]);
}

// Is o within sqrt(f2near) of every corner of the grid's box, which holds every walked
// sphere's centre (then every candidate's |c - o| + r stays within the distance the padding
// serves)? False for NaN.
LRT_DEV bool GridNear(const F3& o, const GridView& g) {
    const GridReach R = grid_reach(g);
    const float fx = __builtin_fmaxf(__builtin_fabsf(o.x - R.lo[0]), __builtin_fabsf(o.x - R.hi[0]));
    const float fy = __builtin_fmaxf(__builtin_fabsf(o.y - R.lo[1]), __builtin_fabsf(o.y - R.hi[1]));
    const float fz = __builtin_fmaxf(__builtin_fabsf(o.z - R.lo[2]), __builtin_fabsf(o.z - R.hi[2]));
    return fx * fx + fy * fy + fz * fz <= R.f2near;
}

// The query as a scan of every sphere, through the walk's own loop: the cell-ordered list as
// one range, which holds every walked sphere at least once (the first-tested ones were tested
// already; a sphere tested twice, or a shadow query's light against its own bar, changes
// nothing), ended by the walk's NaN exit (plane times NaN); cx = -2 marks it, so that its end
// is final. The loop itself is unchanged (r4_x: a scan there, with its pointer and index
// selects, cost ~20 scalar instructions and a vmcnt(0) wait per iteration).
LRT_DEV void GridScan(GridQuery& q, const GridView& g, GridStats* st) {
    if (st) st->fallback += 1;
    q.j = 0;
    q.jend = g.cells_refs;
    q.tnx = q.tny = q.tnz = __builtin_nanf("");
    q.cx = -2;
    q.mode = 0;
}
// The end of q's walk (mode 2): is its answer certain? Not when the origin is away from the
// spheres and its candidates could lie beyond tsafe (q.far, GridStart) and nothing closer than
// tsafe answered: then the query goes on as the scan (returns true).
LRT_DEV bool GridFinish(GridQuery& q, const GridView& g, GridStats* st) {
    if (!(q.far & (q.cx != -2)) || q.bestT < grid_reach(g).tsafe) return false;
    GridScan(q, g, st);
    return true;
}

// Starts q's walk along q.d (q.bestT / q.best / q.li set by the caller): the big spheres,
// then the cell where the ray enters the box.
template <int kL = 0>
LRT_DEV void GridStart(GridQuery& q, const GridView& g, GridStats* st = nullptr) {
    // (a shadow query skips its own light: the light's candidate IS the bar, and a tie with the
    // same index changes nothing -- GridBeats is false for it)
    for (int k = 0; k < g.nbig; ++k) GridTest(q, g.bsph[k], g.bid[k], (q.best != -2) | (g.bid[k] != q.li));
    q.inv = f3(rcp_rn(q.d.x), rcp_rn(q.d.y), rcp_rn(q.d.z));
    q.mode = 2;
    q.cx = 0;   // (not the scan's mark, GridScan)
    q.far = false;
    if (g.count == 0 || g.nx == 0) return;
    // Exactness needs the DDA's rounding (2^-18 (max|o| + tEnter + ext) <= 2^-16 (max|o| + ext);
    // tEnter is at most sqrt(3) (max|o| + ext)) plus how far off its sphere the reference's own
    // hit point can be (hit_excursion, growing with |c - o|) to stay inside the padding: true for
    // every candidate when the origin is near the spheres (GridNear), for those up to tsafe
    // when |o| is within o2dda (GridFinish then checks the rest), for none beyond: a huge origin,
    // NaN or inf scans every sphere (GridFinish). Decided before the box test: its rounding
    // grows with |o| too.
    if (!GridNear(q.o, g)) {   // (rare: origins away from the spheres)
        const GridReach R = grid_reach(g);
        if (!(dot(q.o, q.o) <= R.o2dda)) {   // too far for the DDA (or NaN, inf): the scan at once
            GridScan(q, g, st);
            return;
        }
        q.far = !GridFarClear(q, g, R);   // decided here, where the walk's state is not live yet
    }
    const float hix = GridPlane(g.lox, g.nx, g.hx), hiy = GridPlane(g.loy, g.ny, g.hy),
                hiz = GridPlane(g.loz, g.nz, g.hz);
    // the box's slab interval; an axis the ray does not move along constrains through o
    float t0 = 0.0f, t1 = __builtin_inff();
    auto slab = [&](float o, float d, float inv, float lo, float hi) {   // (selects: no region per axis)
        const bool flat = d == 0.0f;
        const float a = (lo - o) * inv, b = (hi - o) * inv;   // (inv = +-inf when flat: unused)
        t0 = flat ? t0 : __builtin_fmaxf(t0, __builtin_fminf(a, b));
        t1 = flat ? (((o < lo) | (o > hi)) ? -1.0f : t1) : __builtin_fminf(t1, __builtin_fmaxf(a, b));
    };
    slab(q.o.x, q.d.x, q.inv.x, g.lox, hix);
    slab(q.o.y, q.d.y, q.inv.y, g.loy, hiy);
    slab(q.o.z, q.d.z, q.inv.z, g.loz, hiz);
    const float slack = g.pad + 1e-5f * t1;
    if ((t0 > t1 + slack) | (q.bestT < t0 - g.pad - 1e-5f * t0)) return;   // misses the box, or beaten before it
    const F3 p = q.o + q.d * t0;
    auto cell = [](float p, float lo, float ih, int n) {
        const float f = (p - lo) * ih;
        int c = f >= 0.0f ? (int)f : 0;
        return c < n ? c : n - 1;
    };
    q.cx = cell(p.x, g.lox, g.ihx, g.nx);
    q.cy = cell(p.y, g.loy, g.ihy, g.ny);
    q.cz = cell(p.z, g.loz, g.ihz, g.nz);
    q.tnx = q.d.x > 0.0f ? (GridPlane(g.lox, q.cx + 1, g.hx) - q.o.x) * q.inv.x
            : q.d.x < 0.0f ? (GridPlane(g.lox, q.cx, g.hx) - q.o.x) * q.inv.x : __builtin_inff();
    q.tny = q.d.y > 0.0f ? (GridPlane(g.loy, q.cy + 1, g.hy) - q.o.y) * q.inv.y
            : q.d.y < 0.0f ? (GridPlane(g.loy, q.cy, g.hy) - q.o.y) * q.inv.y : __builtin_inff();
    q.tnz = q.d.z > 0.0f ? (GridPlane(g.loz, q.cz + 1, g.hz) - q.o.z) * q.inv.z
            : q.d.z < 0.0f ? (GridPlane(g.loz, q.cz, g.hz) - q.o.z) * q.inv.z : __builtin_inff();
    const uint2 cr = LRT_GRID_LD(kL, g.cells, (q.cz * g.ny + q.cy) * g.nx + q.cx);
    q.j = cr.x;
    q.jend = cr.y;
    q.mode = 0;
    if (st) st->cells += 1;
}

// One iteration of q's query: the next cell if the current one is used up (or the end of the
// walk), then one sphere test. The step is straight-line code: the axis with the nearest
// plane (x, then y, then z on ties) is selected rather than branched on, so a wave whose
// lanes step along different axes issues one sequence, not three.
template <int kL>
LRT_DEV void GridAdvance(GridQuery& q, const GridView& g, GridStats* st) {
    if ((q.mode != 0) | (q.j < q.jend)) return;
    const float T = __builtin_fminf(__builtin_fminf(q.tnx, q.tny), q.tnz);
    const bool ax = q.tnx == T, ay = !ax & (q.tny == T), az = !ax & !ay;
    // each axis updates itself under its own condition (a select between an axis's new and old
    // value; selecting between fields instead turned into pointer selects, and the query into
    // scratch memory)
    const int ux = q.inv.x > 0.0f ? 1 : 0, uy = q.inv.y > 0.0f ? 1 : 0, uz = q.inv.z > 0.0f ? 1 : 0;
    q.cx += ax ? 2 * ux - 1 : 0;
    q.cy += ay ? 2 * uy - 1 : 0;
    q.cz += az ? 2 * uz - 1 : 0;
    // the walk ends when nothing beyond this cell can win or tie (or T is NaN: nowhere to go),
    // or when it leaves the box -- one exit, the conditions combined bitwise
    if ((q.bestT < T - (g.pad + 1e-5f * T)) | !(T == T) | ((unsigned)q.cx >= (unsigned)g.nx) |
        ((unsigned)q.cy >= (unsigned)g.ny) | ((unsigned)q.cz >= (unsigned)g.nz)) {
        q.mode = 2;
        return;
    }
    // the stepped axis' next plane, the same expression GridStart uses
    q.tnx = ax ? (GridPlane(g.lox, q.cx + ux, g.hx) - q.o.x) * q.inv.x : q.tnx;
    q.tny = ay ? (GridPlane(g.loy, q.cy + uy, g.hy) - q.o.y) * q.inv.y : q.tny;
    q.tnz = az ? (GridPlane(g.loz, q.cz + uz, g.hz) - q.o.z) * q.inv.z : q.tnz;
    const uint2 cr = LRT_GRID_LD(kL, g.cells, (q.cz * g.ny + q.cy) * g.nx + q.cx);   // one 8-byte load per cell
    q.j = cr.x;
    q.jend = cr.y;
    if (st) st->cells += 1;
}
// (The fallback scan for far origins runs in GridStart, outside the loop.)
template <int kL = 0>
LRT_DEV void GridIter(GridQuery& q, const GridView& g, GridStats* st) {
    GridAdvance<kL>(q, g, st);
    if (q.mode == 0 && q.j < q.jend) {
        if (st) st->spheres += 1;
        const unsigned j = q.j++;
        const float4 s = LRT_GRID_LD(kL, g.rsph, j);
        const float cand = GridCand(q.o, q.d, s);
        // the original index is read only when it can matter (a win or an exact tie); then
        // GridBeats reduces to (closer, or the lower index of a tie). Bitwise, not short-circuit:
        // each && / || here was a divergent region of its own (exec bookkeeping per iteration).
        const bool closer = cand < q.bestT;
        if (closer | ((cand == q.bestT) & (q.best != -1))) {
            const int id = LRT_GRID_LD(kL, g.rid, j);
            const bool win = closer | (id < (q.best >= 0 ? q.best : q.li));
            q.bestT = win ? cand : q.bestT;
            q.best = win ? id : q.best;
        }
    }
}

LRT_DEV int ClosestHitGrid(const F3& o, const F3& d, const GridView& g, float& tOut, GridStats* st = nullptr) {
    GridQuery q;
    q.o = o;
    q.d = d;
    q.bestT = kMaxT;
    q.best = -1;
    q.li = -1;
    GridStart(q, g, st);
    do {
        while (q.mode != 2) GridIter(q, g, st);
    } while (GridFinish(q, g, st));
    tOut = q.bestT;
    return q.best;
}

// `HitWorld(shadow ray) && hitID == li` (parallel.cpp:122-123): the closest-hit query with the
// light's own (cand, li) as the bar from the start; the first sphere that beats it ends it.
LRT_DEV bool ShadowReachesLightGrid(const F3& o, const F3& d, int li, const float4& lightSph, const GridView& g,
                                    GridStats* st = nullptr) {
    const float candL = GridCand(o, d, lightSph);
    if (!(candL < kMaxT)) return false;
    GridQuery q;
    q.o = o;
    q.d = d;
    q.bestT = candL;
    q.best = -2;
    q.li = li;
    GridStart(q, g, st);
    do {   // (a sphere that beat the light is an answer already)
        while ((q.mode != 2) & (q.best == -2)) GridIter(q, g, st);
    } while ((q.best == -2) && GridFinish(q, g, st));
    return q.best == -2;
}

// The pool kernel's two queries from one origin in one loop (as ClosestHitDualBVH4): the
// deferred shadow ray of the last light (when hasS), then the bounce ray's closest hit.
template <int kL = 0>
LRT_DEV void GridDualInit(GridQuery& q, const F3& o, const F3& db, bool hasS, const F3& ds, int li,
                          const float4& lightSph, const GridView& g, GridStats* st) {
    q.o = o;
    q.db = db;
    q.li = li;
    q.lit = false;
    q.busy = true;
    const float candL = hasS ? GridCand(o, ds, lightSph) : kMaxT;
    q.sh = candL < kMaxT;   // no shadow ray, or the light is not hit at all: not lit
    q.d = q.sh ? ds : db;
    q.bestT = q.sh ? candL : kMaxT;
    q.best = q.sh ? -2 : -1;
    GridStart<kL>(q, g, st);
}
template <int kL = 0>
LRT_DEV void GridDualStep(GridQuery& q, const GridView& g, GridStats* st) {
    GridIter<kL>(q, g, st);
    const bool qdone = (q.mode == 2) | (q.sh & (q.best != -2));
    if (qdone && !((!q.sh | (q.best == -2)) && GridFinish(q, g, st))) {
        if (q.sh) {
            q.lit = q.best == -2;   // nothing beat the light
            q.sh = false;
            q.d = q.db;
            q.bestT = kMaxT;
            q.best = -1;
            GridStart<kL>(q, g, st);
        } else {
            q.busy = false;
        }
    }
}
template <int kL = 0>
LRT_DEV int ClosestHitDualGrid(const F3& o, const F3& db, bool hasS, const F3& ds, int li, const float4& lightSph,
                               const GridView& g, float& tOut, bool& lit, GridStats* st = nullptr) {
    GridQuery q;
    GridDualInit<kL>(q, o, db, hasS, ds, li, lightSph, g, st);
    while (q.busy) GridDualStep<kL>(q, g, st);
    lit = q.lit;
    tOut = q.bestT;
    return q.best;
}

}  // namespace lrt
