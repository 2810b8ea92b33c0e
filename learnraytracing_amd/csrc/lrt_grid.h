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
// sphere not yet tested has cand > the exit >= best and can neither win nor tie. The "hit
// point lies in its box" needs the reference's own rounding: HitSphere's cancellation puts a
// computed hit point up to hit_excursion(D, r) off the sphere (lrt_grid_build.h), growing with
// the origin's distance D, so each sphere's padding covers it up to a distance the padding was
// sized for, and rays from farther away are decided after their walk (GridCertain; DESIGN
// §4.3). No stack: the walk's state is a cell and three plane times, so the traversal holds
// fewer registers than the BVH's and no LDS.
//
// Walk and sphere tests share ONE loop (GridIter): an iteration advances to the next cell
// when the current cell's list is used up, then tests one sphere. A wave therefore runs max
// over lanes of (cells + spheres) iterations, not the sum of per-cell maxima.
#pragma once

namespace lrt {

// Exactness reach (lrt_grid_build.h): an origin within sqrt(f2near) of every corner
// of the grid's box: the walk alone is exact; otherwise, with dot(o, o) <= o2dda, the walk is
// exact up to tsafe from o, and a ray whose candidates could lie farther (GridFarClear) scans
// every sphere at the end unless its answer came first; beyond (or NaN): the scan. (The host's
// record; the view carries the values.)
struct GridReach {
    float o2dda;
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
    float f2near;            // an origin this close (squared) to every corner of the box is near
    float o2dda, tsafe, conea;   // the rest of the exactness reach (GridReach)
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
    bool sh, lit;
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
LRT_DEV bool GridFarClear(const F3& o, const F3& d, const GridView& g, float hix, float hiy, float hiz) {
    const float a = g.conea, b = kConeB, t = g.tsafe;
    // per axis: moving away from the far side at |d| - b >= 0 and beyond it at tsafe
    auto away = [&](float o, float d, float lo, float hi) {
        const float m = d > 0.0f ? o - hi : lo - o;
        const float e = __builtin_fabsf(d) - b;
        return (e >= 0.0f) & (m - a + t * e > 0.0f);
    };
    return away(o.x, d.x, g.lox, hix) | away(o.y, d.y, g.loy, hiy) | away(o.z, d.z, g.loz, hiz);
}

// Is o within sqrt(f2near) of every corner of the grid's box, which holds every walked
// sphere's centre (then every candidate's |c - o| + r stays within the distance the padding
// serves)? False for NaN.
LRT_DEV bool GridNear(const F3& o, const GridView& g, float hix, float hiy, float hiz) {
    const float fx = __builtin_fmaxf(__builtin_fabsf(o.x - g.lox), __builtin_fabsf(o.x - hix));
    const float fy = __builtin_fmaxf(__builtin_fabsf(o.y - g.loy), __builtin_fabsf(o.y - hiy));
    const float fz = __builtin_fmaxf(__builtin_fabsf(o.z - g.loz), __builtin_fabsf(o.z - hiz));
    return fx * fx + fy * fy + fz * fz <= g.f2near;
}

// After q's walk (mode 2): is its answer the reference's? Always when the origin is near the
// spheres; else (the DDA's reach, o2dda, given) when the answer came before tsafe -- the walk
// finds every candidate up to there -- or when no candidate can lie beyond tsafe (GridFarClear).
// Decided after the walk's loop from the query's own origin and direction, so that the loop
// carries none of it (a check and a scan in the loop cost config 4 ~10 %, profiles/r5_e).
LRT_DEV bool GridCertain(const F3& o, const F3& d, float bestT, const GridView& g) {
    const float hix = GridPlane(g.lox, g.nx, g.hx), hiy = GridPlane(g.loy, g.ny, g.hy),
                hiz = GridPlane(g.loz, g.nz, g.hz);
    if ((g.count == 0) | (g.nx == 0) || GridNear(o, g, hix, hiy, hiz)) return true;
    return (int)(dot(o, o) <= g.o2dda) & ((int)(bestT < g.tsafe) | (int)GridFarClear(o, d, g, hix, hiy, hiz));
}
// The reference's own scan over the whole scene in index order, from the query's (bestT, best):
// the spheres tested already again (an equal (cand, id) changes nothing, and a shadow query's
// light is no win over its own bar).
LRT_DEV void GridScanAll(GridQuery& q, const GridView& g, GridStats* st) {
    if (st) {
        st->fallback += 1;
        st->spheres += g.count;
    }
    for (int k = 0; k < g.count; ++k) GridTest(q, g.all[k], k);
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
    if (g.count == 0 || g.nx == 0) return;
    // Exactness needs the DDA's rounding (2^-18 (max|o| + tEnter + ext) <= 2^-16 (max|o| + ext);
    // tEnter is at most sqrt(3) (max|o| + ext)) plus how far off its sphere the reference's own
    // hit point can be (hit_excursion, growing with |c - o|) to stay inside the padding: true for
    // every candidate when the origin is near the spheres (GridNear), for those up to tsafe
    // when |o| is within o2dda (GridCertain then checks the rest), for none beyond: a huge origin,
    // NaN or inf scans every sphere (GridCertain). Decided before the box test: its rounding
    // grows with |o| too.
    const float hix = GridPlane(g.lox, g.nx, g.hx), hiy = GridPlane(g.loy, g.ny, g.hy),
                hiz = GridPlane(g.loz, g.nz, g.hz);
    // near: from registers; the rest (few lanes) from memory (grid_reach: a scalar load, whose
    // wait would also wait for the walk's LDS reads -- read at every query start it cost config
    // 4 ~15 %)
    // (origins too far for the DDA, NaN, inf: no walk; GridCertain sends them to the scan)
    if ((int)!GridNear(q.o, g, hix, hiy, hiz) & (int)!(dot(q.o, q.o) <= g.o2dda)) return;
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
    while (q.mode != 2) GridIter(q, g, st);
    if (!GridCertain(o, d, q.bestT, g)) GridScanAll(q, g, st);
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
    // the bar is candL from the start (only the walk's own finds lower it), so whether the walk's
    // answer will be certain is known before it: if not, the scan instead. (GridCertain without
    // its cone test: in the pool kernel this is the other lights' shadow query inside Scatter,
    // where the cone test's registers added ~30 B of spills per lane to the whole kernel.)
    if ((int)!GridNear(o, g, GridPlane(g.lox, g.nx, g.hx), GridPlane(g.loy, g.ny, g.hy), GridPlane(g.loz, g.nz, g.hz)) &
        (int)!((int)(dot(o, o) <= g.o2dda) & (int)(candL < g.tsafe))) {
        GridScanAll(q, g, st);
        return q.best == -2;
    }
    GridStart(q, g, st);
    while ((q.mode != 2) & (q.best == -2)) GridIter(q, g, st);
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
    const float candL = hasS ? GridCand(o, ds, lightSph) : kMaxT;
    q.sh = candL < kMaxT;   // no shadow ray, or the light is not hit at all: not lit
    // A shadow query the walk cannot answer for certain (GridCertain: its bar is candL, which
    // only the walk's own finds could lower) is answered here by the scan, before the loop.
    if (q.sh && !GridCertain(o, ds, candL, g)) {
        GridQuery s;
        s.o = o;
        s.d = ds;
        s.bestT = candL;
        s.best = -2;
        s.li = li;
        GridScanAll(s, g, st);
        q.lit = s.best == -2;
        q.sh = false;
    }
    q.d = q.sh ? ds : db;
    q.bestT = q.sh ? candL : kMaxT;
    q.best = q.sh ? -2 : -1;
    GridStart<kL>(q, g, st);
}
template <int kL = 0>
LRT_DEV int ClosestHitDualGrid(const F3& o, const F3& db, bool hasS, const F3& ds, int li, const float4& lightSph,
                               const GridView& g, float& tOut, bool& lit, GridStats* st = nullptr) {
    GridQuery q;
    GridDualInit<kL>(q, o, db, hasS, ds, li, lightSph, g, st);
    // Every shadow walk first (to its end: the light reached, or a sphere before it), then the
    // lanes that had one start their bounce walk TOGETHER, then every bounce walk. Round 4 ran
    // both in one loop -- a wave took max over lanes of (shadow + bounce) iterations instead of
    // max(shadow) + max(bounce) -- but each lane's switch from its shadow to its bounce query came
    // at its own iteration, so GridStart (the big spheres, the slab test, the entry cell: the
    // longest block of the walk) ran divergently on almost every iteration. Config 4: 112.7-113.2
    // -> 83.7-83.9 ms/step (profiles/r5_r). The same queries in the same order per lane: the bits
    // are unchanged.
    // (two iterations per trip of each loop: half the loop's exit tests and branches; an
    // iteration on a finished query does nothing. Config 4: 84.0 -> 83.3 ms, profiles/r5_v)
    if (q.sh) {
        while ((q.mode != 2) & (q.best == -2)) {
            GridIter<kL>(q, g, st);
            if (q.best == -2) GridIter<kL>(q, g, st);
        }
        q.lit = q.best == -2;   // nothing beat the light
        q.sh = false;
        q.d = q.db;
        q.bestT = kMaxT;
        q.best = -1;
        GridStart<kL>(q, g, st);
    }
    while (q.mode != 2) {
        GridIter<kL>(q, g, st);
        GridIter<kL>(q, g, st);
    }
    // after the loop (GridCertain), from the values the loop keeps anyway (q.d is the bounce's)
    if (!GridCertain(q.o, q.d, q.bestT, g)) GridScanAll(q, g, st);
    lit = q.lit;
    tOut = q.bestT;
    return q.best;
}

}  // namespace lrt
