// Host build of the uniform grid (lrt_grid.h): box, resolution, the spheres every ray tests
// first, and the cell lists. Also the policy that decides whether a scene gets the grid or
// the BVH (grid_suitable).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "lrt.h"
#include "lrt_trace.h"

namespace lrt {

// ---- How far from its sphere the reference's hit point can lie ------------
// HitSphere (maths.cpp:54-59) forms ifHit = dot(rs,rs) - rsProj^2 - r^2 (rs = c - o) by
// cancellation. For a near-tangent ray its rounding, ~ulp(|rs|^2), can turn a miss into a
// "hit", or move a hit, off the sphere: with D >= |c - o| + r, the point X = o + cand * d of
// the candidate the reference computes satisfies |X - c| <= r + hit_excursion(D, r). (Forward
// error analysis over the seven roundings of ifHit, rsProj and the roots and |d|^2 = 1 +- 12
// eps of a normalised direction: |X - c|^2 <= (sqrt(r^2 + E) + f)^2 with E <= 30 eps D^2,
// f <= 16 eps D; a brute-force search over near-tangent rays reaches 0.55 of it.) Small r:
// ~1.4e-3 D; large r: ~E / 2r. The grid's padding and the BVH's boxes must cover it for every
// ray they serve (the r4 verdict's mismatches: origins 40-400 units away).
inline double hit_excursion(double D, double r) {
    const double E = std::ldexp(D * D, -19);   // 32 eps D^2
    return E / (std::sqrt(r * r + E) + r) + std::ldexp(24.0 * D, -24);
}
// Over the spheres `ids` of s: rs = max |c| + max r (so |c - o| + r <= |o| + rs for each),
// rmin = min r.
inline void sphere_reach(const lrt_sphere* s, const std::vector<int>& ids, double& rs, double& rmin) {
    double cmax = 0.0, rmax = 0.0;
    rmin = INFINITY;
    for (int i : ids) {
        const double x = s[i].center.x, y = s[i].center.y, z = s[i].center.z, r = std::fabs((double)s[i].radius);
        cmax = std::max(cmax, std::sqrt(x * x + y * y + z * z));
        rmax = std::max(rmax, r);
        rmin = std::min(rmin, r);
    }
    rs = cmax + rmax;
    if (!(rmin < INFINITY)) rmin = 0.0;
}
// The box of the centres of the spheres `ids` of s (the near test: an origin within a distance
// of every corner of it is within that distance of every centre).
inline void centre_box(const lrt_sphere* s, const std::vector<int>& ids, float clo[3], float chi[3]) {
    for (int k = 0; k < 3; ++k) {
        clo[k] = INFINITY;
        chi[k] = -INFINITY;
    }
    for (int i : ids) {
        const float c[3] = {s[i].center.x, s[i].center.y, s[i].center.z};
        for (int k = 0; k < 3; ++k) {
            clo[k] = std::min(clo[k], c[k]);
            chi[k] = std::max(chi[k], c[k]);
        }
    }
}
// A squared-distance bound as a float that a ray's computed sum of three squares (relative
// error <= 3 eps) can be compared with: at or below it, the distance is <= reach.
inline float reach_sq(double reach) { return (float)(reach * reach * (1.0 - std::ldexp(1.0, -20))); }

struct GridHost {
    std::vector<unsigned> cells;   // ncells + 1 (CSR offsets)
    std::vector<uint2> ranges;     // per cell [cells[c], cells[c + 1]): the device's view
    std::vector<float4> rsph, bsph;
    std::vector<int> rid, bid;
    int nx = 0, ny = 0, nz = 0;
    float lo[3] = {0, 0, 0}, h[3] = {1, 1, 1}, ih[3] = {1, 1, 1};
    float pad = 0, ext = 0;
    // exactness reach (GridView): the walk alone is exact for |o| <= reach_near; up to a
    // distance (GridFarT) for |o| <= reach_dda
    double reach_near = 0, reach_dda = 0;
    GridReach R = {};
    float f2near = 0;
    int count = 0;
    // build statistics (the policy)
    double mean_refs = 0;   // references per non-empty cell
    int max_refs = 0;
};

// s: the scene (center, radius); sph: its device form float4(center, r^2); density: cells per
// sphere of the box (more cells: fewer spheres per cell, more cell steps per ray).
// The pad serves candidates up to kGridSafe scene radii from the origin (and the DDA origins
// up to kGridDda), see the Padding note below.
constexpr double kGridSafe = 1.6;
constexpr double kGridDda = 8.0;

inline void build_grid_at(const lrt_sphere* s, int n, const std::vector<float4>& sph, float density, GridHost& G) {
    G = GridHost();
    G.count = n;
    std::vector<float> radii(n);
    for (int i = 0; i < n; ++i) radii[i] = std::fabs(s[i].radius);
    std::vector<float> fin;
    for (float r : radii)
        if (std::isfinite(r)) fin.push_back(r);
    float big_r = INFINITY;
    if (!fin.empty()) {
        const size_t m = fin.size() / 2;
        std::nth_element(fin.begin(), fin.begin() + m, fin.end());
        big_r = 8.0f * fin[m];
    }
    std::vector<char> big(n, 0);
    std::vector<int> in;
    for (int i = 0; i < n; ++i) {
        const bool finite = std::isfinite(s[i].center.x) && std::isfinite(s[i].center.y) &&
                            std::isfinite(s[i].center.z) && std::isfinite(radii[i]);
        if (!finite || radii[i] > big_r) {
            big[i] = 1;
        } else {
            in.push_back(i);
        }
    }
    auto box_of = [&](const std::vector<int>& ids, float lo[3], float hi[3]) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = INFINITY;
            hi[k] = -INFINITY;
        }
        for (int i : ids) {
            const float c[3] = {s[i].center.x, s[i].center.y, s[i].center.z};
            for (int k = 0; k < 3; ++k) {
                lo[k] = std::min(lo[k], c[k] - radii[i]);
                hi[k] = std::max(hi[k], c[k] + radii[i]);
            }
        }
    };
    // Outliers (the light above a field of small spheres): up to 16 spheres that alone stretch
    // the box are tested first by every ray instead -- one removal at a time, while it shrinks
    // the box's volume by at least a third.
    float lo[3], hi[3];
    for (int it = 0; it < 16 && in.size() > 2; ++it) {
        box_of(in, lo, hi);
        float fl = 0.0f;
        for (int k = 0; k < 3; ++k) fl = std::max(fl, hi[k] - lo[k]);
        const float floor_ = 1e-3f * fl + 1e-6f;
        auto vol = [&](const float a[3], const float b[3]) {
            double v = 1.0;
            for (int k = 0; k < 3; ++k) v *= std::max(b[k] - a[k], floor_);
            return v;
        };
        const double v0 = vol(lo, hi);
        int bestj = -1;
        double bestv = v0;
        for (int k = 0; k < 3; ++k)
            for (int side = 0; side < 2; ++side) {   // the sphere that sets this face
                int who = -1;
                for (size_t j = 0; j < in.size(); ++j) {
                    const int i = in[j];
                    const float c = k == 0 ? s[i].center.x : k == 1 ? s[i].center.y : s[i].center.z;
                    const float f = side ? c + radii[i] : c - radii[i];
                    if ((side ? f == hi[k] : f == lo[k])) {
                        if (who >= 0) { who = -2; break; }   // shared face: no single outlier
                        who = (int)j;
                    }
                }
                if (who < 0) continue;
                std::vector<int> rest = in;
                rest.erase(rest.begin() + who);
                float l2[3], h2[3];
                box_of(rest, l2, h2);
                const double v = vol(l2, h2);
                if (v < bestv) {
                    bestv = v;
                    bestj = who;
                }
            }
        if (bestj < 0 || bestv > v0 * (2.0 / 3.0)) break;
        big[in[bestj]] = 1;
        in.erase(in.begin() + bestj);
    }
    for (int i = 0; i < n; ++i)
        if (big[i]) {
            G.bsph.push_back(sph[i]);
            G.bid.push_back(i);
        }
    if (in.empty()) {   // every sphere is tested first: no walk at all
        G.cells.assign(1, 0u);
        G.ranges.assign(1, make_uint2(0u, 0u));
        return;
    }
    box_of(in, lo, hi);
    float ext = 0.0f, span = 0.0f;
    for (int k = 0; k < 3; ++k) {
        ext = std::max(ext, std::max(std::fabs(lo[k]), std::fabs(hi[k])));
        span = std::max(span, hi[k] - lo[k]);
    }
    // Padding, per sphere. Every hit point the reference computes must lie in its
    // sphere's padded box, up to the DDA's rounding (below 2^-16 (max|o| + ext), lrt_grid.h).
    // A candidate at distance t has |c - o| + r <= 1.004 t + 3.02 rmax <= Dsafe for t <= tsafe,
    // so sphere i gets pad_i = hit_excursion(Dsafe, r_i) + the DDA's share for origins up to
    // reach_dda: the walk then finds every candidate up to tsafe from any such origin, and
    // every candidate at all from origins within reach_near = Dsafe - rs (|c - o| + r <= |o| +
    // rs). tsafe is kGridSafe scene radii (rs); beyond it GridFarT / GridFinish take over.
    double rs, rmin;
    sphere_reach(s, in, rs, rmin);
    double rmax = 0.0;
    for (int i : in) rmax = std::max(rmax, (double)radii[i]);
    const double tsafe = std::max(kGridSafe * rs, 1.0);
    const double dsafe = 1.004 * tsafe + 3.02 * rmax;
    const double reach_dda = kGridDda * rs + 1.0;
    // the DDA's share: 2^-16 (|o| + ext) for |o| <= reach_dda, with the box's padded extent
    // (ext grows by at most 2 pads, each far below the extent)
    const double ddapad = std::ldexp(reach_dda + 1.01 * ext + 1e-3, -16);
    auto pad_of = [&](double r) { return (float)((hit_excursion(dsafe, r) + ddapad) * (1.0 + 1e-6)); };
    const float pad0 = std::max((float)(1e-5 * ext + 2.5e-4 * span + 1e-6), pad_of(rmin));   // the largest
    float e3[3];
    double vol = 1.0;
    for (int k = 0; k < 3; ++k) {
        lo[k] -= 2 * pad0;
        hi[k] += 2 * pad0;
        e3[k] = hi[k] - lo[k];
        vol *= e3[k];
    }
    const double target = std::max(1.0, (double)density * (double)in.size());
    float cell = (float)std::cbrt(vol / target);
    int nn[3];
    for (int k = 0; k < 3; ++k) nn[k] = std::max(1, std::min(512, (int)std::ceil(e3[k] / cell)));
    while ((long long)nn[0] * nn[1] * nn[2] > (1LL << 22))
        for (int k = 0; k < 3; ++k) nn[k] = std::max(1, nn[k] / 2);
    G.nx = nn[0];
    G.ny = nn[1];
    G.nz = nn[2];
    for (int k = 0; k < 3; ++k) {
        G.lo[k] = lo[k];
        G.h[k] = e3[k] / (float)nn[k];
        G.ih[k] = 1.0f / G.h[k];
    }
    G.ext = 0.0f;
    for (int k = 0; k < 3; ++k) G.ext = std::max(G.ext, std::max(std::fabs(lo[k]), std::fabs(hi[k])));
    G.pad = pad0;
    // near: |c - o| + r <= (the farthest corner of the grid's box from o) + rmax <= dsafe
    G.reach_near = std::max(0.0, dsafe - rmax);   // (a distance from the farthest corner)
    G.reach_dda = std::max(reach_dda, G.reach_near + rs);
    G.R.tsafe = (float)(tsafe * (1.0 - 1e-6));
    G.f2near = reach_sq(G.reach_near);
    G.R.o2dda = reach_sq(G.reach_dda);
    {
        const double c1 = std::sqrt(std::ldexp(1.0, -19)) + std::ldexp(24.0, -24);   // hit_excursion(D) <= c1 D
        if (!((double)kConeB >= 1.004 * c1 * (1.0 + 1.0 / 1024))) abort();   // (lrt_grid.h's constant)
        // plus GridFarClear's rounding: its values stay below reach_dda + ext + tsafe (+ a)
        for (int k = 0; k < 3; ++k) {
            G.R.lo[k] = G.lo[k];
            G.R.hi[k] = G.lo[k] + (float)nn[k] * G.h[k];   // GridPlane(lo, n, h)
        }
        G.R.conea = (float)(3.02 * rmax * c1 * (1.0 + 1.0 / 1024) +
                          std::ldexp(G.reach_dda + (double)G.ext + tsafe + 1.0, -18));
    }
    // cell lists (CSR), spheres in index order within a cell
    const long long ncells = (long long)nn[0] * nn[1] * nn[2];
    std::vector<unsigned> cnt(ncells + 1, 0u);
    auto range = [&](int i, int k, int& a, int& b) {
        const float c = k == 0 ? s[i].center.x : k == 1 ? s[i].center.y : s[i].center.z;
        const float pi = std::min(G.pad, pad_of(radii[i]));   // (pad_of falls with r)
        const float fa = (c - radii[i] - pi - G.lo[k]) * G.ih[k];
        const float fb = (c + radii[i] + pi - G.lo[k]) * G.ih[k];
        a = std::max(0, std::min(nn[k] - 1, (int)std::floor(fa)));
        b = std::max(0, std::min(nn[k] - 1, (int)std::floor(fb)));
    };
    for (int pass = 0; pass < 2; ++pass) {
        for (int i : in) {
            int a[3], b[3];
            for (int k = 0; k < 3; ++k) range(i, k, a[k], b[k]);
            for (int z = a[2]; z <= b[2]; ++z)
                for (int y = a[1]; y <= b[1]; ++y)
                    for (int x = a[0]; x <= b[0]; ++x) {
                        const long long c = ((long long)z * nn[1] + y) * nn[0] + x;
                        if (pass == 0) {
                            ++cnt[c + 1];
                        } else {
                            const unsigned at = cnt[c]++;
                            G.rsph[at] = sph[i];
                            G.rid[at] = i;
                        }
                    }
        }
        if (pass == 0) {
            for (long long c = 0; c < ncells; ++c) cnt[c + 1] += cnt[c];
            G.cells.assign(cnt.begin(), cnt.end());
            G.rsph.resize(cnt[ncells]);
            G.rid.resize(cnt[ncells]);
        }
    }
    G.ranges.resize(ncells);
    for (long long c = 0; c < ncells; ++c) G.ranges[c] = make_uint2(G.cells[c], G.cells[c + 1]);
    long long nonempty = 0;
    for (long long c = 0; c < ncells; ++c) {
        const int r = (int)(G.cells[c + 1] - G.cells[c]);
        nonempty += r > 0;
        G.max_refs = std::max(G.max_refs, r);
    }
    G.mean_refs = nonempty ? (double)G.rsph.size() / (double)nonempty : 0.0;
}

// The device's view of G (host arrays here: the host diagnostics and the resolution choice).
inline GridView grid_view_host(const GridHost& G, const float4* all) {
    GridView g;
    g.cells = G.ranges.data();
    g.rsph = G.rsph.data();
    g.rid = G.rid.data();
    g.bsph = G.bsph.data();
    g.bid = G.bid.data();
    g.all = all;
    g.nbig = (int)G.bsph.size();
    g.count = G.nx > 0 ? G.count : 0;
    g.nx = G.nx;
    g.ny = G.ny;
    g.nz = G.nz;
    g.lox = G.lo[0];
    g.loy = G.lo[1];
    g.loz = G.lo[2];
    g.hx = G.h[0];
    g.hy = G.h[1];
    g.hz = G.h[2];
    g.ihx = G.ih[0];
    g.ihy = G.ih[1];
    g.ihz = G.ih[2];
    g.pad = G.pad;
    g.f2near = G.f2near;
    g.o2dda = G.R.o2dda;
    g.tsafe = G.R.tsafe;
    g.conea = G.R.conea;
    g.ext = G.ext;
    g.on = 1;
    g.cells_refs = (unsigned)G.rsph.size();
    return g;
}

// The walk's cost per ray for G, estimated on the host with the device's own walk: rays from
// random points in the box in random directions (bounce and shadow rays) and from a shell
// around it towards random points in it (camera rays); a sphere test counts 1, a cell step
// kGridCellCost (its 8-byte load sits on the walk's critical path). Deterministic.
constexpr double kGridCellCost = 1.5;
inline double grid_cost(const GridHost& G, const std::vector<float4>& sph) {
    if (G.nx == 0) return 0.0;
    const GridView g = grid_view_host(G, sph.data());
    uint32_t st = 0x9E3779B9u;
    auto rnd = [&]() {   // xorshift32 in [0, 1)
        st ^= st << 13;
        st ^= st >> 17;
        st ^= st << 5;
        return (float)(st >> 8) * (1.0f / 16777216.0f);
    };
    const float hi[3] = {G.lo[0] + G.h[0] * G.nx, G.lo[1] + G.h[1] * G.ny, G.lo[2] + G.h[2] * G.nz};
    float c[3], ext = 0.0f;
    for (int k = 0; k < 3; ++k) {
        c[k] = 0.5f * (G.lo[k] + hi[k]);
        ext = std::max(ext, hi[k] - G.lo[k]);
    }
    double cost = 0.0;
    const int m = 2048;
    for (int i = 0; i < m; ++i) {
        F3 o, t;
        F3* pts[2] = {&o, &t};
        for (int q = 0; q < 2; ++q) {
            const float p3[3] = {G.lo[0] + rnd() * (hi[0] - G.lo[0]), G.lo[1] + rnd() * (hi[1] - G.lo[1]),
                                 G.lo[2] + rnd() * (hi[2] - G.lo[2])};
            *pts[q] = f3(p3[0], p3[1], p3[2]);
        }
        if (i & 1) {   // from a shell at 2x the box's extent towards a point in the box
            F3 u = f3(rnd() - 0.5f, rnd() - 0.5f, rnd() - 0.5f);
            const float l = std::sqrt(dot(u, u)) + 1e-6f;
            o = f3(c[0], c[1], c[2]) + u * (2.0f * ext / l);
        } else {       // from a point on a sphere of the grid, outwards (bounce and shadow rays)
            const int id = G.rid.empty() ? 0 : G.rid[(size_t)(rnd() * (float)G.rid.size()) % G.rid.size()];
            const float4 sp = sph[id];
            F3 u = f3(rnd() - 0.5f, rnd() - 0.5f, rnd() - 0.5f);
            const float l = std::sqrt(dot(u, u)) + 1e-6f;
            u = u * (1.0f / l);
            o = f3(sp.x, sp.y, sp.z) + u * std::sqrt(sp.w);
            F3 v = f3(rnd() - 0.5f, rnd() - 0.5f, rnd() - 0.5f);
            if (dot(v, u) < 0.0f) v = -v;
            t = o + v;
        }
        const Ray r = make_ray(o, t - o);
        GridStats gs;
        float tt;
        (void)ClosestHitGrid(r.orig, r.dir, g, tt, &gs);
        cost += gs.spheres + kGridCellCost * gs.cells;
    }
    return cost / m;
}

// The grid at the resolution of lowest estimated cost among a few densities (cells per
// sphere): how the cells fall against the spheres' own spacing matters as much as their
// number. On config 4's field (a jittered 36 x 28 lattice of spheres) the model picks 36 x 1 x
// 29 cells, one lattice site each: 2.6-2.9 sphere tests per ray against 4.1-4.6 at density 2
// (tools/accel_stats.py); measured densities 0.5-2 ran 163-185 ms (profiles/r4_e, r4_f).
inline void build_grid_host(const lrt_sphere* s, int n, const std::vector<float4>& sph, GridHost& G) {
    double best = 0.0;
    bool have = false;
    for (float dens : {0.5f, 0.6f, 0.75f, 0.9f, 1.0f, 1.25f, 1.5f, 2.0f, 3.0f}) {
        GridHost T;
        build_grid_at(s, n, sph, dens, T);
        const double c = grid_cost(T, sph);
        if (!have || c < best) {
            best = c;
            have = true;
            G = std::move(T);
        }
        if (T.nx == 0 && have) break;   // no walk at all: every density is the same
    }
}

// The scene gets the grid when its spheres spread evenly enough: few spheres per cell and
// few tested by every ray (LRT_ACCEL=bvh | grid forces one).
inline bool grid_forced() {
    const char* e = getenv("LRT_ACCEL");
    return e && std::string(e) == "grid";
}
inline bool grid_suitable(const GridHost& G) {
    const char* e = getenv("LRT_ACCEL");
    if (e && std::string(e) == "bvh") return false;
    if (e && std::string(e) == "grid") return true;
    return G.nx > 0 && G.bsph.size() <= 8 && G.mean_refs <= 4.0 && G.max_refs <= 24;
}

}  // namespace lrt
