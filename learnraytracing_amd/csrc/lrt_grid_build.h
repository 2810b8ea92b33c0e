// Host build of the uniform grid (lrt_grid.h): box, resolution, the spheres every ray tests
// first, and the cell lists. Also the policy that decides whether a scene gets the grid or
// the BVH (grid_suitable).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "lrt.h"

namespace lrt {

struct GridHost {
    std::vector<unsigned> cells;   // ncells + 1 (CSR offsets)
    std::vector<uint2> ranges;     // per cell [cells[c], cells[c + 1]): the device's view
    std::vector<float4> rsph, bsph;
    std::vector<int> rid, bid;
    int nx = 0, ny = 0, nz = 0;
    float lo[3] = {0, 0, 0}, h[3] = {1, 1, 1}, ih[3] = {1, 1, 1};
    float pad = 0, errk = 0, ext = 0;
    int count = 0;
    // build statistics (the policy)
    double mean_refs = 0;   // references per non-empty cell
    int max_refs = 0;
};

// Cells per sphere (LRT_GRID_DENSITY, default 2): more cells, fewer spheres per cell but more
// cell steps per ray.
inline float grid_density() {
    const char* e = getenv("LRT_GRID_DENSITY");
    const float v = e ? (float)atof(e) : 2.0f;
    return v > 0.05f && v < 64.0f ? v : 2.0f;
}

// s: the scene (center, radius); sph: its device form float4(center, r^2).
inline void build_grid_host(const lrt_sphere* s, int n, const std::vector<float4>& sph, GridHost& G) {
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
    // padding: far above the walk's rounding (2^-16 (|o| + ext) for origins up to ~8 scene
    // sizes away, lrt_grid.h), far below a cell (~1/40 of the span)
    const float pad0 = 1e-5f * ext + 2.5e-4f * span + 1e-6f;
    float e3[3];
    double vol = 1.0;
    for (int k = 0; k < 3; ++k) {
        lo[k] -= 2 * pad0;
        hi[k] += 2 * pad0;
        e3[k] = hi[k] - lo[k];
        vol *= e3[k];
    }
    const double target = std::max(1.0, (double)grid_density() * (double)in.size());
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
    G.errk = 0.5f * pad0;
    // cell lists (CSR), spheres in index order within a cell
    const long long ncells = (long long)nn[0] * nn[1] * nn[2];
    std::vector<unsigned> cnt(ncells + 1, 0u);
    auto range = [&](int i, int k, int& a, int& b) {
        const float c = k == 0 ? s[i].center.x : k == 1 ? s[i].center.y : s[i].center.z;
        const float fa = (c - radii[i] - G.pad - G.lo[k]) * G.ih[k];
        const float fb = (c + radii[i] + G.pad - G.lo[k]) * G.ih[k];
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

// The scene gets the grid when its spheres spread evenly enough: few spheres per cell and
// few tested by every ray (LRT_ACCEL=bvh | grid forces one).
inline bool grid_suitable(const GridHost& G) {
    const char* e = getenv("LRT_ACCEL");
    if (e && std::string(e) == "bvh") return false;
    if (e && std::string(e) == "grid") return true;
    return G.nx > 0 && G.bsph.size() <= 8 && G.mean_refs <= 4.0 && G.max_refs <= 24;
}

}  // namespace lrt
