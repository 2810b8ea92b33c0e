// Scenes on the device: the reference's default scene, packing and upload, the BVH and uniform
// grid builds (closest-hit structures for scenes above 16 spheres), and the camera.
#include <functional>

#include "lrt_grid_build.h"
#include "lrt_internal.h"

namespace lrt {

// parallel.cpp:15-51
const lrt_sphere kDefaultSpheres[9] = {
    {{0, -100.5f, -1}, 100.0f}, {{2, 1, -1}, 0.5f},  {{0, 0, -1}, 0.5f},
    {{-2, 0, -1}, 0.5f},        {{2, 0, 1}, 0.5f},   {{0, 0, 1}, 0.5f},
    {{-2, 0, 1}, 0.5f},         {{0.5f, 1, 0.5f}, 0.5f}, {{-1.5f, 1.5f, 0.f}, 0.3f},
};
const lrt_material kDefaultMats[9] = {
    {LRT_LAMBERT, {0.8f, 0.8f, 0.8f}, {0, 0, 0}, 0, 0},
    {LRT_LAMBERT, {0.8f, 0.4f, 0.4f}, {0, 0, 0}, 0, 0},
    {LRT_LAMBERT, {0.4f, 0.8f, 0.4f}, {0, 0, 0}, 0, 0},
    {LRT_METAL, {0.4f, 0.4f, 0.8f}, {0, 0, 0}, 0, 0},
    {LRT_METAL, {0.4f, 0.8f, 0.4f}, {0, 0, 0}, 0, 0},
    {LRT_METAL, {0.4f, 0.8f, 0.4f}, {0, 0, 0}, 0.2f, 0},
    {LRT_METAL, {0.4f, 0.8f, 0.4f}, {0, 0, 0}, 0.6f, 0},
    {LRT_DIELECTRIC, {0.4f, 0.4f, 0.4f}, {0, 0, 0}, 0, 1.5f},
    {LRT_LAMBERT, {0.8f, 0.6f, 0.2f}, {30, 25, 15}, 0, 0},
};

constexpr int kBvhLeaf = 6;   // leaf size (LRT_BVH_LEAF overrides, 1..16; config 4: 4 -> 350 ms, 6 -> 335, 8 -> 336)
constexpr int kBvhMaxBuildDepth = 22;   // < kBvhStackLevels
constexpr int kBvhSahMaxDepth = 12;     // SAH splits above this depth, median splits below

// ---- BVH build (host): SAH splits, median splits on the longest centroid axis deeper down
struct BvhPrim {
    float lo[3], hi[3], c[3];
    int id;
};
struct BvhBuilder {
    std::vector<BvhPrim> P;
    std::vector<float4> nodes, lsph;
    std::vector<int> lid;
    const std::vector<float4>* sph = nullptr;
    int max_depth = 0;   // deepest internal node (root = 0)
    int leaf = kBvhLeaf;

    void sort_axis(int b, int e, int k) {
        std::sort(P.begin() + b, P.begin() + e, [k](const BvhPrim& x, const BvhPrim& y) {
            return x.c[k] < y.c[k] || (x.c[k] == y.c[k] && x.id < y.id);
        });
    }
    static void grow(const BvhPrim& p, float lo[3], float hi[3]) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], p.lo[k]);
            hi[k] = std::max(hi[k], p.hi[k]);
        }
    }
    static float half_area(const float lo[3], const float hi[3]) {
        const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return dx * dy + dy * dz + dz * dx;
    }

    static void bounds(const BvhPrim* p, int n, float lo[3], float hi[3]) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = INFINITY;
            hi[k] = -INFINITY;
        }
        for (int i = 0; i < n; ++i)
            for (int k = 0; k < 3; ++k) {
                lo[k] = std::min(lo[k], p[i].lo[k]);
                hi[k] = std::max(hi[k], p[i].hi[k]);
            }
    }
    int node(int begin, int end, int depth) {
        max_depth = std::max(max_depth, depth);
        const int idx = (int)(nodes.size() / 4);
        nodes.resize(nodes.size() + 4);
        const int n = end - begin;
        float cl[3] = {INFINITY, INFINITY, INFINITY}, ch[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = begin; i < end; ++i)
            for (int k = 0; k < 3; ++k) {
                cl[k] = std::min(cl[k], P[i].c[k]);
                ch[k] = std::max(ch[k], P[i].c[k]);
            }
        int axis = 0;
        for (int k = 1; k < 3; ++k)
            if (ch[k] - cl[k] > ch[axis] - cl[axis]) axis = k;
        int mid = begin + n / 2;
        if (depth < kBvhSahMaxDepth) {
            // surface-area heuristic over every split of the centroid order on each axis
            // (full sweep: scenes are at most a few thousand spheres); only above
            // kBvhSahMaxDepth, so the depth bound of the median split still holds
            float best = INFINITY;
            int bestAxis = axis, bestSplit = n / 2;
            std::vector<float> leftArea(n);
            for (int k = 0; k < 3; ++k) {
                sort_axis(begin, end, k);
                float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
                for (int i = 0; i < n - 1; ++i) {
                    grow(P[begin + i], lo, hi);
                    leftArea[i + 1] = half_area(lo, hi);
                }
                for (int q = 0; q < 3; ++q) {
                    lo[q] = INFINITY;
                    hi[q] = -INFINITY;
                }
                for (int i = n - 1; i >= 1; --i) {
                    grow(P[begin + i], lo, hi);
                    const float cost = leftArea[i] * (float)i + half_area(lo, hi) * (float)(n - i);
                    if (cost < best) {
                        best = cost;
                        bestAxis = k;
                        bestSplit = i;
                    }
                }
            }
            axis = bestAxis;
            mid = begin + bestSplit;
        }
        std::nth_element(P.begin() + begin, P.begin() + mid, P.begin() + end, [axis](const BvhPrim& x, const BvhPrim& y) {
            return x.c[axis] < y.c[axis] || (x.c[axis] == y.c[axis] && x.id < y.id);
        });
        float4 child[2][2];
        const int rng[2][2] = {{begin, mid}, {mid, end}};
        for (int h = 0; h < 2; ++h) {
            const int b = rng[h][0], e = rng[h][1], cnt = e - b;
            float lo[3], hi[3];
            bounds(P.data() + b, cnt, lo, hi);
            int ref, code;
            if (cnt <= leaf || depth + 1 >= kBvhMaxBuildDepth) {
                ref = (int)lsph.size();
                for (int i = b; i < e; ++i) {
                    lsph.push_back((*sph)[P[i].id]);
                    lid.push_back(P[i].id);
                }
                code = cnt;                      // leaf
            } else {
                ref = node(b, e, depth + 1);     // internal
                code = 0;
            }
            float fr, fc;
            memcpy(&fr, &ref, 4);
            memcpy(&fc, &code, 4);
            child[h][0] = make_float4(lo[0], lo[1], lo[2], fr);
            child[h][1] = make_float4(hi[0], hi[1], hi[2], fc);
        }
        nodes[4 * idx + 0] = child[0][0];
        nodes[4 * idx + 1] = child[0][1];
        nodes[4 * idx + 2] = child[1][0];
        nodes[4 * idx + 3] = child[1][1];
        return idx;
    }
};


// Spheres far larger than the typical one (the ground, r = 100) stay out of the tree and
// are tested first; the rest get a BVH2 with leaves of <= kBvhLeaf spheres.
void build_bvh_host(const lrt_sphere* s, int n, const std::vector<float4>& sph, BvhHost& out) {
    std::vector<float> radii(n);
    for (int i = 0; i < n; ++i) radii[i] = std::fabs(s[i].radius);
    std::vector<float> sorted;
    for (float r : radii)
        if (std::isfinite(r)) sorted.push_back(r);
    float big_r = INFINITY;
    if (!sorted.empty()) {
        const size_t m = sorted.size() / 2;
        std::nth_element(sorted.begin(), sorted.begin() + m, sorted.end());
        big_r = 8.0f * sorted[m];
    }
    std::vector<int> big;
    BvhBuilder B;
    B.sph = &sph;
    if (const char* l = getenv("LRT_BVH_LEAF")) B.leaf = std::min(16, std::max(1, atoi(l)));   // (tests: deep trees)
    std::vector<int> tree;
    for (int i = 0; i < n; ++i) {
        const bool finite = std::isfinite(s[i].center.x) && std::isfinite(s[i].center.y) &&
                            std::isfinite(s[i].center.z) && std::isfinite(radii[i]);
        // non-finite spheres have no box (and would break the split's ordering): like the
        // ground they are tested in index order by every ray, as in the reference's scan
        if (!finite || (radii[i] > big_r && big.size() < 16)) big.push_back(i);
        else tree.push_back(i);
    }
    // Exactness: a box must hold every hit point the reference computes for its
    // sphere, which can lie off the sphere by hit_excursion(|c - o| + r, r). Sphere i's box is
    // padded by hit_excursion(dnear, r_i): enough for origins within dnear - rmax of every
    // corner of the centre box (|c - o| + r <= that + rmax) -- as the grid's tsafe, 1.6 scene
    // radii -- and a ray from anywhere else inflates each box it tests (MakeSlabRay).
    double rs = 0.0, rmin = 0.0, rmax = 0.0;
    sphere_reach(s, tree, rs, rmin);
    for (int i : tree) rmax = std::max(rmax, (double)radii[i]);
    const double dnear = 1.004 * std::max(kGridSafe * rs, 1.0) + 3.02 * rmax;
    float clo[3], chi[3];
    centre_box(s, tree, clo, chi);
    out.clo[0] = clo[0], out.clo[1] = clo[1], out.clo[2] = clo[2];
    out.chi[0] = chi[0], out.chi[1] = chi[1], out.chi[2] = chi[2];
    out.f2near = reach_sq(std::max(0.0, dnear - rmax));
    out.rmax = (float)(rmax * (1.0 + 1e-6));
    out.rmin = (float)(rmin * (1.0 - 1e-6));
    std::vector<float> xpad(n, 0.0f);
    for (int i : tree) xpad[i] = (float)(hit_excursion(dnear, radii[i]) * (1.0 + 1e-6));
    float extent = 1.0f;
    for (int i : tree) {
        BvhPrim p;
        const float r = radii[i];
        const float c3[3] = {s[i].center.x, s[i].center.y, s[i].center.z};
        for (int k = 0; k < 3; ++k) {
            // conservative box: c +/- |r|, padded well beyond float rounding and by the
            // reference's hit excursion
            const float pad = 1e-5f * (std::fabs(c3[k]) + r) + 1e-6f + xpad[i];
            p.lo[k] = c3[k] - r - pad;
            p.hi[k] = c3[k] + r + pad;
            p.c[k] = c3[k];
            extent = std::max(extent, std::max(std::fabs(p.lo[k]), std::fabs(p.hi[k])));
        }
        p.id = i;
        B.P.push_back(p);
    }
    if (B.P.size() >= 2) B.node(0, (int)B.P.size(), 0);
    else
        for (const BvhPrim& p : B.P) big.push_back(p.id);
    out.big0 = (int)B.lsph.size();
    for (int i : big) {
        B.lsph.push_back(sph[i]);
        B.lid.push_back(i);
    }
    out.nbig = (int)big.size();
    out.stack_levels = 1;
    if (!B.nodes.empty()) {   // collapse the BVH2 into 4-wide nodes (grandchildren of each node)
        auto ival = [](float f) { int v; memcpy(&v, &f, 4); return v; };
        auto fval = [](int v) { float f; memcpy(&f, &v, 4); return f; };
        std::vector<float4> n4;
        int depth4 = 0;
        std::function<int(int, int)> collapse = [&](int n2, int dep) -> int {
            depth4 = std::max(depth4, dep);
            const int idx = (int)(n4.size() / 8);
            n4.resize(n4.size() + 8);
            float4 kids[4][2];
            int k = 0;
            for (int c = 0; c < 2; ++c) {
                const float4 lo = B.nodes[4 * n2 + 2 * c], hi = B.nodes[4 * n2 + 2 * c + 1];
                if (ival(hi.w) == 0) {   // internal child: take its two children
                    const int m = ival(lo.w);
                    for (int g = 0; g < 2; ++g) {
                        kids[k][0] = B.nodes[4 * m + 2 * g];
                        kids[k][1] = B.nodes[4 * m + 2 * g + 1];
                        ++k;
                    }
                } else {                 // leaf or empty child stays
                    kids[k][0] = lo;
                    kids[k][1] = hi;
                    ++k;
                }
            }
            for (int c = 0; c < k; ++c)
                if (ival(kids[c][1].w) == 0) kids[c][0].w = fval(collapse(ival(kids[c][0].w), dep + 1));
            for (int c = 0; c < 4; ++c) {
                if (c < k) {
                    n4[8 * idx + 2 * c] = kids[c][0];
                    n4[8 * idx + 2 * c + 1] = kids[c][1];
                } else {   // empty slot
                    n4[8 * idx + 2 * c] = make_float4(INFINITY, INFINITY, INFINITY, fval(0));
                    n4[8 * idx + 2 * c + 1] = make_float4(-INFINITY, -INFINITY, -INFINITY, fval(-1));
                }
            }
            return idx;
        };
        collapse(0, 0);
        B.nodes.swap(n4);
        // a traversal holds at most one (node, child mask) entry per level above its node
        // (StackPush, lrt_bvh.h): depth4 entries; one spare
        out.stack_levels = depth4 + 1;
    }
    out.nodes.swap(B.nodes);
    out.lsph.swap(B.lsph);
    out.lid.swap(B.lid);
    out.margin = 1e-5f * extent + 1e-4f;
}

void bvh_view_host(const BvhHost& B, BvhView& bv) {
    bv = BvhView{};
    bv.nodes = B.nodes.data();
    bv.lsph = B.lsph.data();
    bv.lid = B.lid.data();
    bv.margin = B.margin;
    bv.on = 1;
    bv.nnodes = (int)(B.nodes.size() / 8);
    bv.big0 = B.big0;
    bv.nbig = B.nbig;
    bv.clox = B.clo[0];
    bv.cloy = B.clo[1];
    bv.cloz = B.clo[2];
    bv.chix = B.chi[0];
    bv.chiy = B.chi[1];
    bv.chiz = B.chi[2];
    bv.f2near = B.f2near;
    bv.rmax = B.rmax;
    bv.rmin = B.rmin;
}

void free_scene(Context& c) {
    if (c.d_bvh_nodes) (void)hipFree(c.d_bvh_nodes);
    if (c.d_bvh_lsph) (void)hipFree(c.d_bvh_lsph);
    if (c.d_bvh_lid) (void)hipFree(c.d_bvh_lid);
    c.d_bvh_nodes = nullptr;
    c.d_bvh_lsph = nullptr;
    c.d_bvh_lid = nullptr;
    c.bvh = BvhView{};
    c.bvh_on = 0;
    c.bvh_built = false;
    for (void* p : {(void*)c.d_grid_cells, (void*)c.d_grid_rsph, (void*)c.d_grid_rid, (void*)c.d_grid_bsph,
                    (void*)c.d_grid_bid})
        if (p) (void)hipFree(p);
    c.d_grid_cells = nullptr;
    c.d_grid_rsph = nullptr;
    c.d_grid_rid = nullptr;
    c.d_grid_bsph = nullptr;
    c.d_grid_bid = nullptr;
    c.gv = GridView{};
    c.grid_pick = false;
    c.grid_ok = false;
    c.grid_built = false;
    if (c.d_sph) (void)hipFree(c.d_sph);
    if (c.d_mats) (void)hipFree(c.d_mats);
    if (c.d_lights) (void)hipFree(c.d_lights);
    c.d_sph = nullptr;
    c.d_mats = nullptr;
    c.d_lights = nullptr;
}

// The device layout of a scene: float4(center, r^2), three material rows,
// emissive ids in index order.
int pack_scene(const lrt_sphere* s, const lrt_material* m, int n, std::vector<float4>& sph,
               std::vector<float4>& mats, std::vector<int>& lights) {
    if (!s || !m || n < 1 || n > LRT_MAX_SPHERES) return fail(LRT_E_INVALID, "scene: need 1..LRT_MAX_SPHERES spheres");
    sph.assign(n, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    mats.assign(3 * (size_t)n, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    lights.clear();
    for (int i = 0; i < n; ++i) {
        if (m[i].type < 0 || m[i].type > 2) return fail(LRT_E_INVALID, "scene: material type must be 0..2");
        const float r = s[i].radius;
        sph[i] = make_float4(s[i].center.x, s[i].center.y, s[i].center.z, r * r);
        const bool diel = m[i].type == LRT_DIELECTRIC;
        int type = m[i].type;
        float typef;
        memcpy(&typef, &type, 4);
        mats[3 * i + 0] = make_float4(m[i].albedo.x, m[i].albedo.y, m[i].albedo.z, typef);
        mats[3 * i + 1] = make_float4(m[i].emissive.x, m[i].emissive.y, m[i].emissive.z, m[i].roughness);
        mats[3 * i + 2] = diel ? make_float4(1.0f, 1.0f, 1.0f, m[i].ri)
                               : make_float4(m[i].albedo.x, m[i].albedo.y, m[i].albedo.z, m[i].ri);
        // parallel.cpp:96: skip only if every channel <= 0
        if (!(m[i].emissive.x <= 0 && m[i].emissive.y <= 0 && m[i].emissive.z <= 0)) lights.push_back(i);
    }
    return LRT_OK;
}

template <class T>
hipError_t upload(T*& d, const std::vector<T>& h) {   // a device copy (at least one element)
    hipError_t e = hipMalloc(&d, sizeof(T) * std::max<size_t>(h.size(), 1));
    if (e == hipSuccess && !h.empty()) e = hipMemcpy(d, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice);
    return e;
}

template <class T>
static void free_dev(T*& d) {
    if (d) (void)hipFree(d);
    d = nullptr;
}
// The BVH's and the grid's device copies (upload_scene, or later on first use: ensure_*). A failed
// upload frees what it had allocated and leaves the structure unbuilt (the next ensure_* starts
// from nothing instead of allocating over the earlier buffers: advisor r5).
static int upload_bvh(Context& c, BvhHost& B) {
    if (B.nodes.empty()) B.nodes.assign(4, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    hipError_t e = upload(c.d_bvh_nodes, B.nodes);
    if (e == hipSuccess) e = upload(c.d_bvh_lsph, B.lsph);
    if (e == hipSuccess) e = upload(c.d_bvh_lid, B.lid);
    if (e != hipSuccess) {
        free_dev(c.d_bvh_nodes);
        free_dev(c.d_bvh_lsph);
        free_dev(c.d_bvh_lid);
        c.bvh_built = false;
        return hip_fail(e, "BVH upload");
    }
    bvh_view_host(B, c.bvh);
    c.bvh.nodes = c.d_bvh_nodes;
    c.bvh.lsph = c.d_bvh_lsph;
    c.bvh.lid = c.d_bvh_lid;
    c.bvh_stack_levels = B.stack_levels;
    c.bvh_built = true;
    return LRT_OK;
}
static int upload_grid(Context& c, const GridHost& G) {
    hipError_t e = upload(c.d_grid_cells, G.ranges);
    if (e == hipSuccess) e = upload(c.d_grid_rsph, G.rsph);
    if (e == hipSuccess) e = upload(c.d_grid_rid, G.rid);
    if (e == hipSuccess) e = upload(c.d_grid_bsph, G.bsph);
    if (e == hipSuccess) e = upload(c.d_grid_bid, G.bid);
    if (e != hipSuccess) {
        free_dev(c.d_grid_cells);
        free_dev(c.d_grid_rsph);
        free_dev(c.d_grid_rid);
        free_dev(c.d_grid_bsph);
        free_dev(c.d_grid_bid);
        c.grid_built = false;
        return hip_fail(e, "grid upload");
    }
    GridView& g = c.gv;
    g = grid_view_host(G, c.d_sph);
    g.cells = c.d_grid_cells;
    g.rsph = c.d_grid_rsph;
    g.rid = c.d_grid_rid;
    g.bsph = c.d_grid_bsph;
    g.bid = c.d_grid_bid;
    c.grid_built = true;
    return LRT_OK;
}
static void pack_spheres(const std::vector<lrt_sphere>& s, std::vector<float4>& sph) {
    sph.resize(s.size());
    for (size_t i = 0; i < s.size(); ++i)
        sph[i] = make_float4(s[i].center.x, s[i].center.y, s[i].center.z, s[i].radius * s[i].radius);
}
// The BVH is built when the policy picks it at lrt_set_scene, else on the first render that
// asks for it (LRT_F_BVH, a feature launch, the wavefront kernels); the grid when the policy
// needs it (scenes above kBvhMinSpheres, unless LRT_ACCEL=bvh), else on the first LRT_F_GRID
// render. (advisor r4: every scene used to pay for both builds and both uploads.) A structure
// built lazily can therefore fail at that render (LRT_E_HIP / LRT_E_INVALID from
// lrt_render_*), not at lrt_set_scene; the scene itself stays in place.
int ensure_bvh(Context& c) {
    if (c.bvh_built || !c.bvh_on) return LRT_OK;
    std::vector<float4> sph;
    pack_spheres(c.spheres, sph);
    BvhHost B;
    build_bvh_host(c.spheres.data(), c.count, sph, B);
    if (B.stack_levels > kBvhStackLevels) return fail(LRT_E_INVALID, "BVH deeper than the traversal stack");
    return upload_bvh(c, B);
}
int ensure_grid(Context& c) {
    if (c.grid_built || !c.grid_ok) return LRT_OK;
    std::vector<float4> sph;
    pack_spheres(c.spheres, sph);
    GridHost G;
    build_grid_host(c.spheres.data(), c.count, sph, G);
    return upload_grid(c, G);
}

// Builds what the policy needs on the host first and checks it, then replaces the device's
// scene: a refused scene leaves the previous one in place, whole (advisor r3: the BVH depth
// check used to fail after the old scene was freed).
int upload_scene(Context& c, const lrt_sphere* s, const lrt_material* m, int n) {
    std::vector<float4> sph, mats;
    std::vector<int> lights;
    if (const int e = pack_scene(s, m, n, sph, mats, lights)) return e;
    const bool accel = n > kBvhMinSpheres;
    const char* env = getenv("LRT_ACCEL");
    const bool force_bvh = env && std::string(env) == "bvh";
    BvhHost B;
    GridHost G;
    bool have_grid = false, pick = false;
    // the grid where the policy decides (grid_suitable) or is told to (LRT_ACCEL=grid)
    if ((accel && !force_bvh) || (!accel && grid_forced())) {
        build_grid_host(s, n, sph, G);
        have_grid = true;
        pick = accel ? grid_suitable(G) : true;
    }
    const bool have_bvh = accel && !pick;
    if (have_bvh) {
        build_bvh_host(s, n, sph, B);
        // the LDS traversal stack is sized to B.stack_levels entries per lane, which bounds
        // every push (StackPush: at most one entry per level above the current node)
        if (B.stack_levels > kBvhStackLevels) return fail(LRT_E_INVALID, "BVH deeper than the traversal stack");
    }
    free_scene(c);
    LRT_HIP(upload(c.d_sph, sph));
    LRT_HIP(upload(c.d_mats, mats));
    LRT_HIP(upload(c.d_lights, lights));
    c.bvh_on = accel ? 1 : 0;
    c.grid_ok = n > 0;
    c.grid_pick = pick;
    if (have_bvh)
        if (int rc = upload_bvh(c, B)) return rc;
    if (have_grid)
        if (int rc = upload_grid(c, G)) return rc;
    c.count = n;
    ++c.scene_version;
    c.nlights = (int)lights.size();
    c.spheres.assign(s, s + n);
    c.mats.assign(m, m + n);
    return LRT_OK;
}

lrt_float3 L3(float x, float y, float z) {
    lrt_float3 r = {x, y, z};
    return r;
}
// Host float3 helpers for the camera constructor (maths.h:63-97).
lrt_float3 h_sub(lrt_float3 a, lrt_float3 b) { return L3(a.x - b.x, a.y - b.y, a.z - b.z); }
lrt_float3 h_smul(float a, lrt_float3 b) { return L3(a * b.x, a * b.y, a * b.z); }
lrt_float3 h_cross(lrt_float3 a, lrt_float3 b) {
    return L3(a.y * b.z - a.z * b.y, -(a.x * b.z - a.z * b.x), a.x * b.y - a.y * b.x);
}
lrt_float3 h_normalize(lrt_float3 v) {
    float k = 1.0f / sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    return L3(v.x * k, v.y * k, v.z * k);
}

int camera_make(lrt_float3 lookFrom, lrt_float3 lookAt, lrt_float3 vup, float vfov, float aspect, float aperture,
                float focusDist, lrt_camera* out) {   // maths.h:183-202
    if (!out) return fail(LRT_E_INVALID, "camera out is NULL");
    lrt_camera c;
    c.lensRadius = aperture / 2.0f;
    c.origin = lookFrom;
    c.a = h_normalize(h_sub(lookFrom, lookAt));
    c.r = h_normalize(h_cross(vup, c.a));
    c.u = h_normalize(h_cross(c.a, c.r));
    float theta = vfov * kPI / 180.0f;
    float halfHeightTan = tanf(theta / 2.0f);
    float halfWidthTan = aspect * halfHeightTan;
    c.lowerLeftCorner = h_sub(h_sub(h_sub(c.origin, h_smul(halfWidthTan * focusDist, c.r)),
                                    h_smul(halfHeightTan * focusDist, c.u)),
                              h_smul(focusDist, c.a));
    c.horizontalVec = h_smul(2.0f * halfWidthTan * focusDist, c.r);
    c.verticalVec = h_smul(2.0f * halfHeightTan * focusDist, c.u);
    *out = c;
    return LRT_OK;
}

int camera_default(int w, int h, lrt_camera* out) {   // parallel.cpp:299-307
    if (w < 1 || h < 1) return fail(LRT_E_INVALID, "width/height must be >= 1");
    return camera_make(L3(0, 2, 3), L3(0, 0, 0), L3(0, 1, 0), 60.0f, (float)w / (float)h, 0.1f, 3.0f, out);
}

}  // namespace lrt
