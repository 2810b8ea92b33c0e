// Diagnostics behind the C-ABI (tests and tools, never on a render path): BVH and grid
// traversal statistics against the linear scan, the device Scatter and BVH probes, the libm
// restatement on host and device.
#include "lrt_grid_build.h"
#include "lrt_internal.h"

namespace lrt {

LRT_HD float libm_eval(int kind, float x) {
    if (kind == 6 || kind == 7) {   // the path's sincosf (one reduction, both results)
        float sn, cs;
        libm::sincosf(x, &sn, &cs);
        return kind == 6 ? sn : cs;
    }
    return kind == 0   ? libm::sinf(x)
           : kind == 1 ? libm::cosf(x)
           : kind == 2 ? libm::powf5(x)
           : kind == 3 ? libm::powf(x, 0.416666667f)
           : kind == 4 ? sqrt_rn(x)    // the path's correctly rounded sqrt (fast sequence on the device)
                       : rcp_rn(x);    // and reciprocal
}

__global__ void libm_kernel(int kind, const float* __restrict__ in, float* __restrict__ out, long long n) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x = in[i];
    out[i] = libm_eval(kind, x);
}


// lrt_scatter_eval's case i: Scatter (lrt_trace.h, parallel.cpp:78-196) of material ids[i]
// for the ray rays[6i..] (through the Ray ctor) at the hit recs[7i..] under RNG state seeds[i].
template <int kAcc>
LRT_DEV void scatter_case(const SceneView& sc, int i, const int* ids, const float* rays, const float* recs,
                          const uint32_t* seeds, float* out, int* ret, int* counted, uint32_t* state,
                          bool coherent = false) {
    const Ray r = make_ray(f3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]),
                           f3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]));
    Hit rec;
    rec.pos = f3(recs[7 * i], recs[7 * i + 1], recs[7 * i + 2]);
    rec.normal = f3(recs[7 * i + 3], recs[7 * i + 4], recs[7 * i + 5]);
    rec.t = recs[7 * i + 6];
    const Material mat = load_material(sc.mats, ids[i]);
    uint32_t rng = seeds[i];
    int rays_ = 0;
    F3 att = f3(0.0f, 0.0f, 0.0f), lightE = f3(0.0f, 0.0f, 0.0f);
    Ray sc_ray;
    sc_ray.orig = sc_ray.dir = f3(0.0f, 0.0f, 0.0f);
    const bool ok = Scatter<kAcc>(mat, r, rec, att, sc_ray, lightE, rays_, rng, sc, coherent);
    const F3 v[4] = {att, sc_ray.orig, sc_ray.dir, lightE};
    for (int k = 0; k < 4; ++k) {
        out[12 * i + 3 * k] = v[k].x;
        out[12 * i + 3 * k + 1] = v[k].y;
        out[12 * i + 3 * k + 2] = v[k].z;
    }
    ret[i] = ok ? 1 : 0;
    counted[i] = rays_;
    state[i] = rng;
}
template <int kAcc>
__global__ __launch_bounds__(64) void scatter_probe_kernel(SceneView sc, const int* ids, const float* rays,
                                                           const float* recs, const uint32_t* seeds, int n,
                                                           float* out, int* ret, int* counted, uint32_t* state,
                                                           int coherent) {
    __shared__ unsigned short stk[kBvhStackLevels * 64];
    sc.pow = libm::pow_tables();   // the device's table addresses (the host filled in its own)
    sc.bstk = stk + threadIdx.x;
    sc.bstride = 64;
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i < n) scatter_case<kAcc>(sc, i, ids, rays, recs, seeds, out, ret, counted, state, coherent != 0);
}

// lrt_accel_eval's device side: one thread per ray; the BVH per lane or as a packet, or the grid.
template <int kAcc>
__global__ __launch_bounds__(64) void accel_probe_kernel(BvhView bv, GridView g, const float* rays, int n, int* ids,
                                                         float* ts, int packet) {
    __shared__ unsigned short stk[kBvhStackLevels * 64];
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    const Ray r = make_ray(f3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]),
                           f3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]));
    float t = 0.0f;
    if constexpr (kAcc == kAccBvh) ids[i] = ClosestHitBVH(r.orig, r.dir, bv, t, stk + threadIdx.x, 64, nullptr, packet != 0);
    else ids[i] = ClosestHitGrid(r.orig, r.dir, g, t);
    ts[i] = t;
}

}  // namespace lrt

using namespace lrt;

namespace lrt {
bool g_ktiming_on = false;
// (start, stop, device) per recorded launch: events belong to the device current at their
// creation, and a launch on another device (render_host_multi, a second context) gets a pair of
// its own device's (advisor r5: a process-global pool recorded foreign-device events)
struct KTiming {
    hipEvent_t a, b;
    int dev;
};
std::vector<KTiming> g_ktiming_ev;
size_t g_ktiming_used = 0;
void kernel_timing_mark(hipStream_t s, int which) {
    if (which == 0) {
        int dev = -1;
        if (hipGetDevice(&dev) != hipSuccess) {
            g_ktiming_on = false;   // (diagnostic only: stop rather than fail the render)
            return;
        }
        if (g_ktiming_used < g_ktiming_ev.size() && g_ktiming_ev[g_ktiming_used].dev != dev) {
            int cur = -1;   // this slot's events are another device's: replace them
            KTiming& k = g_ktiming_ev[g_ktiming_used];
            (void)hipGetDevice(&cur);
            (void)hipSetDevice(k.dev);
            (void)hipEventDestroy(k.a);
            (void)hipEventDestroy(k.b);
            (void)hipSetDevice(cur);
            g_ktiming_ev.erase(g_ktiming_ev.begin() + (long)g_ktiming_used);
        }
        if (g_ktiming_used >= g_ktiming_ev.size()) {
            hipEvent_t a = nullptr, b = nullptr;
            if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
                g_ktiming_on = false;
                return;
            }
            g_ktiming_ev.insert(g_ktiming_ev.begin() + (long)g_ktiming_used, KTiming{a, b, dev});
        }
        if (hipEventRecord(g_ktiming_ev[g_ktiming_used].a, s) != hipSuccess) g_ktiming_on = false;
    } else {
        if (hipEventRecord(g_ktiming_ev[g_ktiming_used].b, s) != hipSuccess) g_ktiming_on = false;
        ++g_ktiming_used;
    }
}
}  // namespace lrt

extern "C" {

// Diagnostic (host only, no GPU): build the BVH of the given scene and trace n rays
// (o.xyz, d.xyz; d normalised as the Ray ctor does) with the device traversal code.
// out[0..4]: mean nodes visited, mean spheres tested, max nodes, max spheres, fraction of
// rays whose (id, t) differs from the linear scan (must be 0).
int lrt_bvh_stats(const lrt_sphere* spheres, int count, const float* rays, int n, double* out) {
    if (!spheres || count < 2 || !rays || !out || n < 1) return fail(LRT_E_INVALID, "invalid arguments");
    std::vector<float4> sph(count);
    for (int i = 0; i < count; ++i) {
        const float r = spheres[i].radius;
        sph[i] = make_float4(spheres[i].center.x, spheres[i].center.y, spheres[i].center.z, r * r);
    }
    BvhHost H;
    build_bvh_host(spheres, count, sph, H);
    BvhView bv;
    bvh_view_host(H, bv);
    double sn = 0, ss = 0, mn = 0, ms = 0, bad = 0, msp = 0;
    unsigned short stk[kBvhStackLevels];
    for (int i = 0; i < n; ++i) {
        const Ray r = make_ray(f3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]),
                               f3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]));
        BvhStats st;
        float t1, t2;
        const int a = ClosestHitBVH(r.orig, r.dir, bv, t1, stk, 1, &st);
        const int b = ClosestHit(r.orig, r.dir, sph.data(), count, t2);
        if (a != b || memcmp(&t1, &t2, 4) != 0) bad += 1;
        // the bounded shadow-ray traversal: true for the scan's winner, and for any other
        // sphere exactly when it is the winner
        if (b >= 0 && !ShadowReachesLightBVH(r.orig, r.dir, b, sph[b], bv, stk, 1, false, &st)) bad += 1;
        const int other = (int)(((unsigned)i * 7919u) % (unsigned)count);
        if (ShadowReachesLightBVH(r.orig, r.dir, other, sph[other], bv, stk, 1, false, &st) != (b == other)) bad += 1;
        // the two-query loop (pool kernel): this ray as the shadow ray towards `other` (and
        // towards the winner), the next ray's direction from the same origin as the bounce ray
        {
            const int i2 = (i + 1) % n;
            const Ray r2 = make_ray(r.orig, f3(rays[6 * i2 + 3], rays[6 * i2 + 4], rays[6 * i2 + 5]));
            float t3, t4;
            const int c2 = ClosestHitBVH(r2.orig, r2.dir, bv, t3, stk, 1);
            for (int li : {other, b}) {
                if (li < 0) continue;
                bool lit = true;
                const int c3 = ClosestHitDualBVH4(r.orig, r2.dir, true, r.dir, li, sph[li], bv, t4, lit, stk, 1, &st);
                if (c3 != c2 || memcmp(&t3, &t4, 4) != 0 || lit != (b == li)) bad += 1;
            }
            bool lit = true;
            const int c4 = ClosestHitDualBVH4(r.orig, r2.dir, false, r.dir, 0, sph[0], bv, t4, lit, stk, 1, &st);
            if (c4 != c2 || memcmp(&t3, &t4, 4) != 0 || lit) bad += 1;
        }
        sn += st.nodes;
        ss += st.spheres;
        mn = std::max(mn, (double)st.nodes);
        msp = std::max(msp, (double)st.max_sp);
        ms = std::max(ms, (double)st.spheres);
    }
    out[0] = sn / n;
    out[1] = ss / n;
    out[2] = mn;
    out[3] = ms;
    out[4] = bad / n;
    out[5] = msp;                    // deepest stack entry any traversal wrote
    out[6] = (double)H.stack_levels; // the entries the LDS stack holds for this scene
    return LRT_OK;
}

int lrt_grid_stats(const lrt_sphere* spheres, int count, const float* rays, int n, double* out) {
    if (!spheres || count < 1 || !rays || !out || n < 1) return fail(LRT_E_INVALID, "invalid arguments");
    std::vector<float4> sph(count);
    for (int i = 0; i < count; ++i) {
        const float r = spheres[i].radius;
        sph[i] = make_float4(spheres[i].center.x, spheres[i].center.y, spheres[i].center.z, r * r);
    }
    GridHost G;
    build_grid_host(spheres, count, sph, G);
    const GridView g = grid_view_host(G, sph.data());
    double sc = 0, ss = 0, mx = 0, bad = 0, fb = 0;
    for (int i = 0; i < n; ++i) {
        const Ray r = make_ray(f3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]),
                               f3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]));
        GridStats st;
        float t1, t2;
        const int a = ClosestHitGrid(r.orig, r.dir, g, t1, &st);
        const int b = ClosestHit(r.orig, r.dir, sph.data(), count, t2);
        if (a != b || memcmp(&t1, &t2, 4) != 0) bad += 1;
        sc += st.cells;
        ss += st.spheres;
        fb += st.fallback;
        mx = std::max(mx, (double)(st.cells + st.spheres));
        GridStats st2;   // (not counted in the means)
        if (b >= 0 && !ShadowReachesLightGrid(r.orig, r.dir, b, sph[b], g, &st2)) bad += 1;
        const int other = (int)(((unsigned)i * 7919u) % (unsigned)count);
        if (ShadowReachesLightGrid(r.orig, r.dir, other, sph[other], g, &st2) != (b == other)) bad += 1;
        {   // the two-query loop: this ray as the shadow ray, the next ray's direction as the bounce
            const int i2 = (i + 1) % n;
            const Ray r2 = make_ray(r.orig, f3(rays[6 * i2 + 3], rays[6 * i2 + 4], rays[6 * i2 + 5]));
            float t3, t4;
            const int c2 = ClosestHit(r2.orig, r2.dir, sph.data(), count, t3);
            for (int li : {other, b}) {
                if (li < 0) continue;
                bool lit = true;
                const int c3 = ClosestHitDualGrid(r.orig, r2.dir, true, r.dir, li, sph[li], g, t4, lit, &st2);
                if (c3 != c2 || memcmp(&t3, &t4, 4) != 0 || lit != (b == li)) bad += 1;
            }
            bool lit = true;
            const int c4 = ClosestHitDualGrid(r.orig, r2.dir, false, r.dir, 0, sph[0], g, t4, lit, &st2);
            if (c4 != c2 || memcmp(&t3, &t4, 4) != 0 || lit) bad += 1;
        }
    }
    out[0] = sc / n;
    out[1] = ss / n;
    out[2] = mx;
    out[3] = bad / n;
    out[4] = fb / n;
    out[5] = G.nx;
    out[6] = G.ny;
    out[7] = G.nz;
    out[8] = (double)G.bsph.size();
    out[9] = grid_suitable(G) ? 1.0 : 0.0;
    return LRT_OK;
}

int lrt_scatter_eval(const lrt_sphere* spheres, const lrt_material* materials, int count, const int* ids,
                     const float* rays, const float* recs, const uint32_t* seeds, int n, float* out, int* ret,
                     int* counted, uint32_t* state, int on_device) {
    if (!ids || !rays || !recs || !seeds || !out || !ret || !counted || !state || n < 0)
        return fail(LRT_E_INVALID, "scatter probe: null argument");
    std::vector<float4> sph, mats;
    std::vector<int> lights;
    if (const int e = pack_scene(spheres, materials, count, sph, mats, lights)) return e;
    for (int i = 0; i < n; ++i)
        if (ids[i] < 0 || ids[i] >= count) return fail(LRT_E_INVALID, "scatter probe: material id out of range");
    if (n == 0) return LRT_OK;
    const bool bvh = count > kBvhMinSpheres;
    BvhHost B;
    if (bvh) build_bvh_host(spheres, count, sph, B);
    SceneView sc{};
    sc.count = count;
    sc.nlights = (int)lights.size();
    if (lights.empty()) lights.push_back(0);   // never read (nlights = 0): keeps the copy non-empty
    sc.pow = libm::pow_tables();   // host addresses: the probe kernel sets its own
    sc.rnlut = nullptr;
    bvh_view_host(B, sc.bv);
    sc.bv.on = bvh ? 1 : 0;
    sc.bv.nnodes = bvh ? (int)(B.nodes.size() / 8) : 0;
    if (!on_device) {
        sc.sph = sph.data();
        sc.mats = mats.data();
        sc.lights = lights.data();
        sc.bv.nodes = B.nodes.data();
        sc.bv.lsph = B.lsph.data();
        sc.bv.lid = B.lid.data();
        unsigned short stk[kBvhStackLevels];
        sc.bstk = stk;
        sc.bstride = 1;
        for (int i = 0; i < n; ++i) {
            if (bvh) scatter_case<true>(sc, i, ids, rays, recs, seeds, out, ret, counted, state);
            else scatter_case<false>(sc, i, ids, rays, recs, seeds, out, ret, counted, state);
        }
        return LRT_OK;
    }
    // device: one thread per case over device copies of everything
    std::vector<void*> owned;
    auto up = [&](const void* src, size_t bytes) -> void* {   // a device copy (>= 16 B), owned
        void* d = nullptr;
        if (hipMalloc(&d, std::max<size_t>(bytes, 16)) != hipSuccess) return nullptr;
        owned.push_back(d);
        if (bytes && hipMemcpy(d, src, bytes, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
        return d;
    };
    auto release = [&]() {
        for (void* p : owned) (void)hipFree(p);
    };
    void* dd[10] = {up(sph.data(), sph.size() * sizeof(float4)), up(mats.data(), mats.size() * sizeof(float4)),
                    up(lights.data(), lights.size() * sizeof(int)),
                    up(B.nodes.data(), B.nodes.size() * sizeof(float4)),
                    up(B.lsph.data(), B.lsph.size() * sizeof(float4)), up(B.lid.data(), B.lid.size() * sizeof(int)),
                    up(ids, sizeof(int) * n), up(rays, sizeof(float) * 6 * n), up(recs, sizeof(float) * 7 * n),
                    up(seeds, sizeof(uint32_t) * n)};
    float* o_out = nullptr;
    int *o_ret = nullptr, *o_cnt = nullptr;
    uint32_t* o_st = nullptr;
    if (hipMalloc(&o_out, sizeof(float) * 12 * n) == hipSuccess) owned.push_back(o_out);
    if (hipMalloc(&o_ret, sizeof(int) * n) == hipSuccess) owned.push_back(o_ret);
    if (hipMalloc(&o_cnt, sizeof(int) * n) == hipSuccess) owned.push_back(o_cnt);
    if (hipMalloc(&o_st, sizeof(uint32_t) * n) == hipSuccess) owned.push_back(o_st);
    if (std::find(std::begin(dd), std::end(dd), nullptr) != std::end(dd) || !o_out || !o_ret ||
        !o_cnt || !o_st) {
        release();
        return fail(LRT_E_NOMEM, "scatter probe: device allocation failed");
    }
    sc.sph = (const float4*)dd[0];
    sc.mats = (const float4*)dd[1];
    sc.lights = (const int*)dd[2];
    sc.bv.nodes = (const float4*)dd[3];
    sc.bv.lsph = (const float4*)dd[4];
    sc.bv.lid = (const int*)dd[5];
    const unsigned blocks = (unsigned)((n + 63) / 64);
    if (bvh)
        scatter_probe_kernel<true><<<blocks, 64>>>(sc, (const int*)dd[6], (const float*)dd[7], (const float*)dd[8],
                                                   (const uint32_t*)dd[9], n, o_out, o_ret, o_cnt, o_st,
                                                   on_device == 2);
    else
        scatter_probe_kernel<false><<<blocks, 64>>>(sc, (const int*)dd[6], (const float*)dd[7], (const float*)dd[8],
                                                    (const uint32_t*)dd[9], n, o_out, o_ret, o_cnt, o_st, 0);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, o_out, sizeof(float) * 12 * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(ret, o_ret, sizeof(int) * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(counted, o_cnt, sizeof(int) * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(state, o_st, sizeof(uint32_t) * n, hipMemcpyDeviceToHost);
    release();
    if (e != hipSuccess) return fail(LRT_E_HIP, std::string("scatter probe: ") + hipGetErrorString(e));
    return LRT_OK;
}

int lrt_accel_eval(const lrt_sphere* spheres, int count, const float* rays, int n, int accel, int mode, int* ids,
                   float* ts) {
    if (!spheres || count < 1 || !rays || !ids || !ts || n < 0 || accel < 1 || accel > 2 || mode < 0 || mode > 2 ||
        (accel == 2 && mode == 2))
        return fail(LRT_E_INVALID, "accel eval: invalid arguments");
    if (accel == 1 && count < 2) return fail(LRT_E_INVALID, "accel eval: the BVH needs 2 spheres");
    std::vector<float4> sph(count);
    for (int i = 0; i < count; ++i) {
        const float r = spheres[i].radius;
        sph[i] = make_float4(spheres[i].center.x, spheres[i].center.y, spheres[i].center.z, r * r);
    }
    BvhHost H;
    GridHost G;
    BvhView bv{};
    if (accel == 1) {
        build_bvh_host(spheres, count, sph, H);
        bvh_view_host(H, bv);
    } else {
        build_grid_host(spheres, count, sph, G);
    }
    if (mode == 0) {
        const GridView g = accel == 2 ? grid_view_host(G, sph.data()) : GridView{};
        unsigned short stk[kBvhStackLevels];
        for (int i = 0; i < n; ++i) {
            const Ray r = make_ray(f3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]),
                                   f3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]));
            ids[i] = accel == 1 ? ClosestHitBVH(r.orig, r.dir, bv, ts[i], stk, 1) : ClosestHitGrid(r.orig, r.dir, g, ts[i]);
        }
        return LRT_OK;
    }
    if (n == 0) return LRT_OK;
    std::vector<void*> owned;
    auto up = [&](const void* src, size_t bytes) -> void* {   // a device copy (>= 16 B), owned
        void* d = nullptr;
        if (hipMalloc(&d, std::max<size_t>(bytes, 16)) != hipSuccess) return nullptr;
        owned.push_back(d);
        if (bytes && hipMemcpy(d, src, bytes, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
        return d;
    };
    std::vector<void*> need;
    void* d_rays = up(rays, sizeof(float) * 6 * (size_t)n);
    int* o_ids = nullptr;
    float* o_ts = nullptr;
    if (hipMalloc(&o_ids, sizeof(int) * (size_t)n) == hipSuccess) owned.push_back(o_ids);
    if (hipMalloc(&o_ts, sizeof(float) * (size_t)n) == hipSuccess) owned.push_back(o_ts);
    need = {d_rays, o_ids, o_ts};
    GridView g{};
    if (accel == 1) {
        bv.nodes = (const float4*)up(H.nodes.data(), sizeof(float4) * H.nodes.size());
        bv.lsph = (const float4*)up(H.lsph.data(), sizeof(float4) * H.lsph.size());
        bv.lid = (const int*)up(H.lid.data(), sizeof(int) * H.lid.size());
        need.insert(need.end(), {(void*)bv.nodes, (void*)bv.lsph, (void*)bv.lid});
    } else {
        g = grid_view_host(G, sph.data());
        g.cells = (const uint2*)up(G.ranges.data(), sizeof(uint2) * G.ranges.size());
        g.rsph = (const float4*)up(G.rsph.data(), sizeof(float4) * G.rsph.size());
        g.rid = (const int*)up(G.rid.data(), sizeof(int) * G.rid.size());
        g.bsph = (const float4*)up(G.bsph.data(), sizeof(float4) * G.bsph.size());
        g.bid = (const int*)up(G.bid.data(), sizeof(int) * G.bid.size());
        g.all = (const float4*)up(sph.data(), sizeof(float4) * sph.size());
        need.insert(need.end(), {(void*)g.cells, (void*)g.rsph, (void*)g.rid, (void*)g.bsph, (void*)g.bid, (void*)g.all});
    }
    auto release = [&]() {
        for (void* p : owned) (void)hipFree(p);
    };
    if (std::find(need.begin(), need.end(), nullptr) != need.end()) {
        release();
        return fail(LRT_E_NOMEM, "accel eval: device allocation failed");
    }
    const unsigned blocks = (unsigned)((n + 63) / 64);
    if (accel == 1) accel_probe_kernel<kAccBvh><<<blocks, 64>>>(bv, g, (const float*)d_rays, n, o_ids, o_ts, mode == 2);
    else accel_probe_kernel<kAccGrid><<<blocks, 64>>>(bv, g, (const float*)d_rays, n, o_ids, o_ts, 0);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(ids, o_ids, sizeof(int) * (size_t)n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(ts, o_ts, sizeof(float) * (size_t)n, hipMemcpyDeviceToHost);
    release();
    if (e != hipSuccess) return fail(LRT_E_HIP, std::string("accel eval: ") + hipGetErrorString(e));
    return LRT_OK;
}

int lrt_libm_eval_host(int kind, const float* in, float* out, long long n) {
    if (kind < 0 || kind > 7 || !in || !out || n < 0) return fail(LRT_E_INVALID, "invalid libm eval arguments");
    for (long long i = 0; i < n; ++i)
        out[i] = libm_eval(kind, in[i]);
    return LRT_OK;
}

int lrt_libm_eval_device(int kind, const float* d_in, float* d_out, long long n) {
    if (kind < 0 || kind > 7 || !d_in || !d_out || n < 0) return fail(LRT_E_INVALID, "invalid libm eval arguments");
    if (n == 0) return LRT_OK;
    libm_kernel<<<(unsigned)((n + 255) / 256), 256, 0, nullptr>>>(kind, d_in, d_out, n);
    LRT_HIP(hipGetLastError());
    LRT_HIP(hipDeviceSynchronize());
    return LRT_OK;
}


// ---- kernel timing (lrt_kernel_timing) ----------------------------------------------------
int lrt_kernel_timing(int on) {
    lrt::g_ktiming_on = on != 0;
    lrt::g_ktiming_used = 0;
    return LRT_OK;
}
int lrt_kernel_times(float* ms, int max_n, int* n) {
    if (!n || (max_n > 0 && !ms)) return lrt::fail(LRT_E_INVALID, "lrt_kernel_times: null output");
    int k = 0;
    for (size_t i = 0; i < lrt::g_ktiming_used && k < max_n; ++i) {
        auto& p = lrt::g_ktiming_ev[i];
        LRT_HIP(hipEventSynchronize(p.b));
        float t = 0.0f;
        LRT_HIP(hipEventElapsedTime(&t, p.a, p.b));
        ms[k++] = t;
    }
    *n = k;
    lrt::g_ktiming_used = 0;
    return LRT_OK;
}
}  // extern "C"
