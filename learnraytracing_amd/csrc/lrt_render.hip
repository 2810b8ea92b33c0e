// render_device (every render path's core): argument validation, the kernel policy, the
// launch of v0 / the pool kernel / the wavefront kernels, sample mode's merge.
#include "lrt_internal.h"

namespace lrt {

// Sample mode's second half: TraceRowJob's progressive lerp (parallel.cpp:262,280-286)
// over the frame planes in order, one thread per pixel (coalesced plane reads). `a` supplies
// the window's row map and the fused-exchange frame (a.frame); pixel i is the window's
// pixel pix0 + i.
__global__ void merge_samples_kernel(const float4* __restrict__ samp, float4* __restrict__ out, const float* lerp,
                                     int npix, int frame0, int frames, size_t stride, const KernelArgs a, int pix0) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npix) return;
    const float4 o = out[i];
    F3 acc = f3(o.x, o.y, o.z);
    for (int k = 0; k < frames; ++k) {
        const float4 c = samp[(size_t)k * stride + i];
        const int f = frame0 + k;
        const float lerpFac = f < kLerpTable ? lerp[f] : (float)f / (float)(f + 1);
        acc = acc * lerpFac + f3(c.x, c.y, c.z) * (1.0f - lerpFac);
    }
    float* d = reinterpret_cast<float*>(out + i);   // alpha untouched
    d[0] = acc.x;
    d[1] = acc.y;
    d[2] = acc.z;
    if (a.frame) {   // the frame exchange, fused
        const int p = pix0 + i, lx = p % a.xc, ly = p / a.xc;
        a.frame[(size_t)GlobalRow(a, ly) * a.width + a.x0 + lx] = make_float4(acc.x, acc.y, acc.z, o.w);
    }
}

hipError_t launch_merge_samples(const float4* samp, float4* out, const float* lerp, int npix, int frame0, int frames,
                                size_t stride, const KernelArgs& a, int pix0, hipStream_t s) {
    merge_samples_kernel<<<(unsigned)((npix + 255) / 256), 256, 0, s>>>(samp, out, lerp, npix, frame0, frames, stride, a,
                                                                       pix0);
    return hipGetLastError();
}

}  // namespace lrt
#include "lrt_wavefront.h"
namespace lrt {

int validate(const lrt_render_desc* d) {
    if (!d) return fail(LRT_E_INVALID, "desc is NULL");
    if (d->width < 1 || d->height < 1) return fail(LRT_E_INVALID, "width/height must be >= 1");
    if (d->x0 < 0 || d->x_count < 0 || (long long)d->x0 + d->x_count > d->width)
        return fail(LRT_E_INVALID, "column window outside the image");
    if (d->row_block < 1 || d->row_period < 1 || d->row_phase < 0 || d->row_phase >= d->row_period)
        return fail(LRT_E_INVALID, "row_block/row_period/row_phase invalid");
    if (d->y0 < 0 || d->row_count < 0) return fail(LRT_E_INVALID, "y0/row_count must be >= 0");
    if (d->row_count > 0) {
        long long ly = d->row_count - 1;
        long long y = d->y0 + (ly / d->row_block) * (long long)d->row_block * d->row_period +
                      (long long)d->row_phase * d->row_block + ly % d->row_block;
        if (y >= d->height) return fail(LRT_E_INVALID, "local rows map outside the image");
    }
    if (d->frame0 < 0 || d->frames < 0) return fail(LRT_E_INVALID, "frame0/frames must be >= 0");
    if ((long long)d->frame0 + d->frames > 0x7fffffffLL) return fail(LRT_E_INVALID, "frame range overflows int");
    if (d->max_depth < 0 || d->max_depth > kMaxDepthSupported)
        return fail(LRT_E_INVALID, "max_depth must be in 0..64");
    return LRT_OK;
}

#ifdef LRT_EXP_WAVETRACE
// Diagnostic build only: per-wave lifetimes of every v0 launch, appended to the binary
// file $LRT_WAVETRACE (u64 nwaves, then nwaves x {t0, t1, hw_id, xcc_id}; t in 100 MHz ticks).
unsigned long long* wavetrace_buffer(size_t waves) {
    static unsigned long long* d = nullptr;
    static size_t cap = 0;
    if (waves > cap) {
        if (d) (void)hipFree(d);
        (void)hipMalloc(&d, sizeof(unsigned long long) * 4 * waves);
        cap = waves;
    }
    return d;
}
void wavetrace_dump(unsigned long long* d, size_t waves, hipStream_t s) {
    const char* path = getenv("LRT_WAVETRACE");
    if (!path) return;
    std::vector<unsigned long long> h(4 * waves);
    (void)hipMemcpyAsync(h.data(), d, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    FILE* f = fopen(path, "ab");
    if (!f) return;
    unsigned long long n = waves;
    fwrite(&n, sizeof(n), 1, f);
    fwrite(h.data(), sizeof(unsigned long long), h.size(), f);
    fclose(f);
}
#endif

#ifdef LRT_EXP_SECSTATS
unsigned long long* secstats_buffer(hipStream_t s) {
    static unsigned long long* d_sec = nullptr;
    if (!d_sec) (void)hipMalloc(&d_sec, sizeof(unsigned long long) * 3 * kSecN * 16);
    (void)hipMemsetAsync(d_sec, 0, sizeof(unsigned long long) * 3 * kSecN * 16, s);
    return d_sec;
}
void secstats_dump(const unsigned long long* d_sec, hipStream_t s) {
        unsigned long long h[3 * kSecN * 16];
        (void)hipMemcpyAsync(h, d_sec, sizeof(h), hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        const char* names[kSecN] = {"hit", "lambert", "shadow", "metal", "dielectric", "post", "fold", "camera", "other",
                                    "hit0", "shadow0"};
        double tot = 0;
        for (int k = 0; k < kSecN; ++k)
            for (int j = 0; j < 16; ++j) tot += (double)h[3 * (k + kSecN * j) + 2];
        for (int k = 0; k < kSecN; ++k) {
            unsigned long long ex = 0, ln = 0, cy = 0;
            for (int j = 0; j < 16; ++j) {
                ex += h[3 * (k + kSecN * j)];
                ln += h[3 * (k + kSecN * j) + 1];
                cy += h[3 * (k + kSecN * j) + 2];
            }
            fprintf(stderr, "secstats %-10s wave-execs %12llu  lanes/exec %6.2f  cycles %5.1f%%  cyc/exec %8.1f\n", names[k], ex,
                    ex ? (double)ln / ex : 0.0, 100.0 * cy / tot, ex ? (double)cy / ex : 0.0);
        }
}
#endif


hipError_t event_done(hipEvent_t ev, bool* done) {
    *done = false;
    const hipError_t pending = hipGetLastError();
    if (pending != hipSuccess) return pending;
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) {
        *done = true;
        return hipSuccess;
    }
    if (q != hipErrorNotReady) return q;
    (void)hipGetLastError();   // the query's own "not ready"
    return hipSuccess;
}

// Release slot e's buffer from stream s: s waits for the buffer's last use (its event), then
// frees it in stream order. The owning stream may be gone; its recorded event still completes.
static hipError_t scratch_release(Context::Scratch& e, hipStream_t s) {
    hipError_t r = hipSuccess;
    if (e.p) {
        r = hipStreamWaitEvent(s, e.ev, 0);
        if (r == hipSuccess) r = hipFreeAsync(e.p, s);
    }
    e.p = nullptr;
    e.bytes = 0;
    e.s = nullptr;
    return r;
}

hipError_t stream_scratch(hipStream_t s, size_t bytes, void** out) {
    Context& c = ctx();
    Context::Scratch* hit = nullptr;
    for (auto& e : c.scratch)
        if (e.p && e.s == s) hit = &e;
    const unsigned long long now = ++c.order_tick;
    for (auto& e : c.scratch)   // buffers of streams idle for kScratchIdle launches, seen done: released
        if (e.p && &e != hit && now - e.tick > Context::kScratchIdle) {
            bool done = false;
            if (const hipError_t r = event_done(e.ev, &done)) return r;
            if (done)
                if (const hipError_t r = scratch_release(e, s)) return r;
        }
    if (!hit) {   // a free slot, or the least recently used one (taken over in stream order)
        hit = &c.scratch[0];
        for (auto& e : c.scratch)
            if (!e.p || (hit->p && e.tick < hit->tick)) hit = &e;
        if (const hipError_t r = scratch_release(*hit, s)) return r;
        hit->s = s;
    }
    if (!hit->ev)
        if (const hipError_t r = hipEventCreateWithFlags(&hit->ev, hipEventDisableTiming)) return r;
    if (hit->bytes < bytes) {   // grow, ordered on the stream that uses it
        if (hit->p) {
            const hipError_t e = hipFreeAsync(hit->p, s);
            hit->p = nullptr;
            hit->bytes = 0;
            if (e != hipSuccess) return e;
        }
        const hipError_t e = hipMallocAsync(&hit->p, bytes, s);
        if (e != hipSuccess) {
            hit->p = nullptr;
            return e;
        }
        hit->bytes = bytes;
        // (the allocation is the buffer's first use until a launch records over it)
        if (const hipError_t r = hipEventRecord(hit->ev, s)) return r;
    }
    hit->tick = now;
    *out = hit->p;
    return hipSuccess;
}

hipError_t other_stream_busy(hipStream_t s, bool* busy) {
    *busy = false;
    for (auto& e : ctx().scratch)
        if (e.p && e.s != s) {
            bool done = false;
            if (const hipError_t r = event_done(e.ev, &done)) return r;
            if (!done) *busy = true;
        }
    return hipSuccess;
}

hipError_t stream_scratch_used(hipStream_t s) {
    for (auto& e : ctx().scratch)
        if (e.p && e.s == s) return hipEventRecord(e.ev, s);
    return hipSuccess;
}

// Resident blocks per CU for (kernel, LDS bytes), cached: the query costs host time on
// every launch otherwise.
hipError_t occupancy(int* per_cu, const void* kern, int block, size_t lds) {
    struct Entry { const void* k; int b; size_t l; int v; };
    static Entry cache[32];
    static int n = 0;
    for (int i = 0; i < n; ++i)
        if (cache[i].k == kern && cache[i].b == block && cache[i].l == lds) {
            *per_cu = cache[i].v;
            return hipSuccess;
        }
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, kern, block, lds);
    if (e == hipSuccess && n < 32) cache[n++] = {kern, block, lds, *per_cu};
    return e;
}
const char* acc_name(int acc) { return acc == kAccGrid ? "grid" : acc == kAccBvh ? "bvh" : "scan"; }

// Pixels per pool tile: a round holds kPoolSamples samples, so more frames -> fewer pixels.
// Bigger tiles make bigger pools (a round's tail, its last paths with most lanes idle, is a
// smaller share) but fewer tiles per wave (the launch's tail). 64 px at most by default:
// 128-px tiles (taken only while every resident wave still gets one)
// run config 2 pipelined over two streams at 0.2357/0.2373 ms/step against 0.2465/0.2476 and
// config 3 at 1.942/1.936 against 1.950/1.953, but a launch alone at 0.363-0.412 ms against
// 0.286-0.300 (config 3: 2.47-2.66 ms against 2.07-2.09): the few heavy 128-px tiles set the
// end of a launch that no other launch overlaps (profiles/r3_ag, r3_fin2). 256 px left waves
// idle on config 2 (39.4 vs 46.3 Grays/s, r3_g).
int pool_tiles(int pix, int xc, int rows) {
    const int tx = pix >= 128 ? 16 : pix >= 32 ? 8 : pix >= 8 ? 4 : pix >= 2 ? 2 : 1, ty = pix / tx;
    return ((xc + tx - 1) / tx) * ((rows + ty - 1) / ty);
}
int pool_pixels(int frames, int xc, int rows, int cap) {
    const long long slots = 16LL * ctx().num_cus;   // resident waves (4 per SIMD)
    for (int pix : {256, 128, 64, 32, 16})
        if (cap >= pix && pix * frames <= kPoolSamples && (pix <= 64 || pool_tiles(pix, xc, rows) >= slots))
            return pix;
    return 4 * frames <= kPoolSamples ? 4 : 1;
}

// v4 (lrt_wavefront.h): chunks of whole pixels, maxDepth + 1 extend/shade rounds each,
// then the chunk's frame planes merged into the window. Path state is ~100 B + 16 B per
// recursion level per pixel-sample; chunks are sized to a 2 GB budget.
int launch_wavefront(KernelArgs a, bool lds, hipStream_t s) {
    if (a.gv.on && ctx().bvh_on) {   // the wavefront kernels trace through the BVH
        if (int rc = ensure_bvh(ctx())) return rc;
        a.bv = ctx().bvh;
        a.bv.on = 1;
    }
    a.gv.on = 0;
    const int frames = a.frames, levels = std::max(1, a.maxDepth);
    const size_t npix = (size_t)a.xc * a.rows;
    const size_t per_path = 4 + 4 * 16 + 16 + 5 * 4 + 16 * (size_t)levels;
    const size_t budget = (size_t)2 << 30;
    size_t cpix = std::max<size_t>(1, budget / (per_path * (size_t)frames));
    cpix = std::min(cpix, npix);
    const size_t C = cpix * (size_t)frames;
    if (C > 0x7fffffff) return fail(LRT_E_INVALID, "wavefront chunk too large");
    // the persistent grid: every wavefront kernel runs B blocks, block j on region j
    const size_t head = kPowTableBytes + kRenormBytes;
    const size_t scene = lds ? sizeof(float4) * (4 * (size_t)a.count + (size_t)(a.nlights + 3) / 4 + 1) : 0;
    const size_t bstk = a.bv.on ? sizeof(unsigned short) * ctx().bvh_stack_levels * kWfBlock : 0;
    const size_t ldsb = head + scene + bstk;
    const bool bvh = a.bv.on != 0, fixed = lds && !bvh && a.count == kFixedSpheres;
    const void* kx = bvh ? (const void*)wf_extend<true, 0> : fixed ? (const void*)wf_extend<false, kFixedSpheres>
                                                                   : (const void*)wf_extend<false, 0>;
    const void* ks = bvh ? (const void*)wf_shade<true, 0> : fixed ? (const void*)wf_shade<false, kFixedSpheres>
                                                                  : (const void*)wf_shade<false, 0>;
    int per_cu = 0, per_cu_s = 0;
    hipError_t e = occupancy(&per_cu, kx, kWfBlock, ldsb);
    if (e == hipSuccess) e = occupancy(&per_cu_s, ks, kWfBlock, ldsb);
    if (e != hipSuccess) return hip_fail(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    per_cu = std::min(per_cu, per_cu_s);
    if (per_cu < 1) return fail(LRT_E_INVALID, "wavefront kernels do not fit on a CU");
    const int B = per_cu * ctx().num_cus;
    const size_t cnt_bytes = sizeof(unsigned int) * 4 * (size_t)(a.maxDepth + 2) * B;
    const size_t need = per_path * (C + (size_t)B) + cnt_bytes + 256 * 12;
    auto& wf = ctx().wf;
    if (wf.bytes < need) {
        if (wf.buf) (void)hipFree(wf.buf);
        wf.buf = nullptr;
        wf.bytes = 0;
        if (hipMalloc(&wf.buf, need) != hipSuccess) return fail(LRT_E_NOMEM, "hipMalloc(wavefront state)");
        wf.bytes = need;
    }
    if (!wf.rayp) {
        LRT_HIP(hipMalloc(&wf.rayp, sizeof(unsigned long long) * kV0Queues * kCtrStride));
        LRT_HIP(hipMemset(wf.rayp, 0, sizeof(unsigned long long) * kV0Queues * kCtrStride));
    }
    WfArgs w;
    w.a = a;
    char* b = static_cast<char*>(wf.buf);
    auto take = [&](size_t bytes) { void* p = b; b += (bytes + 255) / 256 * 256; return p; };
    const size_t qslots = C + (size_t)B;   // B regions of R0 = ceil(C / B) state slots
    w.o = static_cast<float4*>(take(16 * qslots));
    w.d = static_cast<float4*>(take(16 * qslots));
    w.sl = static_cast<float4*>(take(16 * qslots));
    w.lit = static_cast<float4*>(take(16 * qslots));
    w.samp = static_cast<float4*>(take(16 * C));
    w.stack = static_cast<float4*>(take(16 * qslots * (size_t)levels));
    w.rng = static_cast<uint32_t*>(take(4 * qslots));
    w.qa[0] = static_cast<uint32_t*>(take(4 * qslots));
    w.qa[1] = static_cast<uint32_t*>(take(4 * qslots));
    for (int t = 0; t < 3; ++t) w.qm[t] = static_cast<uint32_t*>(take(4 * qslots));
    w.cnt = static_cast<unsigned int*>(take(cnt_bytes));
    w.rayp = wf.rayp;
    // LDS: [powf tables][renormalize table][scene if staged][bvh traversal stack]
    w.lds = lds ? 1 : 0;
    w.bstk_off = (int)(head + scene);
    const dim3 grid((unsigned)B), block(kWfBlock);
    for (size_t pix0 = 0; pix0 < npix; pix0 += cpix) {
        const size_t cp = std::min(cpix, npix - pix0);
        w.pix0 = (int)pix0;
        w.cpix = (int)cp;
        w.C = (int)(cp * (size_t)frames);
        w.R0 = (int)((w.C + B - 1) / B);
        w.Cs = w.R0 * B;
        LRT_HIP(hipMemsetAsync(w.cnt, 0, cnt_bytes, s));
        wf_camera<<<grid, block, kRenormBytes, s>>>(w);
        for (int it = 0; it <= a.maxDepth; ++it) {
            if (bvh) {
                wf_extend<true, 0><<<grid, block, ldsb, s>>>(w, it);
                wf_shade<true, 0><<<grid, block, ldsb, s>>>(w, it);
            } else if (fixed) {
                wf_extend<false, kFixedSpheres><<<grid, block, ldsb, s>>>(w, it);
                wf_shade<false, kFixedSpheres><<<grid, block, ldsb, s>>>(w, it);
            } else {
                wf_extend<false, 0><<<grid, block, ldsb, s>>>(w, it);
                wf_shade<false, 0><<<grid, block, ldsb, s>>>(w, it);
            }
        }
        e = launch_merge_samples(w.samp, a.out + pix0, a.lerp, (int)cp, a.frame0, a.frames, cp, a, (int)pix0, s);
        if (e != hipSuccess) return hip_fail(e, "wavefront launch");
    }
    snprintf(g_last_launch, sizeof(g_last_launch), "kernel=wf_extend lds=%d bvh=%d grid=%u", lds ? 1 : 0, bvh ? 1 : 0, grid.x);
    wf_rays_collect<<<1, 64, 0, s>>>(wf.rayp, a.rays);
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "wavefront ray collect");
    return LRT_OK;
}


// colours_out (render_host's pipeline): no lerp -- frame f's sample colours go to plane
// f - frame0 of colours_out (x_count * row_count float4 each) and d_buf is not touched.
// frame (lrt_render_device_to_frame): every finished pixel is stored there too, at its global
// row -- the whole width x height RGBA frame, possibly another device's memory.
int render_device(const lrt_render_desc* d, float* d_buf, unsigned long long* d_rays, const lrt_features* feat,
                  hipStream_t s, float4* colours_out, float* frame) {
    int rc = validate(d);
    if (rc) return rc;
    if (!ctx().ready) return fail(LRT_E_STATE, "lrt_initialize() has not been called");
    if (!d_buf || !d_rays) return fail(LRT_E_INVALID, "device buffer / ray counter is NULL");
    constexpr int kKnownFlags = LRT_F_SCENE_GLOBAL | LRT_F_SIMPLE | LRT_F_NO_BVH | LRT_F_NO_DOUBLE_LIGHT |
                                LRT_F_WAVEFRONT | LRT_F_POOL | LRT_F_BVH | LRT_F_GRID;
    if (d->flags & ~kKnownFlags)   // (every path, the colours-only one too; 4/8/16/128: removed kernels)
        return fail(LRT_E_INVALID, "unknown LRT_F_* flag (the v1/v2/v3 kernels were removed: the default picks v0 or v5)");
    if (d->x_count == 0 || d->row_count == 0 || d->frames == 0) return LRT_OK;
    KernelArgs a;
    const lrt_camera& c = d->camera;
    a.cam.origin = f3(c.origin.x, c.origin.y, c.origin.z);
    a.cam.a = f3(c.a.x, c.a.y, c.a.z);
    a.cam.u = f3(c.u.x, c.u.y, c.u.z);
    a.cam.r = f3(c.r.x, c.r.y, c.r.z);
    a.cam.llc = f3(c.lowerLeftCorner.x, c.lowerLeftCorner.y, c.lowerLeftCorner.z);
    a.cam.horiz = f3(c.horizontalVec.x, c.horizontalVec.y, c.horizontalVec.z);
    a.cam.vert = f3(c.verticalVec.x, c.verticalVec.y, c.verticalVec.z);
    a.cam.lensRadius = c.lensRadius;
    a.sph = ctx().d_sph;
    a.mats = ctx().d_mats;
    a.lights = ctx().d_lights;
    a.count = ctx().count;
    a.nlights = ctx().nlights;
    a.width = d->width;
    a.height = d->height;
    a.x0 = d->x0;
    a.xc = d->x_count;
    a.y0 = d->y0;
    a.rows = d->row_count;
    a.rb = d->row_block;
    a.rp = d->row_period;
    a.rph = d->row_phase;
    a.frame0 = d->frame0;
    a.frames = d->frames;
    a.maxDepth = d->max_depth;
    a.out = reinterpret_cast<float4*>(d_buf);
    a.rays = d_rays;
    a.ndl = (d->flags & LRT_F_NO_DOUBLE_LIGHT) ? 1 : 0;
    bool want_feat = false;
    {
        float* const fp[6] = {feat ? feat->normal : nullptr,    feat ? feat->world_pos : nullptr,
                              feat ? feat->albedo : nullptr,    feat ? feat->color_std : nullptr,
                              feat ? feat->normal_std : nullptr, feat ? feat->world_pos_std : nullptr};
        for (int k = 0; k < 6; ++k) {
            a.feat[k] = reinterpret_cast<float4*>(fp[k]);
            want_feat = want_feat || fp[k] != nullptr;
        }
        a.featMax = feat ? feat->max_frame : -1;
    }
    // the uniform grid where the scene suits it (grid_suitable; LRT_F_BVH / LRT_F_GRID force
    // one), except for feature launches (v0's BVH instances); the BVH for the other scenes above
    // kBvhMinSpheres; either built on first use
    const bool use_grid = ctx().grid_ok && !(d->flags & LRT_F_NO_BVH) && !want_feat && !(d->flags & LRT_F_BVH) &&
                          (ctx().grid_pick || (d->flags & LRT_F_GRID));
    const bool use_bvh = ctx().bvh_on && !(d->flags & LRT_F_NO_BVH) && !use_grid;
    if (use_grid)
        if (int rc = ensure_grid(ctx())) return rc;
    if (use_bvh)
        if (int rc = ensure_bvh(ctx())) return rc;
    a.bv = ctx().bvh;
    a.bv.on = use_bvh ? 1 : 0;
    a.gv = ctx().gv;
    a.gv.on = use_grid ? 1 : 0;
    a.bvh_stack_offset = 0;
    const bool lds = !(d->flags & LRT_F_SCENE_GLOBAL) &&
                     sizeof(float4) * (kTraceLdsLevels * kBlock + 4 * (size_t)a.count + a.nlights / 4 + 1) <= 64 * 1024;
    // Kernel policy (auto_kernel, measured): v5 (pool) for calls with >= 4 frames and >= 2
    // tiles per resident wave, v0 otherwise; v4 (wavefront) stays selectable for A/B. The
    // round-1 per-lane state machines (v1/v2/v2s) and round-1's v3 regeneration kernel (slower
    // than v0 or v5 on every config) were removed: their flags are rejected.
    a.regenMin = 0;
    a.lateFetch = 0;
    a.lerp = ctx().d_lerp;
    a.colbuf = nullptr;
    a.poolSlots = 0;
    a.perm = nullptr;
    a.tcost = nullptr;
    a.samp = colours_out;
    a.sampOnly = colours_out ? 1 : 0;
    a.frame = reinterpret_cast<float4*>(frame);
    if (frame && (want_feat || colours_out))
        return fail(LRT_E_INVALID, "a frame destination is for plain renders (no features, no colours-only)");
    if (colours_out) {   // v0, one frame lane per pixel, sample mode
        if (want_feat || !lds || a.bv.on || a.gv.on) return fail(LRT_E_INVALID, "colours-only render: LDS linear-scan scenes only");
        if (d->max_depth <= 8) return launch_v0_d8(a, lds, d->x_count, d->row_count, d->frames, false, true, s);
        return launch_v0_d64(a, lds, d->x_count, d->row_count, d->frames, false, true, s);
    }
    int kflags = d->flags & (LRT_F_SIMPLE | LRT_F_WAVEFRONT | LRT_F_POOL);
    // Pool tiles: 64 px, or 128 px when another stream's pool launch is still running, i.e. this
    // launch will overlap it. A 128-px tile is a pool of twice the samples, so a pool's drain (its
    // last paths finishing with most lanes idle) is paid half as often, but with ~1.8 tiles per
    // wave the launch's own tail grows; beside another launch that tail is filled (config 2 two
    // streams 0.2237 -> 0.2104 ms/step, one stream 0.2564 -> 0.2717 with 128 px, profiles/r6_k).
#ifndef LRT_POOL_PIX_ALONE
#define LRT_POOL_PIX_ALONE 64   // (A/B builds: the tile cap of a launch alone)
#endif
    int pix_cap = LRT_POOL_PIX_ALONE;
    a.split16 = kPoolSplit16Alone;
    if (!(kflags & (LRT_F_SIMPLE | LRT_F_WAVEFRONT)) && d->frames >= 4) {
        bool busy = false;
        if (const hipError_t e = other_stream_busy(s, &busy)) return hip_fail(e, "pool launch events");
        if (busy) {
            pix_cap = kPoolPixOverlap;
            a.split16 = kPoolSplit16Overlap;
        }
    }
    if (kflags == 0) kflags = auto_kernel(a, d, want_feat, pix_cap);
    if (want_feat && !(kflags & LRT_F_SIMPLE))
        return fail(LRT_E_INVALID, "features are implemented by the v0 kernel only");
    if (kflags & LRT_F_WAVEFRONT) return launch_wavefront(a, lds, s);
    if (kflags & LRT_F_POOL) {
        a.colbuf = nullptr;
        if (d->max_depth <= 8) return launch_pool_d8(a, lds, d->x_count, d->row_count, d->frames, pix_cap, s);
        return launch_pool_d64(a, lds, d->x_count, d->row_count, d->frames, pix_cap, s);
    }
    if (d->max_depth <= 8) return launch_v0_d8(a, lds, d->x_count, d->row_count, d->frames, want_feat, false, s);
    // depth 9..64: one instance (MAXD only decides whether stack levels beyond the 8 in LDS
    // exist; 20 and 64 compiled to the same code)
    return launch_v0_d64(a, lds, d->x_count, d->row_count, d->frames, want_feat, false, s);
}

// The library's kernel policy (measured, profiles/r2_p2, r2_p9, r3_t): the pool kernel (v5) given
// at least 4 frames and a tile per resident wave -- BVH scenes (config 4: 223 vs 303
// ms, config 5), bounce budgets above 8 (config 3: 2.45 vs 2.87 ms) and, with its
// heaviest-first tile order (tile_order), the 8-bounce default scene too (config 2: 0.254 vs
// 0.289 ms/step, 0.297 vs 0.329 ms for a launch alone); v0 otherwise (few pixels with many
// frames, a GPU's row shard, take v0's frame lanes and sample mode; features are v0's).
int auto_kernel(const KernelArgs& a, const lrt_render_desc* d, bool feat, int pix_cap) {
    if (feat || d->frames < 4) return LRT_F_SIMPLE;
    if (!(a.bv.on || a.gv.on || d->max_depth > 8) && !pool_order_on()) return LRT_F_SIMPLE;
    const int pix = pool_pixels(d->frames, d->x_count, d->row_count, pix_cap);
    const long long tiles = pool_tiles(pix, d->x_count, d->row_count);
    const long long slots = 16LL * ctx().num_cus;   // resident waves (4 per SIMD)
    // at least a tile per resident wave: config 2's row shard of 2 (7,200 tiles) runs 0.1316 ms
    // on the pool kernel against 0.1473 on v0; a shard of 4 (3,680 tiles) 0.1456 against 0.0773
    // (profiles/r3_t)
    return tiles >= slots ? LRT_F_POOL : LRT_F_SIMPLE;
}

}  // namespace lrt
