// Host backbuffers (lrt_draw_test, lrt_render_host): the staged path, zero copy and the
// pipelined path for page-locked buffers with DrawTest's look-ahead render.
#include "lrt_internal.h"

namespace lrt {

// The pipelined host path's lerp (render_host_pipelined): prev from device memory (copied
// there by DMA while the colours were rendered), the result written straight into the
// caller's page-locked pixels over PCIe (posted writes; no D2H copy command).
__global__ __launch_bounds__(256) void merge_to_host_kernel(const float4* __restrict__ samp,
                                                            const float4* __restrict__ prev, float4* host,
                                                            const float* lerp, int npix, int frame0, int frames,
                                                            size_t stride) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < npix; i += gridDim.x * blockDim.x) {
        const float4 o = prev[i];
        F3 acc = f3(o.x, o.y, o.z);
        for (int k = 0; k < frames; ++k) {   // parallel.cpp:262,282 in frame order
            const float4 c = samp[(size_t)k * stride + i];
            const int f = frame0 + k;
            const float lerpFac = f < kLerpTable ? lerp[f] : (float)f / (float)(f + 1);
            acc = acc * lerpFac + f3(c.x, c.y, c.z) * (1.0f - lerpFac);
        }
        host[i] = make_float4(acc.x, acc.y, acc.z, o.w);   // alpha as read
    }
}


int ensure_frame(size_t bytes) {
    if (ctx().frame_bytes >= bytes) return LRT_OK;
    if (ctx().d_frame) (void)hipFree(ctx().d_frame);
    ctx().d_frame = nullptr;
    ctx().frame_bytes = 0;
    if (hipMalloc(&ctx().d_frame, bytes) != hipSuccess) return fail(LRT_E_NOMEM, "hipMalloc(frame) failed");
    ctx().frame_bytes = bytes;
    return LRT_OK;
}

// The device address of buf when it is page-locked host memory (hipHostMalloc /
// hipHostRegister, e.g. a torch pin_memory tensor), else nullptr.
float* host_pinned(float* buf) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, buf) != hipSuccess) {
        (void)hipGetLastError();   // pageable memory: clear the error so no later check sees it
        return nullptr;
    }
    if (at.type != hipMemoryTypeHost) return nullptr;
    return at.devicePointer ? (float*)at.devicePointer : buf;
}

// A pageable backbuffer is page-locked for the duration of ONE call (HostLock): registered
// when the call starts, unregistered before it returns, after every copy and kernel that
// touches it has completed. The reference's caller owns its buffer across calls and may free
// it and allocate another -- even at the same address -- between any two calls (parallel.h:8
// has no unregister hook), so the library keeps no registration, no pointer and no pages
// from one call to the next. Registering the 14.7 MB of a 1280x720 frame costs microseconds
// (profiles/r4_b: tools/hostreg_probe.hip, which also remaps the same address between calls
// and checks the device reads and writes the new pages), and turns the call's copies into
// true DMA and its lerp into posted PCIe writes (the page-locked paths below) instead of the
// runtime's bounce buffers (staged: 0.77 ms per frame). A buffer the caller page-locked
// itself is used as it is. LRT_HOST_REGISTER=0: pageable buffers stay staged.
bool host_register_on() {
    static const bool on = [] {
        const char* e = getenv("LRT_HOST_REGISTER");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

struct HostLock {
    void* p = nullptr;   // registered by this call (nullptr: nothing to undo)
    float* dev = nullptr;
    // the device address of buf's page-locked pages for this call, or nullptr (staged path)
    float* acquire(float* buf, size_t bytes) {
        if (!host_register_on()) return nullptr;
        if (hipHostRegister(buf, bytes, hipHostRegisterPortable | hipHostRegisterMapped) != hipSuccess) {
            (void)hipGetLastError();   // e.g. part of the range is registered already: stay staged
            return nullptr;
        }
        p = buf;
        dev = host_pinned(buf);
        if (!dev) release();
        return dev;
    }
    // Unregisters once nothing in flight can touch the pages: the call's copies and lerps run on
    // the context's stream and copy stream (idle by now on the normal path; on an error path
    // this waits for what was enqueued). The look-ahead stream never touches them.
    int release() {
        if (!p) return LRT_OK;
        (void)hipStreamSynchronize(ctx().stream);
        if (ctx().s_in) (void)hipStreamSynchronize(ctx().s_in);
        const hipError_t e = hipHostUnregister(p);
        p = nullptr;
        dev = nullptr;
        return e == hipSuccess ? LRT_OK : hip_fail(e, "hipHostUnregister");
    }
    ~HostLock() { (void)release(); }
};

// Page-locked host backbuffers are rendered in place (zero copy): the kernel's 16 B read
// and 16 B write per pixel cross PCIe inside the launch instead of a staging copy either
// side of it (DrawTest at 1280x720: 0.66 ms per frame vs 0.77 staged; staging in row chunks
// on copy streams measured 0.84 ms at 4 chunks -- per-chunk launch tails and cross-stream
// waits; staging only the previous values and letting the kernel write the host pixels
// measured 0.64 ms, within noise of this). LRT_HOST_ZEROCOPY=0 stages them like pageable memory.
bool host_zero_copy() {
    static const bool on = [] {
        const char* e = getenv("LRT_HOST_ZEROCOPY");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

// The pipelined host path for page-locked backbuffers (lrt_draw_test at 1280x720 is
// PCIe-bound). The sample colours do not depend on the buffer's previous values -- only the
// lerp does (parallel.cpp:282) -- so the colours are rendered into device memory while the
// previous values travel host -> device by DMA (LRT_HOST_CHUNKS row chunks on a copy
// stream); each chunk's lerp runs once its copy lands and writes the result straight into
// the caller's pixels over PCIe, while the next chunk's copy comes the other way. Measured
// alternatives (profiles/r2_p2): zero copy for the whole render (kernel reads and writes
// over PCIe, 0.66 ms; GPU-initiated reads and writes share ~64 GB/s); render + one
// streaming zero-copy lerp (0.70 ms); DMA both ways in 8 chunks (0.72 ms: ~20 us per copy
// command, and D2H ran as blit kernels). Pageable buffers stay staged (their async copies
// go through bounce buffers: 1.2 ms pipelined vs 0.77 staged). LRT_HOST_PIPELINE=0: off.
bool host_pipeline(const lrt_render_desc* d, size_t bytes) {
    static const int mode = [] {
        const char* e = getenv("LRT_HOST_PIPELINE");
        return e ? atoi(e) : 1;
    }();
    // (an accelerated scene: the BVH, or the grid where render_device would pick it)
    const bool bvh = !(d->flags & LRT_F_NO_BVH) &&
                     (ctx().bvh_on || (ctx().grid_ok && (ctx().grid_pick || (d->flags & LRT_F_GRID))));
    const bool lds = !(d->flags & LRT_F_SCENE_GLOBAL) &&
                     sizeof(float4) * (kTraceLdsLevels * kBlock + 4 * (size_t)ctx().count + ctx().nlights / 4 + 1) <=
                         64 * 1024;
    const int kflags = d->flags & (LRT_F_SIMPLE | LRT_F_WAVEFRONT | LRT_F_POOL);
    return mode != 0 && d->frames <= 4 && bytes * (size_t)d->frames <= (256u << 20) && !bvh && lds &&
           (kflags == 0 || kflags == LRT_F_SIMPLE) && !(d->flags & LRT_F_NO_DOUBLE_LIGHT) &&
           d->row_count >= Context::kHostChunks;
}

// Row chunks of the DMA copy (LRT_HOST_CHUNKS, 1..8; default 4 for DrawTest's look-ahead calls,
// whose lerps follow the copy chunk by chunk: 0.47 vs 0.50 ms at 2; 2 otherwise, where the
// render sets the pace: 0.53 vs 0.54 ms at 4 -- profiles/r3_m, r3_o).
int host_chunks(bool lookahead) {
    static const int k = [] {
        const char* e = getenv("LRT_HOST_CHUNKS");
        const int v = e ? atoi(e) : 0;
        return v < 0 ? 1 : v > Context::kHostChunks ? Context::kHostChunks : v;
    }();
    return k > 0 ? k : lookahead ? 4 : 2;
}

// lrt_draw_test's look-ahead (LRT_DRAW_LOOKAHEAD, default on). DrawTest's colours depend on
// frameCount, the size and the scene only (parallel.cpp:297-323: `time` is unused, the camera
// is rebuilt from the size), and the reference's caller asks for frameCount + 1 next
// (main.cpp:165,187). So a pipelined DrawTest call also renders the colours of the next
// frame, on a stream of their own that runs beside this call's DMA and PCIe-write lerps (a
// hit: from the call's start; a miss: after its own render), CU-masked so that the lerps
// still find CUs (32 = 4 per XCD; 0-32 within 0.01 ms pinned, 32 best pageable:
// profiles/r3_o); the call returns once its
// own work is done. A later call asking for exactly that render (desc and scene version
// compared) lerps those colours and skips its render, so the render leaves the critical
// path (DMA in -> lerp -> PCIe out); any other call renders as before. Same kernel, same
// seeds: the same bits. Two colour buffers alternate (one read by this call's lerps, the
// other written by the next look-ahead).
bool draw_lookahead_on() {
    static const bool on = [] {
        const char* e = getenv("LRT_DRAW_LOOKAHEAD");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

int lookahead_reserved_cus() { return 32; }

// The look-ahead's CU-masked stream and events (init_context creates them beside the context's
// other streams, so that each has a hardware queue of its own).
int create_lookahead_stream(Context& c) {
    Context::Lookahead& la = c.ahead;
    if (la.stream || !draw_lookahead_on()) return LRT_OK;
    const int n = c.num_cus, keep = std::max(1, n - std::max(0, lookahead_reserved_cus()));
    std::vector<uint32_t> mask((size_t)(n + 31) / 32, 0u);
    for (int k = 0; k < keep; ++k) mask[k / 32] |= 1u << (k % 32);   // spread over XCDs (k % 8)
    LRT_HIP(hipExtStreamCreateWithCUMask(&la.stream, (uint32_t)mask.size(), mask.data()));
    c.masked_streams.emplace_back(la.stream, keep);
    LRT_HIP(hipEventCreateWithFlags(&la.ev, hipEventDisableTiming));
    LRT_HIP(hipEventCreateWithFlags(&la.ev_render, hipEventDisableTiming));
    return LRT_OK;
}

// The lerp grid: a few blocks per CU, each striding over the chunk (posted PCIe writes need
// no more in flight; a full grid would wait for CUs behind the look-ahead render)
unsigned merge_blocks(size_t n) {
    const size_t want = (n + 255) / 256, cap = (size_t)4 * ctx().num_cus;
    return (unsigned)std::max<size_t>(1, std::min(want, cap));
}

int render_host_pipelined(const lrt_render_desc* d, float* buf, float* hdev, size_t bytes, long long* out_rays,
                          bool lookahead, int* ahead_state) {
    hipStream_t s = ctx().stream;
    Context::Lookahead& la = ctx().ahead;
    if (!ctx().s_in) {
        LRT_HIP(hipStreamCreateWithFlags(&ctx().s_in, hipStreamNonBlocking));
        for (int c = 0; c < Context::kHostChunks; ++c)
            LRT_HIP(hipEventCreateWithFlags(&ctx().ev_in[c], hipEventDisableTiming));
        LRT_HIP(hipEventCreateWithFlags(&ctx().ev_ret, hipEventDisableTiming));
    }
    const size_t cbytes = bytes * (size_t)d->frames;
    // a hit: the look-ahead rendered exactly this (this call's lerps wait for its event)
    const bool hit = la.on && la.scene_version == ctx().scene_version && memcmp(&la.d, d, sizeof(*d)) == 0;
    la.on = false;
    *ahead_state = hit ? 1 : 0;
    if (!hit && ctx().col_bytes < cbytes) {
        if (ctx().d_col) (void)hipFree(ctx().d_col);
        ctx().d_col = nullptr;
        ctx().col_bytes = 0;
        if (hipMalloc(&ctx().d_col, cbytes) != hipSuccess) return fail(LRT_E_NOMEM, "hipMalloc(sample colours)");
        ctx().col_bytes = cbytes;
    }
    const bool ahead_on = lookahead && draw_lookahead_on() && d->frames == 1 && d->frame0 < INT_MAX - 1;
    const int K = host_chunks(ahead_on || hit), rows = d->row_count, xc = d->x_count;
    const size_t npix = (size_t)xc * rows;
    auto chunk = [&](int c, size_t& p0, size_t& n) {   // chunk c: rows [c rows / K, (c + 1) rows / K)
        const size_t r0 = (size_t)rows * c / K, r1 = (size_t)rows * (c + 1) / K;
        p0 = r0 * xc;
        n = (r1 - r0) * xc;
    };
    for (int c = 0; c < K; ++c) {   // previous values, host -> device (DMA), beside the render
        size_t p0, n;
        chunk(c, p0, n);
        LRT_HIP(hipMemcpyAsync(ctx().d_frame + 4 * p0, buf + 4 * p0, n * 16, hipMemcpyHostToDevice, ctx().s_in));
        LRT_HIP(hipEventRecord(ctx().ev_in[c], ctx().s_in));
    }
    float4* col = hit ? la.col[la.cur] : ctx().d_col;
    unsigned long long* d_rays = hit ? la.d_rays + la.cur : ctx().d_rays;
    if (hit) {
        LRT_HIP(hipStreamWaitEvent(s, la.ev, 0));
    } else {
        LRT_HIP(hipMemsetAsync(d_rays, 0, sizeof(unsigned long long), s));
        int rc = render_device(d, ctx().d_frame, d_rays, nullptr, s, col);
        if (rc) {
            (void)hipStreamSynchronize(ctx().s_in);
            return rc;
        }
    }
    if (ahead_on) {
        // the next frame's colours into the buffer pair this call does not read
        const int nx = hit ? la.cur ^ 1 : la.cur;
        lrt_render_desc nd = *d;
        nd.frame0 = d->frame0 + 1;
        bool ok = la.stream || create_lookahead_stream(ctx()) == LRT_OK;
        if (ok && la.bytes[nx] < cbytes) {
            if (la.col[nx]) (void)hipFree(la.col[nx]);
            la.col[nx] = nullptr;
            la.bytes[nx] = 0;
            ok = hipMalloc(&la.col[nx], cbytes) == hipSuccess;
            if (ok) la.bytes[nx] = cbytes;
        }
        if (ok && !la.d_rays) ok = hipMalloc(&la.d_rays, 2 * sizeof(unsigned long long)) == hipSuccess;
        // a miss: after this call's own render (the two would share the CUs it needs)
        if (ok && !hit)
            ok = hipEventRecord(la.ev_render, s) == hipSuccess && hipStreamWaitEvent(la.stream, la.ev_render, 0) == hipSuccess;
        if (ok) ok = hipMemsetAsync(la.d_rays + nx, 0, sizeof(unsigned long long), la.stream) == hipSuccess;
        char keep[sizeof(g_last_launch)];   // the launch string stays this call's
        memcpy(keep, g_last_launch, sizeof(keep));
        if (ok) ok = render_device(&nd, ctx().d_frame, la.d_rays + nx, nullptr, la.stream, la.col[nx]) == LRT_OK;
        memcpy(g_last_launch, keep, sizeof(keep));
        if (ok) ok = hipEventRecord(la.ev, la.stream) == hipSuccess;
        if (ok) {
            la.on = true;
            la.cur = nx;
            la.d = nd;
            la.scene_version = ctx().scene_version;
        } else {
            (void)hipGetLastError();   // no look-ahead: the next call renders for itself
        }
    }
    for (int c = 0; c < K; ++c) {   // each chunk's lerp once its values are in, written to the host pixels
        size_t p0, n;
        chunk(c, p0, n);
        LRT_HIP(hipStreamWaitEvent(s, ctx().ev_in[c], 0));
        merge_to_host_kernel<<<merge_blocks(n), 256, 0, s>>>(
            col + p0, reinterpret_cast<const float4*>(ctx().d_frame) + p0, reinterpret_cast<float4*>(hdev) + p0,
            ctx().d_lerp, (int)n, d->frame0, d->frames, npix);
        LRT_HIP(hipGetLastError());
    }
    unsigned long long rays = 0;
    LRT_HIP(hipMemcpyAsync(&rays, d_rays, sizeof(rays), hipMemcpyDeviceToHost, s));
    LRT_HIP(hipEventRecord(ctx().ev_ret, s));
    LRT_HIP(hipEventSynchronize(ctx().ev_ret));
    if (out_rays) *out_rays = (long long)rays;
    return LRT_OK;
}

// drawtest: the reference API's call (lrt_draw_test), whose caller asks for frameCount + 1 next
// (main.cpp:165,187): the pipelined path renders that frame's colours ahead (the look-ahead).
int render_host(const lrt_render_desc* d, float* buf, long long* out_rays, const lrt_features* feat,
                bool drawtest) {
    int rc = validate(d);
    if (rc) return rc;
    if (!ctx().ready) return fail(LRT_E_STATE, "lrt_initialize() has not been called");
    if (!buf) return fail(LRT_E_INVALID, "backbuffer is NULL");
    const size_t bytes = (size_t)d->x_count * d->row_count * 4 * sizeof(float);
    if (bytes == 0 || d->frames == 0) {
        if (out_rays) *out_rays = 0;
        return LRT_OK;
    }
    // lrt_last_launch() names the host path too: host=pipelined | zerocopy | staged, with
    // "registered-" when this call page-locked a pageable buffer (HostLock)
    auto note = [](const char* path, bool registered) {
        const size_t n = strlen(g_last_launch);
        snprintf(g_last_launch + n, sizeof(g_last_launch) - n, " host=%s%s", registered ? "registered-" : "", path);
    };
    float* hdev = (!feat && host_zero_copy()) ? host_pinned(buf) : nullptr;
    HostLock lock;   // a pageable buffer, page-locked for this call only
    const bool registered = !hdev && !feat && host_zero_copy() && (hdev = lock.acquire(buf, bytes)) != nullptr;
    // lrt_initialize_devices: the caller's rows are split over every device (a window of
    // contiguous rows; a caller's own row-block-cyclic shard, or features, stay on device 0).
    // render_host_multi returns with every device's stream idle, so the lock may go.
    if (g_multi.on && d->row_period == 1 && !feat) {
        rc = render_host_multi(d, buf, bytes, out_rays);
        if (rc == LRT_OK) note(registered ? "registered-multi" : hdev ? "multi" : "pageable-multi", false);
        return rc;
    }
    if (hdev && host_pipeline(d, bytes)) {
        if ((rc = ensure_frame(bytes))) return rc;
        int ahead = 0;
        if ((rc = render_host_pipelined(d, buf, hdev, bytes, out_rays, drawtest, &ahead))) return rc;
        note("pipelined", registered);
        const size_t m = strlen(g_last_launch);
        snprintf(g_last_launch + m, sizeof(g_last_launch) - m, " lookahead=%s", ahead ? "hit" : "miss");
        return LRT_OK;
    }
    if (hdev) {   // zero copy: the kernel reads and writes the caller's pixels over PCIe
        LRT_HIP(hipMemsetAsync(ctx().d_rays, 0, sizeof(unsigned long long), ctx().stream));
        if ((rc = render_device(d, hdev, ctx().d_rays, nullptr, ctx().stream))) return rc;
        unsigned long long rays = 0;
        LRT_HIP(hipMemcpyAsync(&rays, ctx().d_rays, sizeof(rays), hipMemcpyDeviceToHost, ctx().stream));
        LRT_HIP(hipStreamSynchronize(ctx().stream));
        if (out_rays) *out_rays = (long long)rays;
        note("zerocopy", registered);
        return LRT_OK;
    }
    if ((rc = ensure_frame(bytes))) return rc;
    hipStream_t s = ctx().stream;
    LRT_HIP(hipMemcpyAsync(ctx().d_frame, buf, bytes, hipMemcpyHostToDevice, s));
    LRT_HIP(hipMemsetAsync(ctx().d_rays, 0, sizeof(unsigned long long), s));
    // host feature buffers go through device mirrors like the backbuffer
    lrt_features dfeat;
    memset(&dfeat, 0, sizeof(dfeat));
    float* const hp[6] = {feat ? feat->normal : nullptr,    feat ? feat->world_pos : nullptr,
                          feat ? feat->albedo : nullptr,    feat ? feat->color_std : nullptr,
                          feat ? feat->normal_std : nullptr, feat ? feat->world_pos_std : nullptr};
    float** const dp[6] = {&dfeat.normal, &dfeat.world_pos, &dfeat.albedo,
                           &dfeat.color_std, &dfeat.normal_std, &dfeat.world_pos_std};
    if (feat) {
        dfeat.max_frame = feat->max_frame;
        for (int k = 0; k < 6; ++k) {
            if (!hp[k]) continue;
            if (ctx().feat_bytes[k] < bytes) {
                if (ctx().d_feat[k]) (void)hipFree(ctx().d_feat[k]);
                ctx().d_feat[k] = nullptr;
                ctx().feat_bytes[k] = 0;
                if (hipMalloc(&ctx().d_feat[k], bytes) != hipSuccess) return fail(LRT_E_NOMEM, "hipMalloc(features)");
                ctx().feat_bytes[k] = bytes;
            }
            *dp[k] = ctx().d_feat[k];
            LRT_HIP(hipMemcpyAsync(ctx().d_feat[k], hp[k], bytes, hipMemcpyHostToDevice, s));
        }
    }
    if ((rc = render_device(d, ctx().d_frame, ctx().d_rays, feat ? &dfeat : nullptr, s))) return rc;
    unsigned long long rays = 0;
    LRT_HIP(hipMemcpyAsync(buf, ctx().d_frame, bytes, hipMemcpyDeviceToHost, s));
    for (int k = 0; k < 6; ++k)
        if (hp[k]) LRT_HIP(hipMemcpyAsync(hp[k], ctx().d_feat[k], bytes, hipMemcpyDeviceToHost, s));
    LRT_HIP(hipMemcpyAsync(&rays, ctx().d_rays, sizeof(rays), hipMemcpyDeviceToHost, s));
    LRT_HIP(hipStreamSynchronize(s));
    if (out_rays) *out_rays = (long long)rays;
    note("staged", false);
    return LRT_OK;
}

}  // namespace lrt
