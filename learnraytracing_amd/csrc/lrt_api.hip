// liblrt_hip.so -- the MI355X path tracer behind the C-ABI of include/lrt.h (the reference's
// renderer API, parallel.h:6-8, plus the extended boundary). This unit holds the globals, the
// per-device contexts and the entry points that only dispatch; lrt_internal.h lists the others.
#include "lrt_internal.h"

namespace lrt {

Context g_devs[kMaxDevices];
int g_ndev = 0;
int g_cur = 0;
Multi g_multi;
std::mutex g_mu;
char g_last_launch[256] = "";
thread_local std::string t_err;
thread_local std::string t_launch;   // lrt_last_launch()'s copy for the calling thread

int fail(int code, const std::string& msg) {
    t_err = msg;
    return code;
}
int hip_fail(hipError_t e, const char* what) {
    return fail(LRT_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// A device's context: its stream, counters, lerp table and the default scene (lrt_initialize,
// and each device of lrt_initialize_devices; the device is current).
int init_context(Context& c, int dev) {
    c = Context();
    c.device = dev;
    LRT_HIP(hipDeviceGetAttribute(&c.num_cus, hipDeviceAttributeMultiprocessorCount, dev));
    // The context's streams are created together, first, the render stream at high priority.
    // HIP deals a process's streams to a few hardware queues (GPU_MAX_HW_QUEUES = 4), and
    // DrawTest's lerps (stream), copies (s_in) and look-ahead render (a CU-masked stream) must
    // not queue behind one another: created lazily, between other streams, they did on some
    // offsets -- a pageable DrawTest at 1280x720 took 0.67-0.77 ms/frame instead of 0.49-0.52
    // (tools/drawtest_queues.py, profiles/r4_m); a high-priority queue is one no stream of normal
    // priority shares.
    {
        int least = 0, greatest = 0;
        LRT_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        LRT_HIP(hipStreamCreateWithPriority(&c.stream, hipStreamNonBlocking, greatest));
        LRT_HIP(hipStreamCreateWithPriority(&c.s_in, hipStreamNonBlocking, least));
    }
    if (int rc = create_lookahead_stream(c)) return rc;
    for (int k = 0; k < Context::kHostChunks; ++k) LRT_HIP(hipEventCreateWithFlags(&c.ev_in[k], hipEventDisableTiming));
    LRT_HIP(hipEventCreateWithFlags(&c.ev_ret, hipEventDisableTiming));
    LRT_HIP(hipMalloc(&c.d_rays, sizeof(unsigned long long)));
    LRT_HIP(hipHostMalloc((void**)&c.h_rays, sizeof(unsigned long long), hipHostMallocDefault));
    LRT_HIP(hipMalloc(&c.d_tiles, sizeof(unsigned long long) * kQueueSlots * kTileSetU64));
    LRT_HIP(hipMemset(c.d_tiles, 0, sizeof(unsigned long long) * kQueueSlots * kTileSetU64));
    {   // parallel.cpp:262's lerpFac per frame number, divided once here instead of per wave
        std::vector<float> t(kLerpTable);
        for (int f = 0; f < kLerpTable; ++f) t[f] = (float)f / (float)(f + 1);
        LRT_HIP(hipMalloc(&c.d_lerp, sizeof(float) * kLerpTable));
        LRT_HIP(hipMemcpy(c.d_lerp, t.data(), sizeof(float) * kLerpTable, hipMemcpyHostToDevice));
    }
    {   // keep freed stream-ordered blocks (the per-launch path-stack overflow) in the
        // pool instead of returning them to the driver at every synchronisation
        hipMemPool_t pool;
        if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
            uint64_t keep = UINT64_MAX;
            (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
        }
    }
    if (int rc = upload_scene(c, kDefaultSpheres, kDefaultMats, 9)) return rc;
    c.ready = true;
    return LRT_OK;
}

// Frees everything init_context and the render paths allocated (the device is current).
void free_context(Context& c) {
    if (c.stream) (void)hipStreamSynchronize(c.stream);
    (void)hipDeviceSynchronize();
    free_scene(c);
    for (float* p : {c.d_frame, c.d_shard, c.d_gath, c.d_pack})
        if (p) (void)hipFree(p);
    if (c.h_rays) (void)hipHostFree(c.h_rays);
    if (c.d_rays) (void)hipFree(c.d_rays);
    if (c.d_tiles) (void)hipFree(c.d_tiles);
    if (c.d_lerp) (void)hipFree(c.d_lerp);
    if (c.wf.buf) (void)hipFree(c.wf.buf);
    if (c.wf.rayp) (void)hipFree(c.wf.rayp);
    for (auto* f : c.d_feat)
        if (f) (void)hipFree(f);
    for (auto& m : c.masked_streams) (void)hipStreamDestroy(m.first);
    if (c.d_col) (void)hipFree(c.d_col);
    for (auto& sc : c.scratch) {
        if (sc.p) (void)hipFree(sc.p);
        if (sc.ev) (void)hipEventDestroy(sc.ev);
    }
    for (auto& o : c.order) {
        if (o.d_base) (void)hipFree(o.d_base);
        if (o.ev_rec) (void)hipEventDestroy(o.ev_rec);
        for (auto& u : o.uses) (void)hipEventDestroy(u.second);
    }
    for (int k = 0; k < Context::kHostChunks; ++k)
        if (c.ev_in[k]) (void)hipEventDestroy(c.ev_in[k]);
    if (c.ev_ret) (void)hipEventDestroy(c.ev_ret);
    for (int k = 0; k < 2; ++k)
        if (c.ahead.col[k]) (void)hipFree(c.ahead.col[k]);
    if (c.ahead.d_rays) (void)hipFree(c.ahead.d_rays);
    if (c.ahead.ev) (void)hipEventDestroy(c.ahead.ev);
    if (c.ahead.ev_render) (void)hipEventDestroy(c.ahead.ev_render);
    // (c.ahead.stream is one of c.masked_streams, destroyed with them)
    if (c.ev_done) (void)hipEventDestroy(c.ev_done);
    if (c.s_in) (void)hipStreamDestroy(c.s_in);
    if (c.stream) (void)hipStreamDestroy(c.stream);
    c = Context();
}

}  // namespace lrt

using namespace lrt;

extern "C" {

const char* lrt_last_error(void) { return t_err.c_str(); }

const char* lrt_version(void) { return LRT_VERSION_STRING; }

const char* lrt_last_launch(void) {
    // a copy taken under the lock: render calls on other threads rewrite g_last_launch
    std::lock_guard<std::mutex> lk(g_mu);
    t_launch = g_last_launch;
    return t_launch.c_str();
}

int lrt_initialize(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ndev > 0) return LRT_OK;
    int dev = 0;
    LRT_HIP(hipGetDevice(&dev));
    g_cur = 0;
    const int rc = init_context(g_devs[0], dev);
    if (rc) {
        free_context(g_devs[0]);
        return rc;
    }
    g_ndev = 1;
    g_multi = Multi();
    return LRT_OK;
}

int lrt_device_count(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_ndev;
}

int lrt_shutdown(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ndev == 0) return LRT_OK;
    if (g_multi.rccl)
        for (int k = 0; k < g_ndev; ++k) (void)ncclCommDestroy(g_multi.comms[k]);
    for (int k = 0; k < g_ndev; ++k) {
        DeviceScope ds(k);
        free_context(g_devs[k]);
    }
    g_ndev = 0;
    g_cur = 0;
    g_multi = Multi();
    return LRT_OK;
}

int lrt_draw_test(float time, int frameCount, int screenWidth, int screenHeight, float* backbuffer,
                  int* outRayCount) {
    RoctxRange rr_("lrt_draw_test");
    (void)time;   // unused by the reference too (JobData::time, parallel.cpp:244)
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);   // context 0's device (device 0 of lrt_initialize_devices)
    lrt_render_desc d;
    memset(&d, 0, sizeof(d));
    int rc = camera_default(screenWidth, screenHeight, &d.camera);
    if (rc) return rc;
    d.width = screenWidth;
    d.height = screenHeight;
    d.x0 = 0;
    d.x_count = screenWidth;
    d.y0 = 0;
    d.row_count = screenHeight;
    d.row_block = screenHeight;
    d.row_period = 1;
    d.row_phase = 0;
    d.frame0 = frameCount;
    d.frames = 1;
    d.max_depth = LRT_REFERENCE_MAX_DEPTH;
    long long rays = 0;
    rc = render_host(&d, backbuffer, &rays, nullptr, true);
    if (rc) return rc;
    if (outRayCount) *outRayCount = (int)rays;
    return LRT_OK;
}

int lrt_camera_make(lrt_float3 lookFrom, lrt_float3 lookAt, lrt_float3 vup, float vfov, float aspect,
                    float aperture, float focusDist, lrt_camera* out) {
    return camera_make(lookFrom, lookAt, vup, vfov, aspect, aperture, focusDist, out);
}

int lrt_camera_default(int width, int height, lrt_camera* out) { return camera_default(width, height, out); }

int lrt_set_scene(const lrt_sphere* spheres, const lrt_material* materials, int count) {
    RoctxRange rr_("lrt_set_scene");
    std::lock_guard<std::mutex> lk(g_mu);
    if (!ctx().ready) return fail(LRT_E_STATE, "lrt_initialize() has not been called");
    for (int k = 0; k < g_ndev; ++k) {   // every device in use holds the scene
        DeviceScope ds(k);
        LRT_HIP(hipStreamSynchronize(ctx().stream));
        LRT_HIP(hipDeviceSynchronize());
        if (int rc = upload_scene(ctx(), spheres, materials, count)) return rc;
    }
    return LRT_OK;
}

int lrt_get_scene(lrt_sphere* spheres, lrt_material* materials, int capacity, int* count) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!ctx().ready) return fail(LRT_E_STATE, "lrt_initialize() has not been called");
    const int n = (int)ctx().spheres.size();
    if (count) *count = n;
    if (!spheres || !materials || capacity < n) return fail(LRT_E_INVALID, "need capacity >= the scene's sphere count");
    memcpy(spheres, ctx().spheres.data(), sizeof(lrt_sphere) * n);
    memcpy(materials, ctx().mats.data(), sizeof(lrt_material) * n);
    return LRT_OK;
}

int lrt_default_scene(lrt_sphere* spheres, lrt_material* materials, int capacity, int* count) {
    if (count) *count = 9;
    if (capacity < 9 || !spheres || !materials) return fail(LRT_E_INVALID, "need capacity >= 9");
    memcpy(spheres, kDefaultSpheres, sizeof(kDefaultSpheres));
    memcpy(materials, kDefaultMats, sizeof(kDefaultMats));
    return LRT_OK;
}

int lrt_render_device(const lrt_render_desc* desc, float* d_backbuffer, unsigned long long* d_rays, void* stream) {
    RoctxRange rr_("lrt_render_device");
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);   // context 0's device (device 0 of lrt_initialize_devices)
    return render_device(desc, d_backbuffer, d_rays, nullptr, (hipStream_t)stream);
}

int lrt_render_device_to_frame(const lrt_render_desc* desc, float* d_backbuffer, unsigned long long* d_rays,
                               float* d_frame, void* stream) {
    RoctxRange rr_("lrt_render_device_to_frame");
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);
    if (!d_frame) return fail(LRT_E_INVALID, "d_frame is NULL");
    return render_device(desc, d_backbuffer, d_rays, nullptr, (hipStream_t)stream, nullptr, d_frame);
}

int lrt_render_device_ex(const lrt_render_desc* desc, float* d_backbuffer, unsigned long long* d_rays,
                         const lrt_features* d_features, void* stream) {
    RoctxRange rr_("lrt_render_device_ex");
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);   // context 0's device (device 0 of lrt_initialize_devices)
    return render_device(desc, d_backbuffer, d_rays, d_features, (hipStream_t)stream);
}

int lrt_render_host_ex(const lrt_render_desc* desc, float* backbuffer, long long* out_rays,
                       const lrt_features* features) {
    RoctxRange rr_("lrt_render_host_ex");
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);   // context 0's device (device 0 of lrt_initialize_devices)
    return render_host(desc, backbuffer, out_rays, features);
}

int lrt_render_host(const lrt_render_desc* desc, float* backbuffer, long long* out_rays) {
    RoctxRange rr_("lrt_render_host");
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);   // context 0's device (device 0 of lrt_initialize_devices)
    return render_host(desc, backbuffer, out_rays);
}

int lrt_stream_create(int reserved_cus, void** out) {
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);
    if (!ctx().ready) return fail(LRT_E_STATE, "lrt_initialize() has not been called");
    if (!out) return fail(LRT_E_INVALID, "stream out is NULL");
    const int n = ctx().num_cus;
    if (reserved_cus < 0 || reserved_cus >= n) return fail(LRT_E_INVALID, "reserved_cus must be in [0, CU count)");
    // the last reserved_cus logical CUs stay free; hipExtStreamCreateWithCUMask takes one
    // bit per CU, 32 per word
    std::vector<uint32_t> mask((size_t)(n + 31) / 32, 0u);
    // Logical CU c sits on XCD c % 8 (measured: reserving CUs 31, 63, ... -- all on one XCD
    // -- slows a full-chip render 20-70 %, because workgroups are dealt to XCDs round-robin),
    // so the last reserved_cus logical CUs spread the reservation evenly over the XCDs.
    int kept = 0;
    for (int c = 0; c < n - reserved_cus; ++c) {
        mask[c / 32] |= 1u << (c % 32);
        ++kept;
    }
    hipStream_t st = nullptr;
    LRT_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
    ctx().masked_streams.emplace_back(st, kept);
    *out = st;
    return LRT_OK;
}

int lrt_host_alloc(size_t bytes, void** out) {
    if (!out) return fail(LRT_E_INVALID, "out is NULL");
    *out = nullptr;
    if (bytes == 0) return fail(LRT_E_INVALID, "bytes must be > 0");
    if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) {
        *out = nullptr;
        return fail(LRT_E_NOMEM, "hipHostMalloc failed");
    }
    return LRT_OK;
}

int lrt_host_free(void* p) {
    if (!p) return LRT_OK;
    LRT_HIP(hipHostFree(p));
    return LRT_OK;
}

int lrt_stream_destroy(void* stream) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto& v = ctx().masked_streams;
    for (size_t i = 0; i < v.size(); ++i)
        if (v[i].first == (hipStream_t)stream) {
            (void)hipStreamSynchronize(v[i].first);
            LRT_HIP(hipStreamDestroy(v[i].first));
            v.erase(v.begin() + (long)i);
            return LRT_OK;
        }
    return fail(LRT_E_INVALID, "not a stream from lrt_stream_create");
}

}  // extern "C"
