// One process, several devices (lrt_initialize_devices): the caller's rows split over the
// devices and gathered by RCCL; and the per-process exchange's IPC frames (lrt_ipc_*).
#include "lrt_internal.h"

namespace lrt {

int ensure_buffer(float*& p, size_t& have, size_t bytes, const char* what) {
    if (have >= bytes) return LRT_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    have = 0;
    if (hipMalloc(&p, bytes) != hipSuccess) return fail(LRT_E_NOMEM, std::string("hipMalloc(") + what + ")");
    have = bytes;
    return LRT_OK;
}

// One host render split over the g_ndev devices of lrt_initialize_devices (BASELINE config 5:
// "row-tiled across 8xMI355X with RCCL gather over xGMI"). The caller's rows are dealt in
// blocks of g_multi.row_block rows round-robin (row-block-cyclic: contiguous bands are
// imbalanced); device k
//   1. receives the previous values of its rows from the caller's buffer (one strided DMA),
//   2. renders them densely into its shard buffer (lrt_render_desc's row map: row_period =
//      N, row_phase = k; any kernel the policy picks),
//   3. hands its rows back, by one of two exchanges:
//      * direct (the default): its own strided DMA straight into the caller's rows, over
//        its own PCIe link -- N links at once, no device in the middle;
//      * gather (LRT_DEV_GATHER, or LRT_DEV_PEER_COPY): the RGB of its shard (12 of the 16 B
//        per pixel: the render never writes alpha, parallel.cpp:283-285) to device 0 -- one
//        grouped ncclGather over RCCL (rccl.h:745) when the devices are distinct, device-to-
//        device copies when one is listed twice (RCCL refuses two ranks on one GPU) or with
//        LRT_DEV_PEER_COPY -- where unshard_rgb_kernel assembles the frame over a copy of the
//        caller's buffer (its alpha) and one DMA returns it.
// The caller's buffer is page-locked for the call (render_host), so every copy is a real DMA
// and every device's work is enqueued before the first blocking call: the devices overlap
// (advisor r3: pageable copies ran synchronously, one device after the other). Per-pixel seeds
// make the frame bit-identical to a 1-device render for any N, block size and exchange.
int render_host_multi_enqueue(const lrt_render_desc* d, float* buf, size_t bytes);
int render_host_multi(const lrt_render_desc* d, float* buf, size_t bytes, long long* out_rays) {
    const int rc = render_host_multi_enqueue(d, buf, bytes);
    long long total = 0;
    hipError_t first = hipSuccess;
    // every device's stream, also after a failure (advisor r4): nothing may still write the
    // counters or DMA to or from the caller's buffer once render_host unlocks it
    for (int k = 0; k < g_ndev; ++k) {
        DeviceScope ds(k);
        const hipError_t e = hipStreamSynchronize(ctx().stream);
        if (e != hipSuccess && first == hipSuccess) first = e;
        total += (long long)*ctx().h_rays;
    }
    if (rc) return rc;
    if (first != hipSuccess) return hip_fail(first, "hipStreamSynchronize(multi-device render)");
    snprintf(g_last_launch + strlen(g_last_launch), sizeof(g_last_launch) - strlen(g_last_launch),
             " devices=%d exchange=%s row_block=%d", g_ndev,
             !g_multi.gather ? "direct" : g_multi.rccl ? "rccl" : "copy", g_multi.row_block);
    if (out_rays) *out_rays = total;
    return LRT_OK;
}

// Bytes each exchange moves for an x_count x rows window over N devices (the CPU test of the
// exchange's size): direct = every shard's RGBA rows back over its own link; gather = the
// packed RGB of the shards into device 0 (the other devices' share crosses xGMI) plus the
// frame's RGBA down from device 0.
void multi_exchange_bytes(int xc, int rows, int b, int N, long long* direct, long long* gather_xgmi) {
    const int maxRows = lrt_shard_rows(rows, b, N, 0);
    *direct = (long long)xc * rows * 16;
    *gather_xgmi = (long long)(N - 1) * maxRows * xc * 12;
}

int render_host_multi_enqueue(const lrt_render_desc* d, float* buf, size_t bytes) {
    const int N = g_ndev, b = g_multi.row_block, xc = d->x_count, rows = d->row_count;
    const size_t rowBytes = (size_t)xc * 16;
    const int maxRows = lrt_shard_rows(rows, b, N, 0);
    const size_t shardBytes = (size_t)maxRows * rowBytes;
    const size_t packBytes = (size_t)maxRows * xc * 12;
    const size_t blk = (size_t)b * rowBytes;
    // shard row j is the caller's row (j / b) * b * N + k * b + j % b: whole blocks are one 2D
    // copy (pitch N blocks), a last partial block one more -- in either direction
    auto rows_copy = [&](int k, int rk, char* dev, hipMemcpyKind kind, hipStream_t s) -> hipError_t {
        const int full = rk / b, tail = rk % b;
        char* host = reinterpret_cast<char*>(buf) + (size_t)k * blk;
        hipError_t e = hipSuccess;
        if (full > 0)
            e = kind == hipMemcpyHostToDevice
                    ? hipMemcpy2DAsync(dev, blk, host, blk * N, blk, (size_t)full, kind, s)
                    : hipMemcpy2DAsync(host, blk * N, dev, blk, blk, (size_t)full, kind, s);
        if (e == hipSuccess && tail > 0)
            e = kind == hipMemcpyHostToDevice
                    ? hipMemcpyAsync(dev + (size_t)full * blk, host + (size_t)full * blk * N, (size_t)tail * rowBytes,
                                     kind, s)
                    : hipMemcpyAsync(host + (size_t)full * blk * N, dev + (size_t)full * blk, (size_t)tail * rowBytes,
                                     kind, s);
        return e;
    };
    for (int k = 0; k < N; ++k) {
        DeviceScope ds(k);
        Context& c = ctx();
        if (int rc = ensure_buffer(c.d_shard, c.shard_bytes, shardBytes, "shard")) return rc;
        if (g_multi.gather)
            if (int rc = ensure_buffer(c.d_pack, c.pack_bytes, packBytes, "packed shard")) return rc;
        if (!c.ev_done) LRT_HIP(hipEventCreateWithFlags(&c.ev_done, hipEventDisableTiming));
        const int rk = lrt_shard_rows(rows, b, N, k);
        if (rk > 0) LRT_HIP(rows_copy(k, rk, reinterpret_cast<char*>(c.d_shard), hipMemcpyHostToDevice, c.stream));
        LRT_HIP(hipMemsetAsync(c.d_rays, 0, sizeof(unsigned long long), c.stream));
        lrt_render_desc sd = *d;
        sd.row_count = rk;
        sd.row_block = b;
        sd.row_period = N;
        sd.row_phase = k;
        if (int rc = render_device(&sd, c.d_shard, c.d_rays, nullptr, c.stream)) return rc;
        LRT_HIP(hipMemcpyAsync(c.h_rays, c.d_rays, sizeof(unsigned long long), hipMemcpyDeviceToHost, c.stream));
        if (!g_multi.gather) {   // direct: this device's rows straight back to the caller
            if (rk > 0) LRT_HIP(rows_copy(k, rk, reinterpret_cast<char*>(c.d_shard), hipMemcpyDeviceToHost, c.stream));
            continue;
        }
        if (rk > 0)
            LRT_HIP(launch_pack_rgb(reinterpret_cast<const float4*>(c.d_shard), c.d_pack, (size_t)rk * xc, c.stream));
        LRT_HIP(hipEventRecord(c.ev_done, c.stream));
    }
    if (!g_multi.gather) return LRT_OK;
    // the gather: every packed shard into device 0, the frame assembled over the caller's values
    DeviceScope ds0(0);
    Context& c0 = ctx();
    if (int rc = ensure_buffer(c0.d_gath, c0.gath_bytes, packBytes * N, "gather")) return rc;
    if (int rc = ensure_frame(bytes)) return rc;
    LRT_HIP(hipMemcpyAsync(c0.d_frame, buf, bytes, hipMemcpyHostToDevice, c0.stream));
    if (g_multi.rccl) {
        const size_t count = packBytes / sizeof(float);
        if (ncclGroupStart() != ncclSuccess) return fail(LRT_E_HIP, "ncclGroupStart");
        ncclResult_t r = ncclSuccess;
        for (int k = 0; k < N && r == ncclSuccess; ++k) {
            DeviceScope ds(k);
            r = ncclGather(g_devs[k].d_pack, k == 0 ? c0.d_gath : nullptr, count, ncclFloat, 0, g_multi.comms[k],
                           g_devs[k].stream);
        }
        const ncclResult_t r2 = ncclGroupEnd();
        if (r != ncclSuccess || r2 != ncclSuccess)
            return fail(LRT_E_HIP, std::string("ncclGather: ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
    } else {
        for (int k = 0; k < N; ++k) {
            LRT_HIP(hipStreamWaitEvent(c0.stream, g_devs[k].ev_done, 0));
            char* dst = reinterpret_cast<char*>(c0.d_gath) + (size_t)k * packBytes;
            if (g_devs[k].device == c0.device)
                LRT_HIP(hipMemcpyAsync(dst, g_devs[k].d_pack, packBytes, hipMemcpyDeviceToDevice, c0.stream));
            else
                LRT_HIP(hipMemcpyPeerAsync(dst, c0.device, g_devs[k].d_pack, g_devs[k].device, packBytes, c0.stream));
        }
    }
    LRT_HIP(launch_unshard_rgb(c0.d_gath, reinterpret_cast<float4*>(c0.d_frame), xc, rows, b, N, maxRows, c0.stream));
    LRT_HIP(hipMemcpyAsync(buf, c0.d_frame, bytes, hipMemcpyDeviceToHost, c0.stream));
    return LRT_OK;
}

}  // namespace lrt

using namespace lrt;

extern "C" {

int lrt_exchange_bytes(int x_count, int rows, int row_block, int devices, long long* direct, long long* gather_xgmi) {
    if (x_count < 0 || rows < 0 || row_block < 1 || devices < 1 || !direct || !gather_xgmi)
        return fail(LRT_E_INVALID, "invalid exchange geometry");
    multi_exchange_bytes(x_count, rows, row_block, devices, direct, gather_xgmi);
    return LRT_OK;
}

int lrt_initialize_devices(int n, const int* device_ids, int flags) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ndev > 0) return fail(LRT_E_STATE, "already initialised: call lrt_shutdown() first");
    if ((flags & ~(LRT_DEV_PEER_COPY | LRT_DEV_GATHER)) != 0)
        return fail(LRT_E_INVALID, "unknown lrt_initialize_devices flags");
    int visible = 0;
    LRT_HIP(hipGetDeviceCount(&visible));
    std::vector<int> ids;
    if (n == 0 && !device_ids) {   // every visible device
        for (int i = 0; i < visible && i < kMaxDevices; ++i) ids.push_back(i);
    } else {
        if (n < 1 || n > kMaxDevices || !device_ids) return fail(LRT_E_INVALID, "need 1..16 device ids");
        ids.assign(device_ids, device_ids + n);
    }
    if (ids.empty()) return fail(LRT_E_INVALID, "no device");
    for (int id : ids)
        if (id < 0 || id >= visible) return fail(LRT_E_INVALID, "device id out of range");
    int prev = 0;
    LRT_HIP(hipGetDevice(&prev));
    int rc = LRT_OK;
    int k = 0;
    for (; k < (int)ids.size() && rc == LRT_OK; ++k) {
        g_cur = k;
        if (hipSetDevice(ids[k]) != hipSuccess) {
            rc = fail(LRT_E_HIP, "hipSetDevice");
            break;
        }
        rc = init_context(g_devs[k], ids[k]);
    }
    g_cur = 0;
    const int N = (int)ids.size();
    bool distinct = true;
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < i; ++j) distinct = distinct && ids[i] != ids[j];
    g_multi = Multi();
    if (const char* e = getenv("LRT_ROW_BLOCK")) g_multi.row_block = std::max(1, atoi(e));
    g_multi.gather = (flags & (LRT_DEV_GATHER | LRT_DEV_PEER_COPY)) != 0;
    if (rc == LRT_OK && g_multi.gather && distinct && !(flags & LRT_DEV_PEER_COPY)) {
        // one communicator per device, all in this process (the single-thread multi-device
        // form of RCCL); the gather is issued as a group (render_host_multi)
        const ncclResult_t r = ncclCommInitAll(g_multi.comms, N, ids.data());
        if (r != ncclSuccess) rc = fail(LRT_E_HIP, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
        g_multi.rccl = r == ncclSuccess;
    } else if (rc == LRT_OK && g_multi.gather) {
        for (int i = 1; i < N; ++i)   // peer copies into device 0 (ignore "already enabled")
            if (ids[i] != ids[0]) {
                (void)hipSetDevice(ids[0]);
                (void)hipDeviceEnablePeerAccess(ids[i], 0);
                (void)hipGetLastError();
            }
    }
    (void)hipSetDevice(prev);
    if (rc) {
        for (int i = 0; i < k; ++i) {
            DeviceScope ds(i);
            free_context(g_devs[i]);
        }
        if (g_multi.rccl)
            for (int i = 0; i < N; ++i) (void)ncclCommDestroy(g_multi.comms[i]);
        g_multi = Multi();
        return rc;
    }
    g_ndev = N;
    g_multi.on = true;
    return LRT_OK;
}

int lrt_ipc_alloc(size_t bytes, void** d_ptr, void* handle) {
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);
    if (!d_ptr || !handle || bytes == 0) return fail(LRT_E_INVALID, "invalid ipc alloc arguments");
    *d_ptr = nullptr;
    LRT_HIP(hipMalloc(d_ptr, bytes));   // its own allocation: the handle maps exactly this buffer
    LRT_HIP(hipMemset(*d_ptr, 0, bytes));
    hipIpcMemHandle_t h;
    const hipError_t e = hipIpcGetMemHandle(&h, *d_ptr);
    if (e != hipSuccess) {
        (void)hipFree(*d_ptr);
        *d_ptr = nullptr;
        return hip_fail(e, "hipIpcGetMemHandle");
    }
    static_assert(sizeof(h) <= LRT_IPC_HANDLE_BYTES, "IPC handle size");
    memcpy(handle, &h, sizeof(h));
    return LRT_OK;
}

int lrt_ipc_free(void* d_ptr) {
    if (!d_ptr) return LRT_OK;
    LRT_HIP(hipFree(d_ptr));
    return LRT_OK;
}

int lrt_ipc_open(const void* handle, void** d_ptr) {
    std::lock_guard<std::mutex> lk(g_mu);
    DeviceScope ds_(0);
    if (!handle || !d_ptr) return fail(LRT_E_INVALID, "invalid ipc open arguments");
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    LRT_HIP(hipIpcOpenMemHandle(d_ptr, h, hipIpcMemLazyEnablePeerAccess));
    return LRT_OK;
}

int lrt_ipc_close(void* d_ptr) {
    if (!d_ptr) return LRT_OK;
    LRT_HIP(hipIpcCloseMemHandle(d_ptr));
    return LRT_OK;
}

}  // extern "C"
