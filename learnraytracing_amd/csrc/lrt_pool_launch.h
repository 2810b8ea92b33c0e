// The pool kernel's launch (lrt_pool.h): grid, colour slots, overflow stack, tile order.
// Instantiated per depth class by lrt_pool_d8.hip and lrt_pool_d64.hip.
#pragma once
#include "lrt_internal.h"
#include "lrt_pool.h"

namespace lrt {

// Waves per block of the grid instance (kPoolGridWaves blocks share the grid's LDS copy); 1
// when the grid does not fit beside the waves' stacks.
inline int pool_grid_wpb(const KernelArgs& a, size_t stack_w, size_t shared_b, size_t static_b, size_t* grid_b) {
    const size_t ncell = (size_t)a.gv.nx * a.gv.ny * a.gv.nz, nref = a.gv.cells_refs;
    *grid_b = (16 * nref + 8 * ncell + 4 * nref + 15) / 16 * 16;
    if (!a.gv.on || a.gv.nx == 0) return 1;
    int dev = 0, maxb = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&maxb, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess)
        return 1;
    return kPoolGridWaves * stack_w + shared_b + *grid_b + static_b <= (size_t)maxb ? kPoolGridWaves : 1;
}

template <int MAXD, int kPix>
int launch_pool(KernelArgs a, bool lds, int xc, int rows, hipStream_t s) {
    constexpr int TX = PoolTile<kPix>::X, TY = PoolTile<kPix>::Y;
    constexpr int kW = kPoolGridWaves;
    const long long ntiles = (long long)((xc + TX - 1) / TX) * ((rows + TY - 1) / TY);
    const int acc = a.gv.on ? kAccGrid : a.bv.on ? kAccBvh : kAccScan;
    // the BVH's traversal stack, or the grid's first-tested spheres (pool_grid_view)
    const size_t bstk = acc == kAccBvh ? sizeof(unsigned short) * ctx().bvh_stack_levels * 64
                        : acc == kAccGrid ? (sizeof(float4) + sizeof(int)) * (size_t)a.gv.nbig : 0;
    size_t grid_b = 0;
    // the instance's static LDS (diagnostic builds' section counters) beside the dynamic
    static const size_t static_b = [] {
        hipFuncAttributes fa{};
        return hipFuncGetAttributes(&fa, (const void*)pool_kernel<MAXD, false, kAccGrid, kPix, 0, kW>) == hipSuccess
                   ? fa.sharedSizeBytes
                   : (size_t)0;
    }();
    int wpb = acc == kAccGrid && !lds
                  ? pool_grid_wpb(a, pool_stack_bytes<kW>(), kPowTableBytes + (bstk + 15) / 16 * 16, static_b, &grid_b)
                  : 1;
    if (wpb > 1) {
        // dynamic LDS above the default limit: raised once per device for this instance
        // (advisor r4: per device, and a refusal falls back to one-wave blocks)
        static signed char raised[kMaxDevices * 4] = {};   // 0 not yet, 1 raised, -1 refused
        int dev = 0, maxb = 0;
        signed char* r = hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < kMaxDevices * 4 ? &raised[dev] : nullptr;
        if (r && *r == 0)
            *r = hipDeviceGetAttribute(&maxb, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) == hipSuccess &&
                         hipFuncSetAttribute((const void*)pool_kernel<MAXD, false, kAccGrid, kPix, 0, kW>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             maxb - (int)static_b) == hipSuccess
                     ? 1
                     : -1;
        if (!r || *r < 0) wpb = 1;
    }
    const int lv = kTraceLdsLevels;   // recursion stack levels in LDS (packed in multi-wave blocks)
    const size_t stack = (wpb > 1 ? (size_t)pool_stack_bytes<kW>() * wpb : (size_t)pool_stack_bytes<1>()) +
                         kPowTableBytes + (acc ? 0 : kRenormBytes);
    const size_t scene = lds ? sizeof(float4) * (4 * (size_t)a.count + (size_t)(a.nlights + 3) / 4 + 1) : 0;
    a.bvh_stack_offset = (int)(stack + scene);
    a.grid_lds_offset = wpb > 1 ? (int)(stack + (bstk + 15) / 16 * 16) : 0;
    const size_t ldsb = wpb > 1 ? stack + (bstk + 15) / 16 * 16 + grid_b : stack + scene + bstk;
    const bool fixed = lds && acc == kAccScan && a.count == kFixedSpheres;
    const void* kern = acc == kAccGrid ? (lds ? (const void*)pool_kernel<MAXD, true, kAccGrid, kPix>
                                          : wpb > 1 ? (const void*)pool_kernel<MAXD, false, kAccGrid, kPix, 0, kW>
                                              : (const void*)pool_kernel<MAXD, false, kAccGrid, kPix>)
                       : acc == kAccBvh ? (lds ? (const void*)pool_kernel<MAXD, true, kAccBvh, kPix>
                                               : (const void*)pool_kernel<MAXD, false, kAccBvh, kPix>)
                       : (fixed ? (const void*)pool_kernel<MAXD, true, kAccScan, kPix, kFixedSpheres>
                          : lds ? (const void*)pool_kernel<MAXD, true, kAccScan, kPix>
                                : (const void*)pool_kernel<MAXD, false, kAccScan, kPix>);
    int per_cu = 0;
    hipError_t e = occupancy(&per_cu, kern, 64 * wpb, ldsb);
    if (e != hipSuccess) return hip_fail(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    if (per_cu < 1) return fail(LRT_E_INVALID, "pool_kernel does not fit on a CU");
    int cus = ctx().num_cus;
    for (const auto& m : ctx().masked_streams)
        if (m.first == s) cus = m.second;
    // a block per queue (as v0: queue q is served by blocks q, q + kV0Queues, ...), no more
    // blocks than tiles (kW > 1: the block's waves beyond its queue's tiles find none)
    long long blocks = std::max((long long)per_cu * cus, (long long)kV0Queues);
    if (blocks > ntiles) blocks = ntiles;
    const dim3 grid((unsigned)blocks);
    a.ovf = nullptr;
    a.colbuf = nullptr;
    a.tiles = ctx().d_tiles + (size_t)(ctx().tiles_next++ % kQueueSlots) * kTileSetU64;
    // waiting lanes that trigger a refill (fold + next samples). Measured (profiles/r2_p2):
    // config 3 2.31 -> 2.05 ms/step at 16 (vs 1), config 4 and config 2 neutral
    a.regenMin = 16;
    // few tiles per wave (config 2: 14,400 tiles on 4,096 waves): reserve late (lrt_pool.h;
    // deciding by whether another stream's launch still runs was measured neutral, r5_ah)
    a.lateFetch = ntiles < 6LL * (long long)grid.x * wpb ? 1 : 0;
    a.poolSlots = kPix * std::min(a.frames, kPoolSamples / kPix);   // one round's samples
    const size_t nwaves = (size_t)grid.x * wpb;
    // the colour slots, then the overflow stack's float4 levels and u16 level tags (lrt_pool.h),
    // in the stream's scratch (kept between launches)
    const size_t col_b = (sizeof(float) * 3 * (size_t)a.poolSlots * nwaves + 255) / 256 * 256;
    const size_t ovf_b = a.maxDepth > lv ? (sizeof(float4) + sizeof(unsigned short)) * nwaves * 64 *
                                               (size_t)(a.maxDepth - lv)
                                         : 0;
    {
        void* p = nullptr;
        e = stream_scratch(s, col_b + ovf_b, &p);
        if (e != hipSuccess) return hip_fail(e, "pool scratch (colour slots, overflow stack)");
        a.colbuf = static_cast<float*>(p);
        if (ovf_b) a.ovf = reinterpret_cast<float4*>(static_cast<char*>(p) + col_b);
    }
#ifdef LRT_EXP_SECSTATS
    unsigned long long* d_sec = secstats_buffer(s);
    a.wtrace = d_sec;
#endif
#ifdef LRT_EXP_WAVETRACE
    a.wtrace = wavetrace_buffer((unsigned)nwaves);
#endif
    int record = 0;
    Context::TileOrder* users[2];
    if (int rc = tile_order(a, kPix, ntiles, record, users, s)) return rc;
    // the split tail: the last split16/16 of the (heaviest-first) tiles served as halves, in
    // launches of few tiles per wave (a.lateFetch) that give every queue a block (the halves are
    // extra queue items: a queue without a block would leave them undone); a recording launch
    // times whole tiles
    const bool split = !a.tcost && wpb == 1 && a.lateFetch && blocks >= kV0Queues;
    a.splitFrom = split ? (int)(ntiles - ntiles * a.split16 / 16) : (int)ntiles;
    bool probed = false;
    if (record == 1 && pool_probe_mode() > 0 && (pool_probe_mode() == 2 || !users[1])) {
        // no measured order to go by: probe the tiles' costs, sort them, and let this
        // (recording) launch take its tiles in that order (probe_kernel, lrt_pool.h)
        Context::TileOrder& o = *users[0];
        KernelArgs pa = a;
        pa.bvh_stack_offset = 0;
        e = launch_tile_probe(pa, acc, o, (int)ntiles, TX, TY, bstk, s);
        if (e != hipSuccess) {
            o.state = 0;
            return hip_fail(e, "tile cost probe");
        }
        a.perm = o.d_perm;
        users[1] = nullptr;   // (a borrowed order, if any, is not used)
        probed = true;
    }
    kernel_timing(s, 0);
    if (acc == kAccGrid) {
        if (lds) pool_kernel<MAXD, true, kAccGrid, kPix><<<grid, 64, ldsb, s>>>(a);
        else if (wpb > 1) pool_kernel<MAXD, false, kAccGrid, kPix, 0, kW><<<grid, 64 * kW, ldsb, s>>>(a);
        else pool_kernel<MAXD, false, kAccGrid, kPix><<<grid, 64, ldsb, s>>>(a);
    } else if (acc == kAccBvh) {
        if (lds) pool_kernel<MAXD, true, kAccBvh, kPix><<<grid, 64, ldsb, s>>>(a);
        else pool_kernel<MAXD, false, kAccBvh, kPix><<<grid, 64, ldsb, s>>>(a);
    } else if (fixed) {
        pool_kernel<MAXD, true, kAccScan, kPix, kFixedSpheres><<<grid, 64, ldsb, s>>>(a);
    } else {
        if (lds) pool_kernel<MAXD, true, kAccScan, kPix><<<grid, 64, ldsb, s>>>(a);
        else pool_kernel<MAXD, false, kAccScan, kPix><<<grid, 64, ldsb, s>>>(a);
    }
    kernel_timing(s, 1);
    e = hipGetLastError();
    if (e != hipSuccess) {
        if (record) users[0]->state = 0;   // nothing recorded: the entry is free again
        return hip_fail(e, "pool_kernel launch");
    }
    e = stream_scratch_used(s);
    if (e != hipSuccess) return hip_fail(e, "pool scratch event");
    if (record) {   // the costs just recorded, sorted on the device behind the launch
        Context::TileOrder& o = *users[0];
        e = sort_tiles_desc(o.d_cost, o.d_keys, o.d_ids, o.d_sort_out, (int)ntiles, o.d_tmp, &o.tmp_bytes, s);
        if (e == hipSuccess) e = hipEventRecord(o.ev_rec, s);
        if (e != hipSuccess) {
            o.state = 0;   // no order for this signature: the next launch records again
            return hip_fail(e, "tile order sort");
        }
    }
    for (auto* u : users)
        if (u)
            if (int rc = order_used(*u, s)) return rc;
    // order: 0 queue order (tile order off), 1 recording in queue order, 2 the signature's own
    // sorted order, 3 recording with the order borrowed from the same geometry, 4 recording in
    // the probe's order, 5 the refining pass (recording in the first pass's sorted order)
    snprintf(g_last_launch, sizeof(g_last_launch),
             "kernel=pool_kernel maxd=%d lds=%d bvh=%d acc=%s pix=%d ns=%d grid=%u tasks=%lld order=%d per_cu=%d wpb=%d "
             "split_from=%d",
             MAXD, lds ? 1 : 0, acc == kAccBvh ? 1 : 0, acc_name(acc), kPix, fixed ? kFixedSpheres : 0, grid.x, ntiles,
             !users[0] ? 0 : !record ? 2 : record == 2 ? 5 : probed ? 4 : users[1] ? 3 : 1, per_cu, wpb, a.splitFrom);
#ifdef LRT_EXP_SECSTATS
    secstats_dump(d_sec, s);
#endif
#ifdef LRT_EXP_WAVETRACE
    wavetrace_dump(a.wtrace, grid.x, s);
#endif
    return LRT_OK;
}

template <int MAXD>
int launch_pool_split(const KernelArgs& a, bool lds, int xc, int rows, int frames, int pix_cap, hipStream_t s) {
    switch (pool_pixels(frames, xc, rows, pix_cap)) {
        case 256: return launch_pool<MAXD, 256>(a, lds, xc, rows, s);
        case 128: return launch_pool<MAXD, 128>(a, lds, xc, rows, s);
        case 64: return launch_pool<MAXD, 64>(a, lds, xc, rows, s);
        case 32: return launch_pool<MAXD, 32>(a, lds, xc, rows, s);
        case 16: return launch_pool<MAXD, 16>(a, lds, xc, rows, s);
        case 4: return launch_pool<MAXD, 4>(a, lds, xc, rows, s);
        default: return launch_pool<MAXD, 1>(a, lds, xc, rows, s);
    }
}

}  // namespace lrt
