// The pool kernel's tile order (tile_order) and the first launch's cost probe.
#include "lrt_probe.h"

namespace lrt {

// v5 (lrt_pool.h): v0's LDS layout, queues, counters and overflow stack, plus the
// per-block colour slots.
// Heaviest-first tile order for the pool kernel (LRT_POOL_ORDER=0: off). A pool tile is
// 4x a v0 task, and a tile over a glass sphere costs several average ones, so a launch in
// queue order ends with a few waves finishing heavy tiles while the rest of the chip idles
// (profiles/r2_p8). The first launch of a render signature (window, frames, depth, flags,
// camera, scene, tile size) records each tile's cost; once it has finished, the next launch
// of that signature sorts the costs on the host and hands tiles out heaviest first -- the
// classic LPT order -- and so does every later one. Each pixel's result is unchanged: only
// the order in which tiles are taken changes.
// The last kOrderSlots signatures keep their orders, so callers alternating renders (two
// windows, a DrawTest beside a device render) neither start over nor wait. A new view of the
// same geometry (the camera moved, the scene was edited) borrows the newest ready order of
// that geometry for its own recording launch and until its costs are in: its first launch
// already runs heaviest-first by the previous view's measure.
uint64_t fnv(uint64_t h, const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}
bool pool_order_on() {
    static const bool on = [] {
        const char* e = getenv("LRT_POOL_ORDER");
        return !(e && atoi(e) == 0);
    }();
    return on;
}
// Waits until every launch that used entry e has passed it (only those streams' events).
int order_release(Context::TileOrder& e) {
    for (auto& u : e.uses) LRT_HIP(hipEventSynchronize(u.second));
    return LRT_OK;
}
// After a launch on stream s that read e's permutation or wrote its costs.
int order_used(Context::TileOrder& e, hipStream_t s) {
    for (auto& u : e.uses)
        if (u.first == s) {
            LRT_HIP(hipEventRecord(u.second, s));
            return LRT_OK;
        }
    hipEvent_t ev = nullptr;
    LRT_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    e.uses.emplace_back(s, ev);
    LRT_HIP(hipEventRecord(ev, s));
    return LRT_OK;
}
// Stream s waits for entry e's recording launch and sort -- until they are seen complete, after
// which no launch needs the wait (one command fewer between a stream's kernels).
int order_wait(Context::TileOrder& e, hipStream_t s) {
    if (!e.rec_done) {
        bool done = false;
        if (const hipError_t q = event_done(e.ev_rec, &done)) return hip_fail(q, "hipEventQuery(tile order)");
        e.rec_done = done;
    }
    if (!e.rec_done) LRT_HIP(hipStreamWaitEvent(s, e.ev_rec, 0));
    return LRT_OK;
}
// Picks a's order for this launch: a.perm (null: queue order) and, for the recording launch,
// a.tcost. *users gets the entries whose buffers the launch touches (order_used after it).
// LRT_POOL_PROBE: 0 off; 1 (default) a new signature without an order of the same geometry
// to borrow probes its tiles (probe_kernel) and runs its recording launch in the probe's
// order; 2 probes even when it could borrow
int pool_probe_mode() {
    static const int m = [] {
        const char* e = getenv("LRT_POOL_PROBE");
        return e ? atoi(e) : 1;
    }();
    return m;
}

// Sizes entry e for ntiles tiles (at least 65,536, so views of other sizes rarely reallocate).
// Entries are allocated together on first use, so a new view's first launch does not wait
// for hipMalloc.
int order_alloc(Context::TileOrder& e, long long ntiles, hipStream_t s) {
    if (e.cap >= ntiles) return LRT_OK;
    const long long cap = std::max(ntiles, 65536LL);
    size_t tmp = 0;
    LRT_HIP(sort_tiles_desc(nullptr, nullptr, nullptr, nullptr, (int)cap, nullptr, &tmp, s));
    const size_t arr = ((size_t)cap * 4 + 255) & ~(size_t)255;   // cost, keys, ids, two perms
    if (e.d_base) (void)hipFree(e.d_base);   // (its launches have passed: order_release)
    e.d_base = nullptr;
    e.cap = 0;
    if (hipMalloc(&e.d_base, 5 * arr + tmp) != hipSuccess) {
        e.d_base = nullptr;
        return fail(LRT_E_NOMEM, "hipMalloc(tile order)");
    }
    char* b = static_cast<char*>(e.d_base);
    e.d_cost = reinterpret_cast<unsigned*>(b);
    e.d_keys = reinterpret_cast<unsigned*>(b + arr);
    e.d_ids = reinterpret_cast<int*>(b + 2 * arr);
    e.d_permb[0] = reinterpret_cast<int*>(b + 3 * arr);
    e.d_permb[1] = reinterpret_cast<int*>(b + 4 * arr);
    e.d_perm = e.d_permb[0];
    e.d_tmp = b + 5 * arr;
    e.tmp_bytes = tmp;
    LRT_HIP(fill_iota(e.d_ids, (int)cap, s));
    // a later signature may take this entry on another stream, whose sort reads d_ids: the
    // fill completes here (allocation is rare -- the first use sizes every entry at once)
    LRT_HIP(hipStreamSynchronize(s));
    e.cap = cap;
    return LRT_OK;
}

int tile_order(KernelArgs& a, int kPix, long long ntiles, int& record, Context::TileOrder* users[2], hipStream_t s) {
    record = 0;
    users[0] = users[1] = nullptr;
    if (!pool_order_on() || ntiles < 2 * kV0Queues) return LRT_OK;
    Context& c = ctx();
    const int geo[] = {a.width, a.height, a.x0, a.xc, a.y0, a.rows, a.rb, a.rp, a.rph, a.frames, a.maxDepth,
                       a.ndl, a.bv.on, a.gv.on, a.count, kPix, a.sph == c.d_sph ? 0 : 1};
    const uint64_t gkey = fnv(1469598103934665603ull, geo, sizeof(geo));
    uint64_t sig = fnv(gkey, &c.scene_version, sizeof(c.scene_version));
    sig = fnv(sig, &a.cam, sizeof(a.cam));
    Context::TileOrder* e = nullptr;
    for (auto& o : c.order)
        if (o.state != 0 && o.sig == sig && o.ntiles == ntiles) e = &o;
    if (!e) {   // a new signature: take a free entry, else the least recently used one
        for (auto& o : c.order)
            if (!e && o.state == 0) e = &o;
        if (!e) {
            e = &c.order[0];
            for (auto& o : c.order)
                if (o.tick < e->tick) e = &o;
        }
        int donor = -1;   // the newest ready order of the same geometry
        for (int i = 0; i < Context::kOrderSlots; ++i) {
            const auto& o = c.order[i];
            if (&o != e && o.state == 2 && o.gkey == gkey && o.ntiles == ntiles &&
                (donor < 0 || o.tick > c.order[donor].tick))
                donor = i;
        }
        if (e->state != 0) {
            // launches that read this entry's permutation (also as a donor) must be done
            // with it; the entries borrowing it lose their donor
            if (int rc = order_release(*e)) return rc;
            for (auto& o : c.order)
                if (o.donor == (int)(e - c.order)) o.donor = -1;
        }
        if (e->cap < ntiles) {
            e->state = 0;
            for (auto& o : c.order)   // the first use sizes every unallocated entry at once
                if (&o == e || (o.cap == 0 && o.state == 0))
                    if (int rc = order_alloc(o, ntiles, s)) return rc;
        }
        if (!e->ev_rec) LRT_HIP(hipEventCreateWithFlags(&e->ev_rec, hipEventDisableTiming));
        e->sig = sig;
        e->gkey = gkey;
        e->ntiles = ntiles;
        // the recording launch writes d_cost and the sort behind it (launch_pool) d_perm:
        // ready for every later launch once ev_rec has passed, which each of them waits for
        e->state = 2;
        e->rec_done = false;
        e->donor = donor;
        e->passes = 1;
        e->d_perm = e->d_permb[0];
        e->d_sort_out = e->d_perm;
        a.tcost = e->d_cost;
        record = 1;
        if (donor >= 0) {   // meanwhile the newest order of the same geometry
            users[1] = &c.order[donor];
            if (int rc = order_wait(*users[1], s)) return rc;
            a.perm = users[1]->d_perm;
            users[1]->tick = ++c.order_tick;
        }
    } else {
        if (int rc = order_wait(*e, s)) return rc;
        a.perm = e->d_perm;
        if (e->passes == 1) {
            // The refining pass: this launch takes its tiles in the first pass's order and records
            // them again. The first pass timed each tile in queue order, where a tile's wall time
            // depends on where in the launch it ran; timed in the sorted order, the heavy tiles run
            // together at the start and the light ones at the end, as every later launch runs them
            // (profiles/r5_x). Its sort writes the other permutation buffer: launches still reading
            // this one are untouched, later ones wait for the sort (ev_rec) and read the new one.
            e->passes = 2;
            e->rec_done = false;
            e->d_sort_out = e->d_permb[e->d_perm == e->d_permb[0] ? 1 : 0];
            e->d_perm = e->d_sort_out;
            a.tcost = e->d_cost;
            record = 2;
        }
    }
    users[0] = e;
    e->tick = ++c.order_tick;
    return LRT_OK;
}

hipError_t launch_tile_probe(const KernelArgs& a, int acc, Context::TileOrder& o, int ntiles, int TX, int TY,
                             size_t bstk, hipStream_t s) {
    const unsigned pblocks = (unsigned)((ntiles + 64 / kProbe - 1) / (64 / kProbe));
    if (acc == kAccGrid) probe_kernel<kAccGrid><<<pblocks, 64, 0, s>>>(a, o.d_cost, ntiles, TX, TY);
    else if (acc == kAccBvh) probe_kernel<kAccBvh><<<pblocks, 64, bstk, s>>>(a, o.d_cost, ntiles, TX, TY);
    else probe_kernel<kAccScan><<<pblocks, 64, 0, s>>>(a, o.d_cost, ntiles, TX, TY);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    probe_order_kernel<<<1, 1024, 0, s>>>(o.d_cost, o.d_perm, ntiles);
    return hipGetLastError();
}

}  // namespace lrt
