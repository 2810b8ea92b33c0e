// Internal declarations shared by liblrt_hip.so's translation units. Each unit owns one
// part of the library and its invariants:
//   lrt_api.hip       the C-ABI's context lifecycle and render entry points, the globals
//   lrt_scene.hip     scene packing and upload, the BVH and grid builds, the camera
//   lrt_render.hip    render_device: validation, the kernel policy, the wavefront launch
//   lrt_v0_d8/d64     the v0 kernel (trace_kernel) instances for depth <= 8 / <= 64
//   lrt_pool_d8/d64   the pool kernel (pool_kernel) instances
//   lrt_order.hip     the pool kernel's tile-order cache and cost probe
//   lrt_hostpath.hip  host backbuffers: DrawTest's pipelined path, its look-ahead, staging
//   lrt_multi.hip     one process, several devices: split, RCCL gather, IPC frames
//   lrt_frame.hip     frame assembly and present kernels
//   lrt_diag.hip      host/device diagnostics (BVH/grid statistics, Scatter and libm probes)
//   lrt_sort.hip      rocPRIM's radix sort (the tile order)
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#ifndef LRT_ROCTX   // roctx ranges (tracing only): the Makefile sets it when the header exists
#define LRT_ROCTX 0
#endif
#if LRT_ROCTX
#include <rocprofiler-sdk-roctx/roctx.h>
#endif
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <mutex>
#include <type_traits>
#include <string>
#include <vector>

#include "lrt.h"
#include "lrt_diag.h"
#include "lrt_trace.h"

#define LRT_VERSION_STRING "lrt-mi355x 0.3.0 gfx950"

namespace lrt {

// v0 workgroup: one wave. A wave finished early in a multi-wave block keeps its slot (and the
// block's LDS) until the slowest wave ends; with path lengths as uneven as these, single-wave
// blocks keep ~1 more wave resident per SIMD.
constexpr int kBlock = 64;
constexpr int kBlockWavesX = kBlock == 256 ? 2 : 1;           // waves per block in x
constexpr int kBlockWavesY = kBlock / 64 / kBlockWavesX;       // and in y
// a wave's pixels: 64 / kSplit of them, 8 wide (kSplit <= 8) or a single row
constexpr int WaveCols(int split) { return split <= 8 ? 8 : 64 / split; }
// Work counters: same-address device-scope atomics serialise at ~12 ns each (measured
// ~80/us chip-wide), so v0's tile queue and ray count are split over kV0Queues
// counters, each on its own 512-B line; block b serves queue b % kV0Queues, which owns
// tiles q, q + kV0Queues, ...
constexpr int kV0Queues = 16;
constexpr int kCtrStride = 64;   // u64s between counters

constexpr int kMaxDepthSupported = 64;

// 4 waves per SIMD: caps VGPRs at 128. The MAXD 20/64 and BVH instances otherwise
// take 129-144 and drop to 3 waves (config 3: 4.44 -> 4.15 ms, config 4: 587 -> 538 ms
// with the cap; the BVH instances spill 28-40 B/lane to scratch, which costs less).
constexpr int kWavesPerEU = 4;
// Samples per round of a tile, at most: with pixels x frames <= kPoolSamples a tile has one
// round. Config 4 (64 spp): 1024 (16 px) 229 ms, 2048 (32 px) 222, 4096 (64 px) 221;
// config 5 (256 spp, one GPU): 1024 (4 px) 3876 ms, 4096 (16 px) 3602 (profiles/r2_p2).
constexpr int kPoolSamples = 4096;

struct KernelArgs {
    CameraDev cam;
    const float4* sph;
    const float4* mats;
    const int* lights;
    int count, nlights;
    int width, height;
    int x0, xc, y0, rows;
    int rb, rp, rph;
    int frame0, frames, maxDepth;
    float4* out;
    unsigned long long* rays;
    BvhView bv;
    GridView gv;
    int bvh_stack_offset;   // bytes into dynamic LDS
    int grid_lds_offset;    // pool kernel, kPoolGridWaves blocks: the grid's LDS copy (bytes), or 0
    float4* ovf;            // recursion stack levels >= kTraceLdsLevels (null when maxDepth fits)
    unsigned long long* wtrace;   // LRT_EXP_WAVETRACE builds only: per-wave start/end/ids
    unsigned long long* tiles;    // this launch's counters: [q] tile queue, [kV0Queues + q] finished
                                  // blocks (bits 48-63) and ray total (bits 0-47) of queue q
    int ndl;                      // LRT_F_NO_DOUBLE_LIGHT
    // lrt_features (kFeat launches): normal, world_pos, albedo, color_std, normal_std,
    // world_pos_std (any may be null) and the last frame they are updated for (< 0: all)
    float4* feat[6];
    int featMax;
    int regenMin;                 // v5: waiting lanes that trigger a refill
    int lateFetch;                // v5: reserve the next tile at this one's end, not its start (lrt_pool.h)
    const float* lerp;            // lerpFac = (float)f / (float)(f + 1) for f < kLerpTable (parallel.cpp:262)
    float4* samp;                 // sample mode: frames planes of xc * rows colours
    float* colbuf;                // v5 (pool): poolSlots colour slots (RGB) per block
    int poolSlots;
    int splitFrom;                // v5: queue items from here on are half tiles (lrt_pool.h)
    int split16;                  // v5 (host): sixteenths of the tiles served as halves (launch_pool)
    const int* perm;              // v5: queue position -> tile, heaviest measured tiles first (null: identity)
    unsigned* tcost;              // v5: per-tile cost recording (100 MHz ticks of the tile's wave), or null
    int sampOnly;                 // colours only (the pipelined host path): samp is the caller's
    float4* frame;                // lrt_render_device_to_frame: the whole width x height frame (any
                                  // device, IPC/peer-mapped) that each finished pixel is also stored
                                  // to at its global row -- the multi-GPU exchange fused into the
                                  // render's last store; null otherwise
};

// Global position of local row ly (lrt_render_desc's row map).
LRT_DEV int GlobalRow(const KernelArgs& a, int ly) { return a.y0 + (ly / a.rb) * a.rb * a.rp + a.rph * a.rb + ly % a.rb; }
constexpr int kLerpTable = 1 << 16;
constexpr int kFixedSpheres = 9;   // the reference's kSphereCount (parallel.cpp:27)

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// A block's last act (one thread): ONE atomic on queue q's 64-bit word that carries the
// count of finished blocks in bits 48-63 and the queue's ray total in bits 0-47 (< 2.8e14
// rays per queue and launch). The block that takes the count to bq -- every fetch on q
// has returned by then -- folds the total into the caller's counter and re-arms q's
// counters for the slot's next launch. No fence is needed (a device-scope fence writes
// back the XCD's L2 on gfx950: measured +28 us per launch), and no collect kernel.
constexpr int kDoneShift = 48;
__device__ inline void block_epilogue(unsigned long long* tiles, unsigned long long* rays, int q, int bq,
                               unsigned long long total) {
    unsigned long long* const word = tiles + (kV0Queues + q) * kCtrStride;
    const unsigned long long inc = (1ull << kDoneShift) + total;
    const unsigned long long old = atomicAdd(word, inc);
    if ((old >> kDoneShift) == (unsigned long long)(bq - 1)) {
        const unsigned long long v = (old + inc) & ((1ull << kDoneShift) - 1ull);
        atomicExch(word, 0ull);
        atomicExch(tiles + q * kCtrStride, 0ull);
        if (v) atomicAdd(rays, v);
    }
}

constexpr int kQueueSlots = 64;
constexpr size_t kTileSetU64 = 2 * kV0Queues * kCtrStride;   // one v0 launch's counters

struct Context {
    bool ready = false;
    int device = 0;
    int num_cus = 0;
    // render streams created by lrt_stream_create: CU-masked, and the CUs they may use
    std::vector<std::pair<hipStream_t, int>> masked_streams;
    unsigned long long* d_tiles = nullptr;   // kQueueSlots x v0 counter sets (trace_kernel)
    float* d_lerp = nullptr;                 // kLerpTable lerp factors (host IEEE division)
    struct Wavefront {                       // v4 path state, grown on demand
        void* buf = nullptr;
        size_t bytes = 0;
        unsigned long long* rayp = nullptr;  // 16 ray-count partials
    } wf;
    unsigned tiles_next = 0;
    unsigned scene_version = 0;   // bumped by every scene upload (tile-order signatures)
    // The pool kernel's tile orders, one per recent render signature (tile_order()): per-tile
    // costs recorded by one launch, then a heaviest-first permutation for the later ones.
    struct TileOrder {
        uint64_t sig = 0;              // the render signature (geometry, camera, scene)
        uint64_t gkey = 0;             // its geometry only: views that can share an order
        long long ntiles = 0, cap = 0;
        int state = 0;                 // 0: free, 2: permutation ready once ev_rec has passed
        void* d_base = nullptr;        // one allocation: cost, sorted keys, tile ids, perm, sort scratch
        unsigned* d_cost = nullptr;    // written by the recording launch
        unsigned* d_keys = nullptr;
        int* d_ids = nullptr;          // 0..cap-1
        int* d_perm = nullptr;         // the live permutation, read by every later launch
        int* d_permb[2] = {nullptr, nullptr};   // its two buffers (the refining pass sorts into the other)
        int* d_sort_out = nullptr;     // where the sort behind the current recording launch writes
        int passes = 0;                // recording launches so far (1: the first; 2: refined)
        void* d_tmp = nullptr;
        size_t tmp_bytes = 0;
        hipEvent_t ev_rec = nullptr;   // after the recording launch and the sort behind it
        bool rec_done = false;         // ev_rec seen complete: later launches need not wait on it
        int donor = -1;                // the entry whose order the recording launch borrowed
        // the streams whose launches read d_perm / wrote d_cost, each with an event after its
        // last such launch: the entry is reused only once all of them have passed it
        std::vector<std::pair<hipStream_t, hipEvent_t>> uses;
        unsigned long long tick = 0;   // least recently used goes first
    };
    // Per-stream scratch of the pool kernel (colour slots, overflow stack), kept from launch to
    // launch: an allocation and a free around every launch put two more commands between
    // consecutive kernels of a stream (profiles/r5_s). Reuse on the same stream is ordered by the
    // stream itself; a buffer grows by a stream-ordered free + allocation on that stream. `ev` is
    // recorded behind the buffer's last use: a slot taken over by another stream (or idle for
    // kScratchIdle launches) is freed on the taking stream after waiting for it -- no device sync.
    struct Scratch {
        hipStream_t s = nullptr;
        void* p = nullptr;
        size_t bytes = 0;
        unsigned long long tick = 0;
        hipEvent_t ev = nullptr;
    };
    static constexpr unsigned long long kScratchIdle = 64;
    static constexpr int kScratchSlots = 8;
    Scratch scratch[kScratchSlots];
    static constexpr int kOrderSlots = 8;
    TileOrder order[kOrderSlots];
    unsigned long long order_tick = 0;
    hipStream_t stream = nullptr;
    int count = 0, nlights = 0;
    float4* d_sph = nullptr;
    float4* d_mats = nullptr;
    int* d_lights = nullptr;
    std::vector<lrt_sphere> spheres;
    std::vector<lrt_material> mats;
    // BVH (scenes with more than kBvhMinSpheres spheres)
    float4* d_bvh_nodes = nullptr;
    float4* d_bvh_lsph = nullptr;
    int* d_bvh_lid = nullptr;
    BvhView bvh{};   // geometry and the device pointers above (on: unused here)
    int bvh_on = 0;            // the scene has more than kBvhMinSpheres spheres: the BVH applies
    bool bvh_built = false;    // ... and has been built (ensure_bvh)
    int bvh_stack_levels = kBvhStackLevels;   // this scene's traversal depth (<= kBvhStackLevels)
    // uniform grid (the same scenes; lrt_grid.h): gv holds the device pointers and geometry,
    // gv.on = built; grid_pick = the policy's choice over the BVH (grid_suitable)
    uint2* d_grid_cells = nullptr;
    float4* d_grid_rsph = nullptr;
    int* d_grid_rid = nullptr;
    float4* d_grid_bsph = nullptr;
    int* d_grid_bid = nullptr;
    GridView gv{};
    bool grid_pick = false;
    bool grid_ok = false;      // any scene: the grid applies (LRT_F_GRID below kBvhMinSpheres)
    bool grid_built = false;   // ... and has been built (ensure_grid); gv.on then

    float* d_frame = nullptr;   // lrt_draw_test / lrt_render_host staging
    float4* d_col = nullptr;    // the pipelined host path's sample colours
    size_t col_bytes = 0;
    hipStream_t s_in = nullptr;   // its H2D copy stream
    static constexpr int kHostChunks = 8;
    hipEvent_t ev_in[kHostChunks] = {};
    hipEvent_t ev_ret = nullptr;  // the pipelined call's own work done (the look-ahead may follow)
    // lrt_draw_test's look-ahead (render_host_pipelined): the colours of the frame after the
    // last one, rendered on `stream` behind that call's work, for the call that asks for it
    struct Lookahead {
        bool on = false;
        lrt_render_desc d;            // the render they are (memcmp: descs are zero-filled)
        unsigned scene_version = 0;
        int cur = 0;                  // the buffer pair holding them (the other is free)
        float4* col[2] = {};
        size_t bytes[2] = {};
        unsigned long long* d_rays = nullptr;   // 2 counters
        hipStream_t stream = nullptr;  // CU-masked: leaves CUs for the lerps it runs beside
        hipEvent_t ev = nullptr;       // recorded after the look-ahead render
        hipEvent_t ev_render = nullptr;
    } ahead;
    float* d_feat[6] = {};      // lrt_render_host_ex feature staging
    size_t feat_bytes[6] = {};
    size_t frame_bytes = 0;
    unsigned long long* d_rays = nullptr;
    // multi-device renders (lrt_initialize_devices): this device's row shard, packed for
    // the exchange, and (device 0) the gathered shards
    float* d_shard = nullptr;
    size_t shard_bytes = 0;
    float* d_gath = nullptr;
    size_t gath_bytes = 0;
    float* d_pack = nullptr;   // the shard's RGB (the gather exchange)
    size_t pack_bytes = 0;
    unsigned long long* h_rays = nullptr;   // page-locked: the ray count's D2H stays asynchronous
    hipEvent_t ev_done = nullptr;   // this device's part of a multi-device render is enqueued
};

// One context per device in use: lrt_initialize binds the caller's current device (context
// 0); lrt_initialize_devices binds a list, and host renders are split over all of them.
// (Defined in lrt_api.hip; every access holds g_mu.)
constexpr int kMaxDevices = 16;
extern Context g_devs[kMaxDevices];
extern int g_ndev;   // contexts in use
extern int g_cur;    // the context the functions below act on (set under g_mu)
inline Context& ctx() { return g_devs[g_cur]; }

// Multi-device state (lrt_initialize_devices, lrt_multi.hip).
struct Multi {
    bool on = false;          // host renders are split over the g_ndev contexts
    bool gather = false;      // the shards go to device 0 (LRT_DEV_GATHER / LRT_DEV_PEER_COPY); else direct
    bool rccl = false;        // ... by RCCL (distinct devices); else peer copies
    int row_block = 8;        // rows per block of the row-block-cyclic split (LRT_ROW_BLOCK)
    ncclComm_t comms[kMaxDevices] = {};
};
extern Multi g_multi;

extern std::mutex g_mu;
extern char g_last_launch[256];   // lrt_last_launch(): the kernel instance of the last render call
extern thread_local std::string t_err;

int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);
#define LRT_HIP(call)                                            \
    do {                                                         \
        hipError_t _e = (call);                                  \
        if (_e != hipSuccess) return hip_fail(_e, #call);        \
    } while (0)

// Makes context k the one ctx() returns and its device the calling thread's current one, for
// the scope's lifetime (both restored after).
struct DeviceScope {
    int prev_cur, prev_dev = -1;
    explicit DeviceScope(int k) : prev_cur(g_cur) {
        g_cur = k;
        int dev = 0;
        if (hipGetDevice(&dev) == hipSuccess && dev != g_devs[k].device) {
            prev_dev = dev;
            (void)hipSetDevice(g_devs[k].device);
        }
    }
    ~DeviceScope() {
        if (prev_dev >= 0) (void)hipSetDevice(prev_dev);
        g_cur = prev_cur;
    }
};

// roctx ranges around the C-ABI's work entry points (SURVEY §5 tracing): rocprofv3
// --marker-trace shows each lrt_* call on the host timeline above the kernels it launched.
struct RoctxRange {
#if LRT_ROCTX
    explicit RoctxRange(const char* name) { roctxRangePushA(name); }
    ~RoctxRange() { roctxRangePop(); }
#else
    explicit RoctxRange(const char*) {}
#endif
};

// ---- lrt_scene.hip
extern const lrt_sphere kDefaultSpheres[9];   // parallel.cpp:15-51
extern const lrt_material kDefaultMats[9];
constexpr int kBvhMinSpheres = 16;   // scenes above this get the BVH and the grid
struct BvhHost {
    std::vector<float4> nodes, lsph;
    std::vector<int> lid;
    int big0 = 0, nbig = 0;
    float margin = 0.0f;
    float clo[3] = {0, 0, 0}, chi[3] = {0, 0, 0};   // exactness reach (BvhView)
    float f2near = 0.0f, rmax = 0.0f, rmin = 0.0f;
    int stack_levels = 1;   // traversal stack entries needed: one deferred sibling per level
};
void build_bvh_host(const lrt_sphere* s, int n, const std::vector<float4>& sph, BvhHost& out);
void bvh_view_host(const BvhHost& B, BvhView& bv);   // the view of B's host arrays
void free_scene(Context& c);
int pack_scene(const lrt_sphere* s, const lrt_material* m, int n, std::vector<float4>& sph,
               std::vector<float4>& mats, std::vector<int>& lights);
int upload_scene(Context& c, const lrt_sphere* s, const lrt_material* m, int n);
int ensure_bvh(Context& c);    // the structures on first use (lazy builds)
int ensure_grid(Context& c);
int camera_make(lrt_float3 lookFrom, lrt_float3 lookAt, lrt_float3 vup, float vfov, float aspect, float aperture,
                float focusDist, lrt_camera* out);
int camera_default(int w, int h, lrt_camera* out);

// ---- lrt_render.hip
int validate(const lrt_render_desc* d);
// At least `bytes` of device scratch for launches on stream s (Context::scratch).
// Has ev completed? An error left pending by an earlier asynchronous call is returned first (not
// cleared); only the "not ready" the query itself sets is cleared, so that it does not look like
// a later launch's error.
hipError_t event_done(hipEvent_t ev, bool* done);
hipError_t stream_scratch(hipStream_t s, size_t bytes, void** out);
// After the launch that used stream s's scratch: marks its last use (stream_scratch eviction).
hipError_t stream_scratch_used(hipStream_t s);
// lrt_kernel_timing (lrt_diag.h): events right around each render kernel launch on its stream
extern bool g_ktiming_on;
void kernel_timing_mark(hipStream_t s, int which);   // 0 before the kernel, 1 after
inline void kernel_timing(hipStream_t s, int which) {
    if (g_ktiming_on) kernel_timing_mark(s, which);
}
hipError_t occupancy(int* per_cu, const void* kern, int block, size_t lds);
const char* acc_name(int acc);
int pool_tiles(int pix, int xc, int rows);
// Tile pixels of a pool launch: the largest power of two <= cap whose pool fits a round and,
// above 64 px, still gives every resident wave a tile.
int pool_pixels(int frames, int xc, int rows, int cap);
// Largest pool tile for a launch that overlaps another stream's pool launch (lrt_render.hip).
#ifndef LRT_POOL_PIX_OVERLAP
#define LRT_POOL_PIX_OVERLAP 128
#endif
constexpr int kPoolPixOverlap = LRT_POOL_PIX_OVERLAP;
// Sixteenths of a launch's (lightest) tiles served as halves, alone and overlapped (launch_pool;
// config 2 alone 0.2580-0.2586 -> 0.2538-0.2558 ms at 5/16, 3/16 and 8/16 less, profiles/r6_v)
#ifndef LRT_POOL_SPLIT16_ALONE
#define LRT_POOL_SPLIT16_ALONE 5
#endif
#ifndef LRT_POOL_SPLIT16_OVERLAP
#define LRT_POOL_SPLIT16_OVERLAP 0
#endif
constexpr int kPoolSplit16Alone = LRT_POOL_SPLIT16_ALONE;
constexpr int kPoolSplit16Overlap = LRT_POOL_SPLIT16_OVERLAP;
// Is a pool launch of another stream than s still running (its scratch slot's last-use event)?
hipError_t other_stream_busy(hipStream_t s, bool* busy);
// sample mode's merge (merge_samples_kernel) on stream s
hipError_t launch_merge_samples(const float4* samp, float4* out, const float* lerp, int npix, int frame0, int frames,
                                size_t stride, const KernelArgs& a, int pix0, hipStream_t s);
int launch_wavefront(KernelArgs a, bool lds, hipStream_t s);
// colours_out / frame: see the definition
int render_device(const lrt_render_desc* d, float* d_buf, unsigned long long* d_rays, const lrt_features* feat,
                  hipStream_t s, float4* colours_out = nullptr, float* frame = nullptr);
int auto_kernel(const KernelArgs& a, const lrt_render_desc* d, bool feat, int pix_cap = 64);
#ifdef LRT_EXP_WAVETRACE
unsigned long long* wavetrace_buffer(size_t waves);
void wavetrace_dump(unsigned long long* d, size_t waves, hipStream_t s);
#endif
#ifdef LRT_EXP_SECSTATS
unsigned long long* secstats_buffer(hipStream_t s);
void secstats_dump(const unsigned long long* d_sec, hipStream_t s);
#endif

// ---- lrt_v0_d8.hip / lrt_v0_d64.hip: v0 launches for max_depth <= 8 / <= 64. colours: the
// pipelined host path's colours-only render (one frame lane, sample planes)
int launch_v0_d8(const KernelArgs& a, bool lds, int xc, int rows, int frames, bool feat, bool colours, hipStream_t s);
int launch_v0_d64(const KernelArgs& a, bool lds, int xc, int rows, int frames, bool feat, bool colours, hipStream_t s);
// ---- lrt_pool_d8.hip / lrt_pool_d64.hip
int launch_pool_d8(const KernelArgs& a, bool lds, int xc, int rows, int frames, int pix_cap, hipStream_t s);
int launch_pool_d64(const KernelArgs& a, bool lds, int xc, int rows, int frames, int pix_cap, hipStream_t s);

// ---- lrt_order.hip
bool pool_order_on();
int pool_probe_mode();
int order_used(Context::TileOrder& e, hipStream_t s);
// record: 0 none, 1 the signature's first recording launch, 2 its refining pass (tile_order)
int tile_order(KernelArgs& a, int kPix, long long ntiles, int& record, Context::TileOrder* users[2], hipStream_t s);
// the tile-cost probe of a recording launch: costs into o.d_cost, heaviest-first into o.d_perm
hipError_t launch_tile_probe(const KernelArgs& a, int acc, Context::TileOrder& o, int ntiles, int TX, int TY,
                             size_t bstk, hipStream_t s);
// ---- lrt_sort.hip
hipError_t sort_tiles_desc(const unsigned* cost_in, unsigned* keys_out, const int* ids_in, int* perm_out, int n,
                           void* tmp, size_t* tmp_bytes, hipStream_t s, unsigned end_bit = 32);
hipError_t fill_iota(int* v, int n, hipStream_t s);

// ---- lrt_hostpath.hip
int ensure_frame(size_t bytes);
float* host_pinned(float* buf);
// drawtest: the reference API's call (lrt_draw_test: the look-ahead render)
int create_lookahead_stream(Context& c);
int render_host(const lrt_render_desc* d, float* buf, long long* out_rays, const lrt_features* feat = nullptr,
                bool drawtest = false);

// ---- lrt_multi.hip
int render_host_multi(const lrt_render_desc* d, float* buf, size_t bytes, long long* out_rays);

// ---- lrt_frame.hip
hipError_t launch_unshard(const float4* src, float4* dst, int width, int height, int rb, int period, int maxRows,
                          hipStream_t s);
hipError_t launch_pack_rgb(const float4* src, float* dst, size_t n, hipStream_t s);
hipError_t launch_unshard_rgb(const float* src, float4* dst, int width, int height, int rb, int period, int maxRows,
                              hipStream_t s);

// ---- lrt_api.hip
int init_context(Context& c, int dev);
void free_context(Context& c);

}  // namespace lrt
