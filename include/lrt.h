/* lrt.h — C-ABI of the MI355X path tracer (liblrt_hip.so).
 *
 * Drop-in boundary for the reference's src/cpu renderer API
 * (Sefaice/LearnRayTracing src/cpu/parallel.h:6-8):
 *
 *     void InitializeTest();                                         -> lrt_initialize
 *     void ShutdownTest();                                           -> lrt_shutdown
 *     void DrawTest(float time, int frameCount, int screenWidth,
 *                   int screenHeight, float* backbuffer, int& outRayCount);
 *                                                                    -> lrt_draw_test
 *
 * plus the extended entry points the multi-GPU / benchmark callers need
 * (runtime scene and camera, device-resident progressive buffer, S samples per
 * call, D bounces, row-block-cyclic sharding, 64-bit ray counts).
 *
 * Plain types and pointers only. Every function returns LRT_OK (0) or a negative
 * LRT_E_* code; lrt_last_error() describes the last failure of the calling thread.
 * Not re-entrant per process (like the reference's global scheduler, parallel.cpp:229).
 */
#ifndef LRT_H
#define LRT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LRT_OK 0
#define LRT_E_INVALID (-1) /* bad argument (sizes, pointers, scene contents)        */
#define LRT_E_HIP (-2)     /* a HIP runtime call failed                              */
#define LRT_E_STATE (-3)   /* lrt_initialize() not called / already shut down        */
#define LRT_E_NOMEM (-4)   /* device allocation failed                               */

/* Material::Type, parallel.cpp:31 */
#define LRT_LAMBERT 0
#define LRT_METAL 1
#define LRT_DIELECTRIC 2

/* Reference kMaxDepth (parallel.cpp:12): lrt_draw_test allows this many scatter events. */
#define LRT_REFERENCE_MAX_DEPTH 20
/* Largest scene the device path accepts (spheres + materials are staged per workgroup). */
#define LRT_MAX_SPHERES 4096

/* float3, maths.h:10-61 (12 bytes, no padding) */
typedef struct lrt_float3 { float x, y, z; } lrt_float3;

/* Sphere, maths.h:156-163 (16 bytes) */
typedef struct lrt_sphere { lrt_float3 center; float radius; } lrt_sphere;

/* Material, parallel.cpp:29-37 (36 bytes: type @0, albedo @4, emissive @16,
 * roughness @28, ri @32). type is the enum's int value. */
typedef struct lrt_material {
    int32_t type;
    lrt_float3 albedo;
    lrt_float3 emissive;
    float roughness;
    float ri;
} lrt_material;

/* Camera, maths.h:176-225 (88 bytes: the member order of the reference). */
typedef struct lrt_camera {
    lrt_float3 origin;
    lrt_float3 a, u, r;
    lrt_float3 lowerLeftCorner;
    lrt_float3 horizontalVec;
    lrt_float3 verticalVec;
    float lensRadius;
} lrt_camera;

/* One render call (the extended form of DrawTest, parallel.cpp:297-323).
 *
 * The image is width x height; pixel (x, y) has row 0 at the bottom (v grows with y,
 * maths.h:198,214). The call renders the column window [x0, x0 + x_count) of
 * row_count LOCAL rows; local row ly maps to the global row
 *     y = y0 + (ly / row_block) * row_block * row_period + row_phase * row_block + ly % row_block
 * (row_period = 1, row_phase = 0 gives the contiguous rows y0 .. y0 + row_count - 1;
 *  row_period = G, row_phase = g gives GPU g's share of a row-block-cyclic split).
 * For each pixel it runs samples frame0 .. frame0 + frames - 1 in order; sample f
 * uses the per-pixel XorShift32 stream seeded with
 *     ((uint32)(x * 1973 + y * 9277 + f * 26699)) | 1
 * and is blended into the buffer with the reference's progressive lerp
 * (parallel.cpp:262,280-286): rgb = prev * (f / (f + 1)) + col * (1 - f / (f + 1)).
 * max_depth is the number of scatter events a path may take (the reference's
 * kMaxDepth = 20; "8 bounces" = 8). */
typedef struct lrt_render_desc {
    lrt_camera camera;
    int32_t width, height;
    int32_t x0, x_count;
    int32_t y0, row_count;
    int32_t row_block, row_period, row_phase;
    int32_t frame0, frames;
    int32_t max_depth;
    int32_t flags; /* LRT_F_* */
} lrt_render_desc;

#define LRT_F_NONE 0
#define LRT_F_SCENE_GLOBAL 1 /* read the scene from global memory instead of LDS staging */
#define LRT_F_SIMPLE 2       /* v0 kernel (the default): the reference's per-pixel loop,
                                a pixel's frames spread over adjacent lanes, persistent
                                single-wave blocks fed from tile queues               */
#define LRT_F_NO_BVH 32      /* scan every sphere (the reference's HitWorld loop) even
                                when the scene has a BVH (> 16 spheres)                */
#define LRT_F_NO_DOUBLE_LIGHT 64 /* opt-in GL-path rule (fragmentShader.fs.glsl:430,456-457,
                                "doMaterialE"): a scatter event reached through a Lambert
                                bounce does not add its emissive again (that light was
                                sampled explicitly); the terminating hit always adds it.
                                Off by default: the CPU reference double counts
                                (parallel.cpp:214). v0 kernel only.                   */
#define LRT_F_WAVEFRONT 256  /* v4: wavefront (breadth-first) path tracing: path state in
                                HBM, closest-hit and per-material shading kernels over
                                compacted queues, frame planes merged in order. No
                                lrt_features.                                          */

#define LRT_F_POOL 512       /* v5 kernel: the v0 loop with sample-pool regeneration: a lane
                                whose path ends takes the wave's next pixel-sample at once;
                                colours are lerped in frame order per pixel when the pool
                                is done. No lrt_features.                             */
#define LRT_F_BVH 1024       /* closest hits through the 4-wide BVH even where the library
                                would pick the uniform grid (scenes above 16 spheres) */
#define LRT_F_GRID 2048      /* closest hits through the uniform grid (lrt_grid.h) even where
                                the library would pick the BVH; same bits either way */
/* With none of SIMPLE / WAVEFRONT / POOL set the library picks v0 or v5 per call. Any bit not
 * defined above (4, 8, 16 and 128 belonged to kernels removed in rounds 2-3) is rejected with
 * LRT_E_INVALID. */

/* ---- the reference API (parallel.h:6-8) ---------------------------------- */

/* InitializeTest (parallel.cpp:231-235): binds the calling thread's current HIP device,
 * creates the stream, uploads the reference's default 9-sphere scene (parallel.cpp:15-51). */
int lrt_initialize(void);

/* ShutdownTest (parallel.cpp:237-240): frees every device resource. */
int lrt_shutdown(void);

/* DrawTest (parallel.cpp:297-323): one progressive frame of the current scene with
 * DrawTest's camera (parallel.cpp:299-307) and kMaxDepth 20 into a caller-owned host
 * buffer of screenWidth*screenHeight*4 floats (RGBA stride, alpha untouched), blocking.
 * `time` is accepted and unused, as in the reference. */
int lrt_draw_test(float time, int frameCount, int screenWidth, int screenHeight,
                  float* backbuffer, int* outRayCount);

/* ---- multi-GPU (one process) ---------------------------------------------- */

/* InitializeTest over several devices (BASELINE config 5: the frame row-tiled across the
 * node's GPUs). Instead of lrt_initialize: n device ids (n = 0 and device_ids = NULL: every
 * visible device). Afterwards lrt_draw_test and lrt_render_host(_ex without features) split
 * the caller's rows over all of them in blocks of 8 rows dealt round-robin (row-block-cyclic;
 * LRT_ROW_BLOCK overrides); each device copies its rows' previous values from the caller's
 * buffer (page-locked for the call), renders them, and by default copies them straight back
 * over its own PCIe link. With LRT_DEV_GATHER the shards' RGB is gathered into the first
 * device instead -- ncclCommInitAll + a grouped ncclGather (RCCL, over xGMI) when the ids are
 * distinct, device-to-device copies when an id repeats (RCCL refuses two ranks on one GPU) or
 * with LRT_DEV_PEER_COPY -- which assembles the frame and copies it to the caller. The result
 * is bit-identical to one device either way. The other calls (lrt_render_device, streams,
 * scene) act on the first device; lrt_set_scene updates every device. lrt_shutdown releases
 * all. */
#define LRT_DEV_PEER_COPY 1 /* gather, with device-to-device copies instead of RCCL */
#define LRT_DEV_GATHER 2    /* gather the shards into the first device (RCCL when the ids are distinct) */
int lrt_initialize_devices(int n, const int* device_ids, int flags);
/* Bytes one multi-device host render of an x_count x rows window moves between the devices
 * and the caller: *direct = the RGBA rows each device copies back over its own link (the
 * default exchange); *gather_xgmi = the packed RGB (12 B per pixel) the other devices' shards
 * send to the first one (LRT_DEV_GATHER). No device is touched. */
int lrt_exchange_bytes(int x_count, int rows, int row_block, int devices, long long* direct, long long* gather_xgmi);
/* Devices in use (0 before lrt_initialize / lrt_initialize_devices). */
int lrt_device_count(void);

/* ---- extended API -------------------------------------------------------- */

const char* lrt_last_error(void);
/* Library version string ("lrt-mi355x <semver> gfx950"). */
const char* lrt_version(void);
/* The kernel instance the last render call on any thread launched, as "key=value" words
 * (e.g. "kernel=trace_kernel maxd=8 lds=1 bvh=1 split=16 samp=0 feat=0 ns=0 grid=4096
 * tasks=..."): lets tests and benchmarks name the exact instance they exercised. */
const char* lrt_last_launch(void);

/* Camera constructor (maths.h:183-202). */
int lrt_camera_make(lrt_float3 lookFrom, lrt_float3 lookAt, lrt_float3 vup, float vfov,
                    float aspect, float aperture, float focusDist, lrt_camera* out);
/* DrawTest's camera for a width x height image (parallel.cpp:299-307). */
int lrt_camera_default(int width, int height, lrt_camera* out);

/* Replace the scene (the reference's s_Spheres / s_SphereMats, parallel.cpp:15-51).
 * 1 <= count <= LRT_MAX_SPHERES; material types must be 0..2. Emissive spheres are
 * those with any emissive channel > 0 (parallel.cpp:96). */
int lrt_set_scene(const lrt_sphere* spheres, const lrt_material* materials, int count);
/* The scene the devices hold (what lrt_set_scene last uploaded, or the default scene):
 * *count spheres; copies them when capacity >= *count. */
int lrt_get_scene(lrt_sphere* spheres, lrt_material* materials, int capacity, int* count);

/* Copy the reference's default scene (9 spheres) into caller arrays of >= 9 entries. */
int lrt_default_scene(lrt_sphere* spheres, lrt_material* materials, int capacity, int* count);

/* Render into a DEVICE buffer of row_count * x_count RGBA float quads (row-major,
 * local rows), adding the counted rays into *d_rays (device uint64, caller-zeroed).
 * Asynchronous on `stream` (a hipStream_t, used as given: NULL is the default stream), and
 * ordered only against that stream: a buffer or counter filled on another stream must be
 * ordered before the call by the caller (an event, or a stream wait). */
int lrt_render_device(const lrt_render_desc* desc, float* d_backbuffer,
                      unsigned long long* d_rays, void* stream);

/* lrt_render_device plus the multi-GPU frame exchange fused into the render: every finished
 * pixel is also stored, as RGBA, into d_frame -- the whole width x height frame, row-major --
 * at its global row (the row map above). d_frame may be another device's memory opened with
 * lrt_ipc_open (one process per GPU) or peer-accessible memory: each rank's render writes its
 * rows straight into rank 0's frame over xGMI, with no pack, gather or assembly launch; the
 * frame is complete once every rank's render has completed (e.g. after a barrier). */
int lrt_render_device_to_frame(const lrt_render_desc* desc, float* d_backbuffer,
                               unsigned long long* d_rays, float* d_frame, void* stream);

/* Device memory shareable across processes (hipIpc*) for that exchange: lrt_ipc_alloc makes a
 * zeroed buffer of `bytes` on the first device and its handle (LRT_IPC_HANDLE_BYTES bytes, to
 * send to the other processes); lrt_ipc_open maps a handle from another process (peer access
 * enabled lazily); lrt_ipc_close unmaps it; lrt_ipc_free frees an lrt_ipc_alloc buffer. */
#define LRT_IPC_HANDLE_BYTES 64
int lrt_ipc_alloc(size_t bytes, void** d_ptr, void* handle);
int lrt_ipc_free(void* d_ptr);
int lrt_ipc_open(const void* handle, void** d_ptr);
int lrt_ipc_close(void* d_ptr);

/* Same on a HOST buffer: H2D of prev, render, D2H, blocking. *out_rays = counted rays. */
int lrt_render_host(const lrt_render_desc* desc, float* backbuffer, long long* out_rays);

/* Opt-in first-hit features of the reference's GL path (fragmentShader.fs.glsl:444-451,
 * 494-568): per pixel, running means (the backbuffer's lerp, parallel.cpp:282) of the
 * first hit's normal, world position and material albedo (zero on a camera-ray miss),
 * and running standard deviations (AdaptiveStdvar, :494-497, pow(x,2) taken as x*x) of
 * the linear colour, the normal and the world position. Each non-NULL buffer has the
 * backbuffer's shape (row_count * x_count RGBA float quads, alpha untouched) and is
 * read and updated in place; features update for frames f <= max_frame (the GL path
 * uses 4), every frame if max_frame < 0. The backbuffer is bit-identical to a render
 * without features. v0 kernel only; a feature render keeps each pixel on one lane. */
typedef struct lrt_features {
    float* normal;
    float* world_pos;
    float* albedo;
    float* color_std;
    float* normal_std;
    float* world_pos_std;
    int32_t max_frame;
    int32_t reserved;   /* 0 */
} lrt_features;

/* lrt_render_device / lrt_render_host with features (device resp. host buffers;
 * features == NULL is the plain call). */
int lrt_render_device_ex(const lrt_render_desc* desc, float* d_backbuffer,
                         unsigned long long* d_rays, const lrt_features* d_features, void* stream);
int lrt_render_host_ex(const lrt_render_desc* desc, float* backbuffer, long long* out_rays,
                       const lrt_features* features);

/* A render stream for lrt_render_device(_ex) that leaves the last `reserved_cus` CUs of the
 * device free (hipExtStreamCreateWithCUMask), so that work on other streams -- the RCCL
 * gather of the previous frame -- can run beside the persistent render kernel instead of
 * waiting for its workgroups to retire; renders on it size their grid to the remaining
 * CUs. Destroy with lrt_stream_destroy (lrt_shutdown destroys any left). */
int lrt_stream_create(int reserved_cus, void** stream);
int lrt_stream_destroy(void* stream);

/* Page-locked host memory for a backbuffer (hipHostMalloc; contents undefined, like the
 * `new float[]` of main.cpp:40 it replaces). lrt_draw_test / lrt_render_host(_ex without
 * features) detect such a buffer -- or any other page-locked one -- and render it in place
 * over PCIe instead of staging it through device memory either side of the kernel
 * (LRT_HOST_ZEROCOPY=0 turns that off). Free with lrt_host_free. */
int lrt_host_alloc(size_t bytes, void** out);
int lrt_host_free(void* p);
/* A PAGEABLE host backbuffer (the reference's `new float[]`, main.cpp:40) is page-locked by
 * lrt_draw_test / lrt_render_host for the duration of that one call (hipHostRegister when it
 * starts, hipHostUnregister before it returns) and takes the page-locked paths. The library
 * keeps nothing of the caller's buffer between calls: the caller may free it, or reuse or
 * remap its address, at any time between calls -- DrawTest's own contract (parallel.h:8).
 * LRT_HOST_REGISTER=0 stages pageable buffers instead. */

/* Number of local rows GPU `phase` owns in a row-block-cyclic split of `height` rows
 * into blocks of row_block rows dealt over `period` GPUs. */
int lrt_shard_rows(int height, int row_block, int period, int phase);

/* Frame assembly after a gather: src holds `period` shard buffers of max_rows rows each
 * (max_rows = lrt_shard_rows(height, row_block, period, 0)), shard g at
 * src + g * max_rows * width * 4; dst receives the full width x height RGBA image.
 * Device pointers, asynchronous on stream. */
int lrt_unshard_rows(const float* d_src, float* d_dst, int width, int height, int row_block,
                     int period, void* stream);

/* The RGB-only form of the exchange (12 of 16 bytes per pixel cross the interconnect; the
 * render never writes alpha): lrt_pack_rgb copies npix RGBA quads to packed RGB triples;
 * lrt_unshard_rows_rgb assembles `period` packed shards of max_rows rows each (shard g at
 * d_src_rgb + g * max_rows * width * 3) into the RGBA frame, leaving its alpha untouched.
 * Device pointers, asynchronous on stream. */
int lrt_pack_rgb(const float* d_rgba, float* d_rgb, long long npix, void* stream);
int lrt_unshard_rows_rgb(const float* d_src_rgb, float* d_dst, int width, int height, int row_block,
                         int period, void* stream);

/* Present step (main.cpp:109-141 LinearToSRGB + BGRA8 pack, GDI blit removed):
 * d_rgba (width*height*4 floats) -> d_bgra (width*height uint32, b | g<<8 | r<<16). */
int lrt_present_bgra8(const float* d_rgba, uint32_t* d_bgra, int width, int height, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LRT_H */
