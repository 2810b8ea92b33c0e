// TEST INFRASTRUCTURE ONLY — never linked into the product (learnraytracing_amd/).
//
// Thin extern "C" driver around the reference's OWN hot-path sources, compiled
// where they lie under /root/reference (nothing is copied into this repo):
//   /root/reference/src/cpu/maths.cpp    (XorShift32, samplers, HitSphere)
//   /root/reference/src/cpu/parallel.cpp (scene, HitWorld, Scatter, Trace, TraceRowJob, DrawTest)
// Built by oracle/Makefile into oracle/_ref/libref.so (git-ignored, travels to the GPU box).
//
// Including the .cpp files into this translation unit gives access to their
// `static` symbols (s_RndState, Trace, TraceRowJob, JobData, s_Spheres,
// s_SphereMats) WITHOUT editing the reference. Everything below only drives them.
//
// Modes:
//   R  reference stream: one global RNG from s_RndState = 1, TraceRowJob(0,H) per
//      frame, single thread (config 1; parallel.cpp:254-294 exactly as written).
//   P  per-pixel seeded: s_RndState = seed(x,y,f) before each pixel, then the body of
//      TraceRowJob (parallel.cpp:270-286) with the reference's own Trace() started at
//      depth kMaxDepth - D so that exactly D scatter events are allowed
//      (parallel.cpp:12,212).
//   F  fuzz: Mode P after overwriting s_Spheres / s_SphereMats (non-const statics,
//      parallel.cpp:15,40; kSphereCount stays 9).
#include <stdint.h>
#include <string.h>
#include <unistd.h>
#include <sys/mman.h>
#include <sys/wait.h>

#include "maths.cpp"
#include "parallel.cpp"

namespace {
Sphere g_defaultSpheres[kSphereCount];
Material g_defaultMats[kSphereCount];
bool g_saved = false;

void SaveDefaults() {
    if (g_saved) return;
    memcpy(g_defaultSpheres, s_Spheres, sizeof(s_Spheres));
    memcpy(g_defaultMats, s_SphereMats, sizeof(s_SphereMats));
    g_saved = true;
}

// Seed of the per-pixel stream: the constants of the reference's alternative seed
// (fragmentShader.fs.glsl:517) evaluated in uint32 on integer pixel indices.
inline uint32_t PixelSeed(uint32_t x, uint32_t y, uint32_t f) {
    return (x * 1973u + y * 9277u + f * 26699u) | 1u;
}

// Camera exactly as DrawTest builds it (parallel.cpp:299-307).
Camera DefaultCamera(int w, int h) {
    float3 lookfrom(0, 2, 3);
    float3 lookat(0, 0, 0);
    float distToFocus = 3;
    float aperture = 0.1f;
    return Camera(lookfrom, lookat, float3(0, 1, 0), 60, float(w) / float(h), aperture, distToFocus);
}

Camera CameraFromArray(const float* c) {
    // layout (22 floats): origin, a, u, r, lowerLeftCorner, horizontalVec, verticalVec, lensRadius
    Camera cam(float3(0, 0, 1), float3(0, 0, 0), float3(0, 1, 0), 60, 1, 0, 1);
    cam.origin = float3(c[0], c[1], c[2]);
    cam.a = float3(c[3], c[4], c[5]);
    cam.u = float3(c[6], c[7], c[8]);
    cam.r = float3(c[9], c[10], c[11]);
    cam.lowerLeftCorner = float3(c[12], c[13], c[14]);
    cam.horizontalVec = float3(c[15], c[16], c[17]);
    cam.verticalVec = float3(c[18], c[19], c[20]);
    cam.lensRadius = c[21];
    return cam;
}

void CameraToArray(const Camera& cam, float* c) {
    const float3* v[7] = {&cam.origin, &cam.a, &cam.u, &cam.r, &cam.lowerLeftCorner,
                          &cam.horizontalVec, &cam.verticalVec};
    for (int i = 0; i < 7; ++i) {
        c[3 * i + 0] = v[i]->x;
        c[3 * i + 1] = v[i]->y;
        c[3 * i + 2] = v[i]->z;
    }
    c[21] = cam.lensRadius;
}

// The per-pixel body of TraceRowJob (parallel.cpp:270-286) under a per-pixel seed.
// `pix` points at the RGBA quad of the pixel; alpha is left untouched.
inline void ModePPixel(const Camera& cam, int w, int h, int x, int y, int frame, int depth,
                       float* pix, long long& rays) {
    float invWidth = 1.0f / w;
    float invHeight = 1.0f / h;
    float lerpFac = float(frame) / float(frame + 1);
    s_RndState = PixelSeed((uint32_t)x, (uint32_t)y, (uint32_t)frame);
    int rayCount = 0;
    float u = float(x + RandomFloat01()) * invWidth;
    float v = float(y + RandomFloat01()) * invHeight;
    Ray r = cam.GetRay(u, v);
    float3 col = Trace(r, kMaxDepth - depth, rayCount);
    float3 prev(pix[0], pix[1], pix[2]);
    col = prev * lerpFac + col * (1 - lerpFac);
    pix[0] = col.x;
    pix[1] = col.y;
    pix[2] = col.z;
    rays += rayCount;
}

void RenderRowsP(const Camera& cam, int w, int h, int x0, int xc, int y0, int yc, int frame0,
                 int frames, int depth, float* buf, long long& rays, int rowStart, int rowStep) {
    for (int ly = rowStart; ly < yc; ly += rowStep)
        for (int lx = 0; lx < xc; ++lx) {
            float* pix = buf + ((size_t)ly * xc + lx) * 4;
            for (int f = frame0; f < frame0 + frames; ++f)
                ModePPixel(cam, w, h, x0 + lx, y0 + ly, f, depth, pix, rays);
        }
}
}  // namespace

extern "C" {

int ref_scene_count(void) { return kSphereCount; }

// spheres: 4 floats each (center xyz, radius); mats: 9 floats each
// (type, albedo xyz, emissive xyz, roughness, ri).
void ref_get_scene(float* spheres, float* mats) {
    SaveDefaults();
    for (int i = 0; i < kSphereCount; ++i) {
        spheres[4 * i + 0] = s_Spheres[i].center.x;
        spheres[4 * i + 1] = s_Spheres[i].center.y;
        spheres[4 * i + 2] = s_Spheres[i].center.z;
        spheres[4 * i + 3] = s_Spheres[i].radius;
        const Material& m = s_SphereMats[i];
        float* o = mats + 9 * i;
        o[0] = (float)m.type;
        o[1] = m.albedo.x; o[2] = m.albedo.y; o[3] = m.albedo.z;
        o[4] = m.emissive.x; o[5] = m.emissive.y; o[6] = m.emissive.z;
        o[7] = m.roughness; o[8] = m.ri;
    }
}

void ref_set_scene(const float* spheres, const float* mats) {
    SaveDefaults();
    for (int i = 0; i < kSphereCount; ++i) {
        s_Spheres[i].center = float3(spheres[4 * i], spheres[4 * i + 1], spheres[4 * i + 2]);
        s_Spheres[i].radius = spheres[4 * i + 3];
        const float* o = mats + 9 * i;
        s_SphereMats[i].type = (Material::Type)(int)o[0];
        s_SphereMats[i].albedo = float3(o[1], o[2], o[3]);
        s_SphereMats[i].emissive = float3(o[4], o[5], o[6]);
        s_SphereMats[i].roughness = o[7];
        s_SphereMats[i].ri = o[8];
    }
}

void ref_reset_scene(void) {
    SaveDefaults();
    memcpy(s_Spheres, g_defaultSpheres, sizeof(s_Spheres));
    memcpy(s_SphereMats, g_defaultMats, sizeof(s_SphereMats));
}

// ---- known-answer probes of maths.{h,cpp} -----------------------------------
void ref_xorshift(uint32_t seed, int n, uint32_t* out) {
    s_RndState = seed;
    for (int i = 0; i < n; ++i) out[i] = XorShift32();
}
void ref_random01(uint32_t seed, int n, float* out) {
    s_RndState = seed;
    for (int i = 0; i < n; ++i) out[i] = RandomFloat01();
}
// kind 0: RandomInUnitDisk, 1: RandomUnitVector, 2: RandomInUnitSphere. Returns end state.
uint32_t ref_sampler(int kind, uint32_t seed, int n, float* out3) {
    s_RndState = seed;
    for (int i = 0; i < n; ++i) {
        float3 p = kind == 0 ? RandomInUnitDisk() : kind == 1 ? RandomUnitVector() : RandomInUnitSphere();
        out3[3 * i] = p.x; out3[3 * i + 1] = p.y; out3[3 * i + 2] = p.z;
    }
    return s_RndState;
}
// ray (o, d) goes through the Ray ctor (normalises d). out: pos xyz, normal xyz, t.
int ref_hit_sphere(const float* o, const float* d, const float* sph, float tMin, float tMax, float* out) {
    Ray r(float3(o[0], o[1], o[2]), float3(d[0], d[1], d[2]));
    Hit h;
    bool hit = HitSphere(r, Sphere(float3(sph[0], sph[1], sph[2]), sph[3]), tMin, tMax, h);
    if (hit) {
        out[0] = h.pos.x; out[1] = h.pos.y; out[2] = h.pos.z;
        out[3] = h.normal.x; out[4] = h.normal.y; out[5] = h.normal.z;
        out[6] = h.t;
    }
    return hit ? 1 : 0;
}
// HitWorld over the current scene. Returns id or -1; out as ref_hit_sphere.
int ref_hit_world(const float* o, const float* d, float tMin, float tMax, float* out) {
    Ray r(float3(o[0], o[1], o[2]), float3(d[0], d[1], d[2]));
    Hit h;
    int id = -1;
    if (!HitWorld(r, tMin, tMax, h, id)) return -1;
    out[0] = h.pos.x; out[1] = h.pos.y; out[2] = h.pos.z;
    out[3] = h.normal.x; out[4] = h.normal.y; out[5] = h.normal.z;
    out[6] = h.t;
    return id;
}
// HitWorld's loop (parallel.cpp:54-73) over an arbitrary sphere array: the reference's own
// HitSphere (maths.cpp:51-94) on each sphere in index order with the shrinking closestT,
// for scenes other than the 9 static ones (the accelerated closest-hit structures' checks).
// spheres: 4 floats each (center xyz, radius). Returns id or -1; out as ref_hit_sphere.
int ref_hit_spheres(const float* o, const float* d, const float* spheres, int n, float tMin, float tMax,
                    float* out) {
    Ray r(float3(o[0], o[1], o[2]), float3(d[0], d[1], d[2]));
    Hit tmp, h;
    int id = -1;
    float closestT = tMax;
    for (int i = 0; i < n; ++i) {
        const float* s = spheres + 4 * i;
        if (HitSphere(r, Sphere(float3(s[0], s[1], s[2]), s[3]), tMin, closestT, tmp)) {
            h = tmp;
            closestT = tmp.t;
            id = i;
        }
    }
    if (id < 0) return -1;
    out[0] = h.pos.x; out[1] = h.pos.y; out[2] = h.pos.z;
    out[3] = h.normal.x; out[4] = h.normal.y; out[5] = h.normal.z;
    out[6] = h.t;
    return id;
}
// Batched form: n_rays rays (o.xyz, d.xyz each) -> ids[i], ts[i] (t = 0 when no hit).
void ref_hit_spheres_batch(const float* rays, int n_rays, const float* spheres, int n, int* ids, float* ts) {
    float out[7];
    for (int i = 0; i < n_rays; ++i) {
        ids[i] = ref_hit_spheres(rays + 6 * i, rays + 6 * i + 3, spheres, n, kMinT, kMaxT, out);
        ts[i] = ids[i] >= 0 ? out[6] : 0.0f;
    }
}
float ref_schlick(float c, float ri) { return schlick(c, ri); }
int ref_refract(const float* v, const float* n, float nint, float* out) {
    float3 o;
    bool ok = refract(float3(v[0], v[1], v[2]), float3(n[0], n[1], n[2]), nint, o);
    if (ok) { out[0] = o.x; out[1] = o.y; out[2] = o.z; }
    return ok ? 1 : 0;
}
void ref_reflect(const float* v, const float* n, float* out) {
    float3 o = reflect(float3(v[0], v[1], v[2]), float3(n[0], n[1], n[2]));
    out[0] = o.x; out[1] = o.y; out[2] = o.z;
}
void ref_default_camera(int w, int h, float* out22) { CameraToArray(DefaultCamera(w, h), out22); }
void ref_make_camera(const float* from, const float* at, const float* up, float vfov, float aspect,
                     float aperture, float focus, float* out22) {
    Camera c(float3(from[0], from[1], from[2]), float3(at[0], at[1], at[2]), float3(up[0], up[1], up[2]),
             vfov, aspect, aperture, focus);
    CameraToArray(c, out22);
}
// GetRay under an explicit RNG state; out: orig xyz, dir xyz. Returns the end state.
uint32_t ref_get_ray(const float* cam22, uint32_t seed, float u, float v, float* out6) {
    Camera cam = CameraFromArray(cam22);
    s_RndState = seed;
    Ray r = cam.GetRay(u, v);
    out6[0] = r.orig.x; out6[1] = r.orig.y; out6[2] = r.orig.z;
    out6[3] = r.dir.x; out6[4] = r.dir.y; out6[5] = r.dir.z;
    return s_RndState;
}
// One reference Trace() of a camera-space ray under an explicit RNG state.
// out: rgb, returns counted rays.
int ref_trace(const float* o, const float* d, int depth, uint32_t seed, float* out3) {
    s_RndState = seed;
    int rays = 0;
    float3 c = Trace(Ray(float3(o[0], o[1], o[2]), float3(d[0], d[1], d[2])), kMaxDepth - depth, rays);
    out3[0] = c.x; out3[1] = c.y; out3[2] = c.z;
    return rays;
}

// One reference Scatter() (parallel.cpp:78-196) of the static scene's material `id` (its
// own table entry, so the `&mat == &smat` self test sees the address it expects) under
// an explicit RNG state. ray: o, d (through the Ray ctor); rec: pos, normal, t.
// out12: attenuation, scattered orig, scattered dir, lightE. Returns Scatter's bool;
// *rays = counted shadow rays, *state = s_RndState after.
int ref_scatter(int id, const float* ray, const float* rec, uint32_t seed, float* out12, int* rays,
                uint32_t* state) {
    Ray r(float3(ray[0], ray[1], ray[2]), float3(ray[3], ray[4], ray[5]));
    Hit h;
    h.pos = float3(rec[0], rec[1], rec[2]);
    h.normal = float3(rec[3], rec[4], rec[5]);
    h.t = rec[6];
    float3 att(0, 0, 0), lightE(0, 0, 0);
    Ray scattered(float3(0, 0, 0), float3(0, 0, 1));
    scattered.dir = float3(0, 0, 0);
    int n = 0;
    s_RndState = seed;
    const bool ok = Scatter(s_SphereMats[id], r, h, att, scattered, lightE, n);
    const float3* v[4] = {&att, &scattered.orig, &scattered.dir, &lightE};
    for (int k = 0; k < 4; ++k) {
        out12[3 * k] = v[k]->x;
        out12[3 * k + 1] = v[k]->y;
        out12[3 * k + 2] = v[k]->z;
    }
    *rays = n;
    *state = s_RndState;
    return ok ? 1 : 0;
}

// ---- frame renderers ----------------------------------------------------------
// Mode R: TraceRowJob(0, H) once per frame from the global stream (s_RndState = 1 at
// the start of frame0's call only when reset != 0). buf: w*h*4 floats, caller-zeroed.
long long ref_render_mode_r(int w, int h, int frame0, int frames, int reset, float* buf) {
    if (reset) s_RndState = 1;
    Camera cam = DefaultCamera(w, h);
    long long rays = 0;
    for (int f = frame0; f < frame0 + frames; ++f) {
        JobData data;
        data.time = 0;
        data.frameCount = f;
        data.screenWidth = w;
        data.screenHeight = h;
        data.backbuffer = buf;
        data.cam = &cam;
        data.rayCount = 0;
        TraceRowJob(0, (uint32_t)h, 0, &data);
        rays += data.rayCount;
    }
    return rays;
}

// Mode P (and F after ref_set_scene) over the window [x0,x0+xc) x [y0,y0+yc) of a w x h
// image. cam22 == NULL -> DrawTest's camera. buf: xc*yc*4 floats (row-major window).
long long ref_render_mode_p(int w, int h, int x0, int xc, int y0, int yc, int frame0, int frames,
                            int depth, const float* cam22, float* buf) {
    Camera cam = cam22 ? CameraFromArray(cam22) : DefaultCamera(w, h);
    long long rays = 0;
    RenderRowsP(cam, w, h, x0, xc, y0, yc, frame0, frames, depth, buf, rays, 0, 1);
    return rays;
}

// Mode P on `procs` forked worker processes (the reference keeps one global RNG,
// maths.cpp:5, so threads cannot share it; processes each get their own copy).
// Rows are dealt cyclically. Used only as the CPU baseline / large-oracle leg.
long long ref_render_mode_p_procs(int w, int h, int x0, int xc, int y0, int yc, int frame0,
                                  int frames, int depth, const float* cam22, float* buf, int procs) {
    if (procs <= 1) return ref_render_mode_p(w, h, x0, xc, y0, yc, frame0, frames, depth, cam22, buf);
    size_t bytes = (size_t)xc * yc * 4 * sizeof(float);
    size_t cbytes = (size_t)procs * sizeof(long long);
    void* shm = mmap(nullptr, bytes + cbytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (shm == MAP_FAILED) return -1;
    float* sbuf = (float*)shm;
    long long* counts = (long long*)((char*)shm + bytes);
    memcpy(sbuf, buf, bytes);
    Camera cam = cam22 ? CameraFromArray(cam22) : DefaultCamera(w, h);
    pid_t* pids = new pid_t[procs];
    int started = 0;
    for (int p = 0; p < procs; ++p) {
        pid_t pid = fork();
        if (pid == 0) {
            long long r = 0;
            RenderRowsP(cam, w, h, x0, xc, y0, yc, frame0, frames, depth, sbuf, r, p, procs);
            counts[p] = r;
            _exit(0);
        }
        if (pid < 0) break;
        pids[started++] = pid;
    }
    bool ok = started == procs;
    for (int p = 0; p < started; ++p) {
        int st = 0;
        waitpid(pids[p], &st, 0);
        if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) ok = false;
    }
    delete[] pids;
    long long rays = -1;
    if (ok) {
        rays = 0;
        for (int p = 0; p < procs; ++p) rays += counts[p];
        memcpy(buf, sbuf, bytes);
    }
    munmap(shm, bytes + cbytes);
    return rays;
}

// The reference's own multithreaded DrawTest (enkiTS, kMaxDepth 20, shared racy RNG),
// exactly as main.cpp:165 calls it. Output is non-deterministic by construction.
int ref_draw_test(float time, int frameCount, int w, int h, float* buf) {
    int rays = 0;
    DrawTest(time, frameCount, w, h, buf, rays);
    return rays;
}
void ref_initialize(void) { InitializeTest(); }
// InitializeTest (parallel.cpp:231-235) with an explicit worker count: the GPU box's host
// share is 16 cores while the reference asks sysconf for the whole machine's CPUs
// (enkiTS Threads.h:91-94). Same scheduler, same g_TS, only the thread count is given.
void ref_initialize_threads(int threads) {
    g_TS = enkiNewTaskScheduler();
    enkiInitTaskSchedulerNumThreads(g_TS, (uint32_t)threads);
}
void ref_shutdown(void) { ShutdownTest(); }

}  // extern "C"
