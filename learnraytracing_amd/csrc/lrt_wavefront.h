// v4: WAVEFRONT (breadth-first) path tracing -- SURVEY §8(f) row 4's scheduling variant.
//
// The megakernels (v0, v3) keep a path's whole state in registers and let a wave run
// until its longest path ends. Here every path's state lives in HBM (SoA, one chunk of
// pixel-samples at a time) and the bounces are separate kernels over compacted queues:
//
//   wf_camera   TraceRowJob's per-sample body (parallel.cpp:270-274): jitter, GetRay
//   wf_extend   one closest hit per queued ray (HitWorld, parallel.cpp:204), together with
//               the previous scatter's deferred shadow ray (TraceDual's pass); misses end
//               their path (sky, :223-225); hits go to the Lambert / Metal / Dielectric
//               queue of their material
//   wf_shade    Scatter (parallel.cpp:78-196) over the three material queues back to back,
//               so every wave holds one material; continuing paths re-enter the ray queue
//
// wf_extend and wf_shade run maxDepth + 1 times; a path that ends folds its recursion
// stack (parallel.cpp:214, leaf outwards) and writes its colour into the chunk's frame
// planes, which merge_samples_kernel lerps in frame order (parallel.cpp:262,282). Same
// per-ray arithmetic, RNG streams, draw order and ray counts as TraceDual, so the image is
// bit-identical.
//
// Queues without global atomics: every kernel runs the same persistent grid of B blocks,
// and block j owns region j (R0 = ceil(C / B) slots) of every queue. wf_camera deals the
// chunk's pixel-samples to the regions round-robin (region j gets samples j, j + B, ...
// -- a spatially spread sample, so regions stay equally loaded as paths die); block j of
// each kernel consumes region j of its input queues and appends to region j of its output
// queues through wave ballots and LDS counters. Path state is stored by SLOT
// (j R0 + k for region j's k-th sample), so a region's state is contiguous and a wave's
// loads stay coalesced after compaction. (Same-address global atomics serialise at
// ~12 ns: one per wave and queue made the first version 10x slower.)
#pragma once

namespace lrt {

constexpr int kWfBlock = 256;

struct WfArgs {
    KernelArgs a;            // scene, camera, window, frames, maxDepth, lerp table, flags
    int lds;                 // scene staged in LDS
    int bstk_off;            // bytes into dynamic LDS: the BVH traversal stack
    int pix0, cpix;          // this chunk: window pixels [pix0, pix0 + cpix), all frames
    int C;                   // paths in the chunk = cpix * frames
    uint32_t* rng;
    float4* o;               // origin / hit position; w: depth (int bits)
    float4* d;               // direction; w: flags (int bits): 1 prevLambert, 2 pending event
    float4* sl;              // deferred shadow ray direction; w: light index (int bits), -1 none
    float4* lit;             // pending event's lit sum (xyz); w: the hit's sphere id (int bits)
    float4* stack;           // MAXD levels x C
    float4* samp;            // frames planes x cpix colours
    uint32_t* qa[2];         // ray queues (ping-pong by iteration), B regions of R0 slots
    uint32_t* qm[3];         // material queues, same regions
    unsigned int* cnt;       // per iteration it and block j: [(4 it + k) B + j], k = 0 rays, 1 + type
    int R0;                  // region size
    int Cs;                  // state slots = B * R0 (the stride of the stack levels)
    unsigned long long* rayp;   // 16 ray-count partials (stride kCtrStride)
};

// Scene staging for the wavefront kernels: [powf tables][renormalize table][spheres]
// [materials][lights][bvh traversal stack]; no recursion stack (it lives in HBM).
template <int kAcc>
__device__ __forceinline__ SceneView wf_scene(const KernelArgs& a, bool lds, int bstk_off, float4* smem, int tid) {
    double* s_pow = reinterpret_cast<double*>(smem);
    {
        const libm::PowTables g = libm::pow_tables();
        for (int i = tid; i < 16; i += kWfBlock) {
            s_pow[i] = g.invc[i];
            s_pow[16 + i] = g.logc[i];
        }
        for (int i = tid; i < 32; i += kWfBlock) reinterpret_cast<uint64_t*>(s_pow + 32)[i] = g.exp2[i];
    }
    float* s_lut = reinterpret_cast<float*>(s_pow + 64);
    renorm_lut_fill(s_lut, tid, kWfBlock);
    float4* s_sph = smem + (kPowTableBytes + kRenormBytes) / 16;
    float4* s_mat = s_sph + a.count;
    int* s_lights = reinterpret_cast<int*>(s_mat + 3 * a.count);
    if (lds) {
        for (int i = tid; i < a.count; i += kWfBlock) s_sph[i] = a.sph[i];
        for (int i = tid; i < 3 * a.count; i += kWfBlock) s_mat[i] = a.mats[i];
        for (int i = tid; i < a.nlights; i += kWfBlock) s_lights[i] = a.lights[i];
    }
    __syncthreads();
    SceneView sc;
    sc.pow.invc = s_pow;
    sc.pow.logc = s_pow + 16;
    sc.pow.exp2 = reinterpret_cast<const uint64_t*>(s_pow + 32);
    sc.rnlut = s_lut;
    sc.sph = lds ? s_sph : a.sph;
    sc.mats = lds ? s_mat : a.mats;
    sc.lights = lds ? s_lights : a.lights;
    sc.count = a.count;
    sc.nlights = a.nlights;
    sc.bv = a.bv;
    sc.bstk = reinterpret_cast<unsigned short*>(reinterpret_cast<char*>(smem) + bstk_off) + tid;
    sc.bstride = kWfBlock;
    return sc;
}

// Append `p` to this block's region of queue `q` for the lanes with `on`: one LDS
// atomic per wave on the block's counter `lcnt`.
__device__ __forceinline__ void wf_push(bool on, uint32_t p, uint32_t* q, unsigned int* lcnt) {
    const unsigned long long m = __ballot(on);
    if (m == 0) return;
    const int leader = __ffsll((long long)m) - 1;
    unsigned int base = 0;
    if ((int)__lane_id() == leader) base = atomicAdd(lcnt, (unsigned int)__popcll(m));
    base = (unsigned int)__shfl((int)base, leader, 64);
    if (on) {
        const unsigned int r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        q[base + r] = p;
    }
}

__device__ __forceinline__ void wf_rays(const WfArgs& w, unsigned long long n) {
    __shared__ unsigned long long s_n;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    n = wave_sum(n);
    if ((threadIdx.x & 63) == 0 && n) atomicAdd(&s_n, n);
    __syncthreads();
    if (threadIdx.x == 0 && s_n) atomicAdd(w.rayp + (blockIdx.x % kV0Queues) * kCtrStride, s_n);
}

// The path's colour: the recursion stack folded leaf-outwards, into its frame plane.
__device__ __forceinline__ void wf_finish(const WfArgs& w, const SceneView& sc, uint32_t p, int depth, F3 T) {
    for (int k = depth - 1; k >= 0; --k) {
        const float4 s = w.stack[(size_t)k * w.Cs + p];
        const float4 b = sc.mats[3 * __float_as_int(s.w) + 2];
        T = f3(s.x, s.y, s.z) + f3(b.x, b.y, b.z) * T;
    }
    const int frames = w.a.frames;
    const uint32_t i = (p % w.R0) * gridDim.x + p / w.R0;   // slot -> the chunk's sample index
    const uint32_t px = i / frames, fi = i % frames;
    w.samp[(size_t)fi * w.cpix + px] = make_float4(T.x, T.y, T.z, 0.0f);
}

__global__ __launch_bounds__(kWfBlock) void wf_camera(const WfArgs w) {
    const KernelArgs& a = w.a;
    extern __shared__ float4 smem[];
    float* s_lut = reinterpret_cast<float*>(smem);
    renorm_lut_fill(s_lut, threadIdx.x, kWfBlock);
    __syncthreads();
    const float invWidth = 1.0f / (float)a.width;     // parallel.cpp:260
    const float invHeight = 1.0f / (float)a.height;   // parallel.cpp:261
    // region j = blockIdx.x holds paths j, j + B, j + 2B, ...
    const int B = gridDim.x, j = blockIdx.x;
    const int nj = j < w.C ? (w.C - 1 - j) / B + 1 : 0;
    for (int k = threadIdx.x; k < nj; k += kWfBlock) {
        const int i = j + k * B;
        const int pix = w.pix0 + i / a.frames;
        const int f = a.frame0 + i % a.frames;
        const int lx = pix % a.xc, ly = pix / a.xc;
        const int x = a.x0 + lx;
        const int y = a.y0 + (ly / a.rb) * a.rb * a.rp + a.rph * a.rb + ly % a.rb;
        uint32_t rng = PixelSeed((uint32_t)x, (uint32_t)y, (uint32_t)f);
        const float u = ((float)x + RandomFloat01(rng)) * invWidth;   // :272
        const float v = ((float)y + RandomFloat01(rng)) * invHeight;  // :273
        const Ray r = GetRay(a.cam, u, v, rng, s_lut);
        const size_t slot = (size_t)j * w.R0 + k;
        w.rng[slot] = rng;
        w.o[slot] = make_float4(r.orig.x, r.orig.y, r.orig.z, __int_as_float(0));
        w.d[slot] = make_float4(r.dir.x, r.dir.y, r.dir.z, __int_as_float(0));
        w.qa[0][slot] = (uint32_t)slot;
    }
    if (threadIdx.x == 0) w.cnt[j] = (unsigned int)nj;
}

template <int kAcc, int kNS>
__global__ __launch_bounds__(kWfBlock) void wf_extend(const WfArgs w, int it) {
    extern __shared__ float4 smem[];
    const SceneView sc = wf_scene<kAcc>(w.a, w.lds != 0, w.bstk_off, smem, threadIdx.x);
    const int B = gridDim.x, j = blockIdx.x;
    const unsigned int n = w.cnt[(size_t)(4 * it) * B + j];
    const uint32_t* q = w.qa[it & 1] + (size_t)j * w.R0;
    __shared__ unsigned int s_cnt[3];
    if (threadIdx.x < 3) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    unsigned long long rays = 0;
    // whole waves iterate together (wf_push is wave-collective)
    for (unsigned int i0 = threadIdx.x & ~63u; i0 < n; i0 += kWfBlock) {
        const unsigned int i = i0 + (threadIdx.x & 63);
        const bool on = i < n;
        uint32_t p = 0;
        int type = -1;
        if (on) {
            p = q[i];
            float4 o = w.o[p], d = w.d[p];
            int depth = __float_as_int(o.w), flags = __float_as_int(d.w);
            const F3 org = f3(o.x, o.y, o.z), dir = f3(d.x, d.y, d.z);
            ++rays;
            int nid;
            float nt;
            if constexpr (kAcc) {
                nid = ClosestHitBVH(org, dir, sc.bv, nt, sc.bstk, sc.bstride);
            } else {
                const float4 s4 = (flags & 2) ? w.sl[p] : make_float4(0.0f, 0.0f, 0.0f, __int_as_float(-1));
                const bool shadow = __float_as_int(s4.w) >= 0;
                int sid;
                DualClosestHit<kNS>(org, dir, shadow, f3(s4.x, s4.y, s4.z), sc, nid, nt, sid);
                if (shadow && sid == __float_as_int(s4.w)) {   // the light is reached (:123-132)
                    const float4 l = w.lit[p];
                    float* slot = reinterpret_cast<float*>(w.stack + (size_t)depth * w.Cs + p);
                    slot[0] = l.x;
                    slot[1] = l.y;
                    slot[2] = l.z;
                }
            }
            if (flags & 2) {   // the scatter event that produced this ray is on the stack (:214)
                ++depth;
                flags &= ~2;
            }
            if (nid < 0) {   // sky (parallel.cpp:223-225)
                const float t = 0.5f * (dir.y + 1.0f);
                wf_finish(w, sc, p, depth, ((1.0f - t) * f3(1.0f, 1.0f, 1.0f) + t * f3(0.5f, 0.7f, 1.0f)) * 0.3f);
            } else {         // HitWorld's winner position (maths.cpp:74,86); the normal is the shader's
                Ray r;
                r.orig = org;
                r.dir = dir;
                const F3 pos = point_at(r, nt);
                w.o[p] = make_float4(pos.x, pos.y, pos.z, __int_as_float(depth));
                w.d[p] = make_float4(dir.x, dir.y, dir.z, __int_as_float(flags));
                w.lit[p].w = __int_as_float(nid);
                type = __float_as_int(sc.mats[3 * nid].w);
            }
        }
        for (int t = 0; t < 3; ++t) wf_push(type == t, p, w.qm[t] + (size_t)j * w.R0, &s_cnt[t]);
    }
    __syncthreads();
    if (threadIdx.x < 3) w.cnt[(size_t)(4 * it + 1 + threadIdx.x) * B + j] = s_cnt[threadIdx.x];
    wf_rays(w, rays);
}

template <int kAcc, int kNS>
__global__ __launch_bounds__(kWfBlock) void wf_shade(const WfArgs w, int it) {
    extern __shared__ float4 smem[];
    const SceneView sc = wf_scene<kAcc>(w.a, w.lds != 0, w.bstk_off, smem, threadIdx.x);
    const int B = gridDim.x, j = blockIdx.x;
    const unsigned int nL = w.cnt[(size_t)(4 * it + 1) * B + j], nM = w.cnt[(size_t)(4 * it + 2) * B + j],
                       nD = w.cnt[(size_t)(4 * it + 3) * B + j];
    const unsigned int n = nL + nM + nD;
    const size_t r0 = (size_t)j * w.R0;
    __shared__ unsigned int s_cnt;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    unsigned long long rays = 0;
    for (unsigned int i0 = threadIdx.x & ~63u; i0 < n; i0 += kWfBlock) {
        const unsigned int i = i0 + (threadIdx.x & 63);
        bool cont = false;
        uint32_t p = 0;
        if (i < n) {
            p = i < nL ? w.qm[0][r0 + i] : i < nL + nM ? w.qm[1][r0 + i - nL] : w.qm[2][r0 + i - nL - nM];
            const float4 o = w.o[p], d = w.d[p];
            const int depth = __float_as_int(o.w);
            int flags = __float_as_int(d.w);
            const int id = __float_as_int(w.lit[p].w);
            const float4 s = sc.sph[id];
            Hit rec;
            rec.pos = f3(o.x, o.y, o.z);
            rec.normal = normalize(rec.pos - f3(s.x, s.y, s.z));   // maths.cpp:75,87
            rec.t = 0.0f;
            const Material mat = load_material(sc.mats, id);
            F3 matE = mat.emissive;
            if (depth < w.a.maxDepth) {   // :212
                Ray r;
                r.orig = rec.pos;
                r.dir = f3(d.x, d.y, d.z);
                uint32_t rng = w.rng[p];
                F3 lightE;
                DeferredLight dl;
                dl.on = false;
                int nr = 0;
                const F3 X = ScatterDir<kAcc, kNS>(mat, id, r, rec, lightE, nr, rng, sc, kAcc ? nullptr : &dl);
                rays += (unsigned long long)nr;
                w.rng[p] = rng;
                const F3 dir = renormalize(normalize(X), sc.rnlut);
                if (mat.type != 1 || dot(dir, rec.normal) > 0.0f) {   // Metal absorbs (:147)
                    if (w.a.ndl && (flags & 1)) matE = f3(0.0f, 0.0f, 0.0f);
                    flags = (mat.type == 0 ? 1 : 0) | 2;
                    const F3 e = matE + lightE;   // pushed now; the lit sum replaces it if the shadow ray hits
                    w.stack[(size_t)depth * w.Cs + p] = make_float4(e.x, e.y, e.z, __int_as_float(id));
                    if (dl.on) {
                        const F3 el = matE + (lightE + dl.contrib);
                        w.lit[p] = make_float4(el.x, el.y, el.z, 0.0f);
                        w.sl[p] = make_float4(dl.l.x, dl.l.y, dl.l.z, __int_as_float(dl.li));
                    } else {
                        w.sl[p] = make_float4(0.0f, 0.0f, 0.0f, __int_as_float(-1));
                    }
                    w.d[p] = make_float4(dir.x, dir.y, dir.z, __int_as_float(flags));
                    cont = true;
                }
            }
            if (!cont) wf_finish(w, sc, p, depth, matE);
        }
        wf_push(cont, p, w.qa[(it + 1) & 1] + r0, &s_cnt);
    }
    __syncthreads();
    if (threadIdx.x == 0) w.cnt[(size_t)(4 * (it + 1)) * B + j] = s_cnt;
    wf_rays(w, rays);
}

__global__ void wf_rays_collect(unsigned long long* rayp, unsigned long long* rays) {
    const int l = threadIdx.x;
    unsigned long long v = 0;
    if (l < kV0Queues) {
        v = rayp[l * kCtrStride];
        rayp[l * kCtrStride] = 0;
    }
    v = wave_sum(v);
    if (l == 0 && v) atomicAdd(rays, v);
}

}  // namespace lrt
