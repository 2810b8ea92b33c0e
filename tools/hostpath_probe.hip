// Host-path cost probe (diagnostic, not part of the product): what a drop-in DrawTest with a
// caller-owned PAGEABLE backbuffer can cost per frame without keeping any state across calls.
//   1. hipHostRegister + hipHostUnregister of the frame, per call (register flags vary)
//   2. hipMemcpy H2D / D2H straight from pageable memory (the runtime's bounce buffers)
//   3. CPU copies pageable <-> library-owned pinned memory with T threads (memcpy of RGBA, and
//      the RGB pack / unpack a staging ring would do)
//   4. DMA H2D / D2H of pinned memory
// Build: hipcc -O2 --offload-arch=gfx950 -o tools/hostpath_probe tools/hostpath_probe.hip -lpthread
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class F>
static void par(int T, size_t n, F f) {   // f(begin, end) over [0, n) split into T parts
    if (T <= 1) {
        f((size_t)0, n);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back([=] { f(n * t / T, n * (t + 1) / T); });
    for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
    const int w = 1280, h = 720, iters = argc > 1 ? atoi(argv[1]) : 20;
    const size_t npix = (size_t)w * h, bytes = npix * 16;
    float* pg = (float*)malloc(bytes);
    for (size_t i = 0; i < npix * 4; ++i) pg[i] = (float)(i % 977) * 0.25f;
    float* pin = nullptr;
    float* pin2 = nullptr;
    CK(hipHostMalloc((void**)&pin, bytes, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&pin2, bytes, hipHostMallocDefault));
    void* dev = nullptr;
    CK(hipMalloc(&dev, bytes));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    printf("frame %zu bytes, %u hw threads\n", bytes, std::thread::hardware_concurrency());

    const unsigned flags[3] = {hipHostRegisterDefault, hipHostRegisterMapped,
                               hipHostRegisterMapped | hipHostRegisterPortable};
    const char* fname[3] = {"default", "mapped", "mapped|portable"};
    for (int k = 0; k < 3; ++k) {
        double treg = 0, tun = 0, tdma = 0;
        for (int i = 0; i < iters; ++i) {
            double t0 = now();
            CK(hipHostRegister(pg, bytes, flags[k]));
            double t1 = now();
            CK(hipMemcpyAsync(dev, pg, bytes, hipMemcpyHostToDevice, s));
            CK(hipMemcpyAsync(pg, dev, bytes, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            double t2 = now();
            CK(hipHostUnregister(pg));
            double t3 = now();
            treg += t1 - t0;
            tdma += t2 - t1;
            tun += t3 - t2;
        }
        printf("register[%s]: %.3f ms  H2D+D2H registered %.3f ms  unregister %.3f ms\n", fname[k],
               1e3 * treg / iters, 1e3 * tdma / iters, 1e3 * tun / iters);
    }
    {
        double th2d = 0, td2h = 0;
        for (int i = 0; i < iters; ++i) {
            double t0 = now();
            CK(hipMemcpy(dev, pg, bytes, hipMemcpyHostToDevice));
            double t1 = now();
            CK(hipMemcpy(pg, dev, bytes, hipMemcpyDeviceToHost));
            double t2 = now();
            th2d += t1 - t0;
            td2h += t2 - t1;
        }
        printf("pageable hipMemcpy: H2D %.3f ms  D2H %.3f ms\n", 1e3 * th2d / iters, 1e3 * td2h / iters);
    }
    {
        double th2d = 0, td2h = 0;
        for (int i = 0; i < iters; ++i) {
            double t0 = now();
            CK(hipMemcpyAsync(dev, pin, bytes, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
            double t1 = now();
            CK(hipMemcpyAsync(pin, dev, bytes, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            double t2 = now();
            th2d += t1 - t0;
            td2h += t2 - t1;
        }
        printf("pinned DMA: H2D %.3f ms  D2H %.3f ms\n", 1e3 * th2d / iters, 1e3 * td2h / iters);
    }
    for (int T : {1, 2, 4, 8, 12, 16}) {
        double tcp = 0, tpack = 0, tunp = 0;
        for (int i = 0; i < iters; ++i) {
            double t0 = now();
            par(T, npix, [&](size_t b, size_t e) { memcpy(pin + 4 * b, pg + 4 * b, (e - b) * 16); });
            double t1 = now();
            par(T, npix, [&](size_t b, size_t e) {   // RGB of each pixel, packed
                const float* src = pg + 4 * b;
                float* dst = pin2 + 3 * b;
                for (size_t p = b; p < e; ++p, src += 4, dst += 3) {
                    dst[0] = src[0];
                    dst[1] = src[1];
                    dst[2] = src[2];
                }
            });
            double t2 = now();
            par(T, npix, [&](size_t b, size_t e) {   // back into RGBA, alpha untouched
                const float* src = pin2 + 3 * b;
                float* dst = pg + 4 * b;
                for (size_t p = b; p < e; ++p, src += 3, dst += 4) {
                    dst[0] = src[0];
                    dst[1] = src[1];
                    dst[2] = src[2];
                }
            });
            double t3 = now();
            tcp += t1 - t0;
            tpack += t2 - t1;
            tunp += t3 - t2;
        }
        printf("threads %2d: memcpy RGBA %.3f ms  pack RGB %.3f ms  unpack RGB %.3f ms\n", T, 1e3 * tcp / iters,
               1e3 * tpack / iters, 1e3 * tunp / iters);
    }
    CK(hipFree(dev));
    CK(hipHostFree(pin));
    CK(hipHostFree(pin2));
    free(pg);
    return 0;
}
