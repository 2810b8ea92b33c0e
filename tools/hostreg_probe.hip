// Per-call registration probe (diagnostic, not part of the product). A drop-in DrawTest may
// page-lock the caller's pageable buffer for the duration of ONE call (hipHostRegister at the
// start, hipHostUnregister before returning), keeping no state the caller could invalidate.
// This checks that it is both cheap and correct when the caller frees its buffer and gets the
// same virtual address back (munmap + mmap MAP_FIXED) between calls:
//   fresh   a new mapping per call: register, DMA in + out, unregister, munmap (timed)
//   same    one address, remapped between calls: the data the device reads must be the NEW
//           pages' contents and the data written back must land in them
//   zc      the registered range's device address written by a kernel (the PCIe-write lerp)
// Build: hipcc -O2 --offload-arch=gfx950 -o tools/hostreg_probe tools/hostreg_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <chrono>

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

__global__ void add_kernel(const float* __restrict__ src, float* dst, size_t n, float v) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i] + v;
}

static void fill(float* p, size_t n, float base) {
    for (size_t i = 0; i < n; ++i) p[i] = base + (float)(i % 1021);
}
static size_t check(const float* p, size_t n, float base) {
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) bad += p[i] != base + (float)(i % 1021);
    return bad;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20;
    const size_t n = (size_t)1280 * 720 * 4, bytes = n * 4;
    float* dev = nullptr;
    float* pin = nullptr;
    CK(hipMalloc((void**)&dev, bytes));
    CK(hipHostMalloc((void**)&pin, bytes, hipHostMallocDefault));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const unsigned flags = hipHostRegisterMapped | hipHostRegisterPortable;
    size_t bad = 0;
    {   // warm the DMA engines
        CK(hipMemcpyAsync(dev, pin, bytes, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
    }
    double treg = 0, tdma = 0, tun = 0;
    for (int i = 0; i < iters; ++i) {   // fresh: a new mapping every call
        float* p = (float*)mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        fill(p, n, (float)(i * 7));
        const double t0 = now();
        CK(hipHostRegister(p, bytes, flags));
        const double t1 = now();
        CK(hipMemcpyAsync(dev, p, bytes, hipMemcpyHostToDevice, s));
        add_kernel<<<1024, 256, 0, s>>>(dev, dev, n, 1.0f);
        CK(hipMemcpyAsync(p, dev, bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        const double t2 = now();
        CK(hipHostUnregister(p));
        const double t3 = now();
        bad += check(p, n, (float)(i * 7) + 1.0f);
        munmap(p, bytes);
        treg += t1 - t0;
        tdma += t2 - t1;
        tun += t3 - t2;
    }
    printf("fresh: register %.4f ms  DMA in+add+out %.4f ms  unregister %.4f ms  bad %zu\n", 1e3 * treg / iters,
           1e3 * tdma / iters, 1e3 * tun / iters, bad);
    // same address, remapped between calls
    float* a = (float*)mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    bad = 0;
    size_t moved = 0;
    treg = tdma = tun = 0;
    for (int i = 0; i < iters; ++i) {
        fill(a, n, (float)(1000 + i * 5));
        const double t0 = now();
        CK(hipHostRegister(a, bytes, flags));
        const double t1 = now();
        float* ad = nullptr;
        CK(hipHostGetDevicePointer((void**)&ad, a, 0));
        CK(hipMemcpyAsync(dev, a, bytes, hipMemcpyHostToDevice, s));
        // zero copy: the kernel writes the caller's pixels over PCIe through the device address
        add_kernel<<<1024, 256, 0, s>>>(dev, ad, n, 2.0f);
        CK(hipStreamSynchronize(s));
        const double t2 = now();
        CK(hipHostUnregister(a));
        const double t3 = now();
        bad += check(a, n, (float)(1000 + i * 5) + 2.0f);
        // the caller frees its buffer and maps a new one at the same address
        munmap(a, bytes);
        float* b = (float*)mmap(a, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED, -1, 0);
        moved += b != a;
        a = b;
        treg += t1 - t0;
        tdma += t2 - t1;
        tun += t3 - t2;
    }
    printf("same-address remap: register %.4f ms  DMA in+zero-copy out %.4f ms  unregister %.4f ms  bad %zu moved %zu\n",
           1e3 * treg / iters, 1e3 * tdma / iters, 1e3 * tun / iters, bad, moved);
    // malloc'd (glibc mmap chunk, not page aligned), freed and reallocated each call
    bad = 0;
    size_t same = 0;
    void* last = nullptr;
    treg = 0;
    for (int i = 0; i < iters; ++i) {
        float* p = (float*)malloc(bytes);
        same += p == last;
        last = p;
        fill(p, n, (float)(3 * i));
        const double t0 = now();
        CK(hipHostRegister(p, bytes, flags));
        treg += now() - t0;
        CK(hipMemcpyAsync(dev, p, bytes, hipMemcpyHostToDevice, s));
        add_kernel<<<1024, 256, 0, s>>>(dev, dev, n, 3.0f);
        CK(hipMemcpyAsync(p, dev, bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        CK(hipHostUnregister(p));
        bad += check(p, n, (float)(3 * i) + 3.0f);
        free(p);
    }
    printf("malloc/free per call: register %.4f ms  bad %zu  same address %zu of %d\n", 1e3 * treg / iters, bad, same,
           iters);
    CK(hipFree(dev));
    CK(hipHostFree(pin));
    return bad != 0;
}
