// drawtest_host.cpp — a headless main.cpp (src/cpu/main.cpp:40-77,165,188-189) that only
// sees the reference's API, parallel.h: InitializeTest, DrawTest once per frame with
// frameCount = 0, 1, ..., ShutdownTest. Linked with parallel_lrt.cpp it runs the
// reference's call sequence on liblrt_hip.so (tests/test_integration.py compares the
// PFM it writes with the oracle).
//
//   drawtest_ref_api width height frames out.pfm
#include "parallel.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

int main(int argc, char** argv) {
    if (argc != 5) {
        std::fprintf(stderr, "usage: %s width height frames out.pfm\n", argv[0]);
        return 2;
    }
    const int w = std::atoi(argv[1]), h = std::atoi(argv[2]), frames = std::atoi(argv[3]);
    if (w < 1 || h < 1 || frames < 1) return 2;
    // main.cpp:40-41: the caller owns a zeroed RGBA float backbuffer
    float* backbuffer = new float[(size_t)w * h * 4];
    std::memset(backbuffer, 0, sizeof(float) * (size_t)w * h * 4);
    InitializeTest();                                                  // main.cpp:48
    long long rays = 0, steady_rays = 0;
    double secs = 0.0, steady = 0.0;
    for (int f = 0; f < frames; ++f) {                                 // main.cpp:165
        int r = 0;
        const auto t0 = std::chrono::steady_clock::now();
        DrawTest(0.0f, f, w, h, backbuffer, r);
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        secs += dt;
        rays += r;
        if (f >= 2) {   // main.cpp:180 averages over more than 10 frames; the first two set up
            steady += dt;
            steady_rays += r;
        }
    }
    ShutdownTest();                                                    // main.cpp:74
    const double s = secs / frames;                                    // main.cpp:188-189
    std::printf("%.2fms (%.1f FPS) %.1fMrays/s %.2fMrays/frame frames %i rays %lld\n", s * 1000.0, 1.0 / s,
                (double)rays / frames / s * 1.0e-6, (double)rays / frames * 1.0e-6, frames, rays);
    if (frames > 2) {
        const double ss = steady / (frames - 2);
        std::printf("steady %.3fms (%.1f FPS) %.1fMrays/s over frames 2..%i\n", ss * 1000.0, 1.0 / ss,
                    (double)steady_rays / steady * 1.0e-6, frames - 1);
    }
    FILE* fp = std::fopen(argv[4], "wb");
    if (!fp) return 1;
    std::fprintf(fp, "PF\n%d %d\n-1.0\n", w, h);   // linear RGB, bottom row first (the backbuffer's order)
    for (size_t i = 0; i < (size_t)w * h; ++i) std::fwrite(backbuffer + 4 * i, sizeof(float), 3, fp);
    std::fclose(fp);
    delete[] backbuffer;
    return 0;
}
