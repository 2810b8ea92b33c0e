// parallel_lrt.cpp — the reference's src/cpu/parallel.h (parallel.h:6-8) implemented by
// liblrt_hip.so. This is the binding a maintainer adds to the reference: build it in place
// of parallel.cpp, keep parallel.h and main.cpp, link -llrt_hip. It is compiled here
// against the reference's own parallel.h (integration/Makefile; tests/test_integration.py).
#include "parallel.h"
#include "lrt.h"

#include <cstdio>
#include <cstdlib>

static void Check(int rc, const char* what) {
    if (rc != LRT_OK) {
        std::fprintf(stderr, "%s: %s\n", what, lrt_last_error());
        std::abort();
    }
}

// parallel.cpp:231-235 (the enkiTS scheduler becomes the HIP device + stream)
void InitializeTest() { Check(lrt_initialize(), "lrt_initialize"); }

// parallel.cpp:237-240
void ShutdownTest() { Check(lrt_shutdown(), "lrt_shutdown"); }

// parallel.cpp:297-323: one progressive frame into the caller's RGBA float backbuffer
void DrawTest(float time, int frameCount, int screenWidth, int screenHeight, float* backbuffer, int& outRayCount) {
    Check(lrt_draw_test(time, frameCount, screenWidth, screenHeight, backbuffer, &outRayCount), "lrt_draw_test");
}
