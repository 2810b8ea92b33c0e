// parallel_lrt.cpp — the reference's src/cpu/parallel.h (parallel.h:6-8) implemented by
// liblrt_hip.so. This is the binding a maintainer adds to the reference: build it in place
// of parallel.cpp, keep parallel.h and main.cpp, link -llrt_hip. It is compiled here
// against the reference's own parallel.h (integration/Makefile; tests/test_integration.py).
#include "parallel.h"
#include "lrt.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>

static void Check(int rc, const char* what) {
    if (rc != LRT_OK) {
        std::fprintf(stderr, "%s: %s\n", what, lrt_last_error());
        std::abort();
    }
}

// parallel.cpp:231-235 (the enkiTS scheduler becomes the HIP device + stream). The reference
// spreads DrawTest's rows over every core (parallel.cpp:317-320); LRT_DEVICES spreads them over
// GPUs: "all" (every visible device) or a list "0,1,2,3" (lrt_initialize_devices: row blocks
// dealt round-robin, RCCL gather into the first). Unset: the calling thread's device.
void InitializeTest() {
    const char* e = std::getenv("LRT_DEVICES");
    if (!e || !*e) {
        Check(lrt_initialize(), "lrt_initialize");
        return;
    }
    if (std::strcmp(e, "all") == 0) {
        Check(lrt_initialize_devices(0, nullptr, 0), "lrt_initialize_devices");
        return;
    }
    int ids[16], n = 0;
    for (const char* p = e; *p && n < 16;) {
        char* end = nullptr;
        ids[n++] = (int)std::strtol(p, &end, 10);
        if (end == p) break;
        p = (*end == ',') ? end + 1 : end;
    }
    Check(lrt_initialize_devices(n, ids, 0), "lrt_initialize_devices");
}

// parallel.cpp:237-240
void ShutdownTest() { Check(lrt_shutdown(), "lrt_shutdown"); }

// parallel.cpp:297-323: one progressive frame into the caller's RGBA float backbuffer
void DrawTest(float time, int frameCount, int screenWidth, int screenHeight, float* backbuffer, int& outRayCount) {
    Check(lrt_draw_test(time, frameCount, screenWidth, screenHeight, backbuffer, &outRayCount), "lrt_draw_test");
}
