/* lrt_demo — plain-C host for liblrt_hip.so: the headless stand-in for the reference's
 * Win32 app (src/cpu/main.cpp). It calls the reference API exactly as main.cpp does
 * (InitializeTest :48, DrawTest per frame :165, ShutdownTest :74), prints the same
 * statistics line as the on-screen overlay (main.cpp:180-190), and, instead of the GDI
 * blit (main.cpp:117-141, removed), optionally writes the last frame as a PPM after
 * the same LinearToSRGB conversion.
 *
 *   lrt_demo [width height frames [out.ppm|out.pfm]]      defaults: 1280 720 16
 * (.pfm: the linear float RGB backbuffer; otherwise sRGB 8-bit PPM)
 */
#define _POSIX_C_SOURCE 199309L
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "lrt.h"

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* main.cpp:109-115 */
static uint32_t linear_to_srgb(float x) {
    x = x < 0.0f ? 0.0f : x;
    x = 1.055f * powf(x, 0.416666667f) - 0.055f;
    x = x < 0.0f ? 0.0f : x;
    uint32_t u = (uint32_t)(x * 255.9f);
    return u < 255u ? u : 255u;
}

int main(int argc, char** argv) {
    int w = argc > 2 ? atoi(argv[1]) : 1280;
    int h = argc > 2 ? atoi(argv[2]) : 720;
    int frames = argc > 3 ? atoi(argv[3]) : 16;
    const char* ppm = argc > 4 ? argv[4] : NULL;
    if (w < 1 || h < 1 || frames < 1) {
        fprintf(stderr, "usage: %s [width height frames [out.ppm|out.pfm]]\n", argv[0]);
        return 2;
    }
    if (lrt_initialize() != LRT_OK) {
        fprintf(stderr, "lrt_initialize: %s\n", lrt_last_error());
        return 1;
    }
    /* main.cpp:40-41, page-locked so that lrt_draw_test renders it in place */
    const size_t bytes = (size_t)w * h * 4 * sizeof(float);
    float* backbuffer = NULL;
    if (lrt_host_alloc(bytes, (void**)&backbuffer) != LRT_OK) {
        fprintf(stderr, "lrt_host_alloc: %s\n", lrt_last_error());
        return 1;
    }
    memset(backbuffer, 0, bytes);
    double total_s = 0.0;
    long long total_rays = 0;
    for (int f = 0; f < frames; ++f) {
        int rays = 0;
        double t0 = now_s();
        if (lrt_draw_test((float)t0, f, w, h, backbuffer, &rays) != LRT_OK) {
            fprintf(stderr, "lrt_draw_test: %s\n", lrt_last_error());
            return 1;
        }
        total_s += now_s() - t0;
        total_rays += rays;
    }
    double s = total_s / frames;
    /* main.cpp:188-189 */
    printf("%.2fms (%.1f FPS) %.1fMrays/s %.2fMrays/frame frames %i rays %lld\n", s * 1000.0, 1.0 / s,
           (double)total_rays / frames / s * 1.0e-6, (double)total_rays / frames * 1.0e-6, frames, total_rays);
    const size_t plen = ppm ? strlen(ppm) : 0;
    if (ppm && plen > 4 && strcmp(ppm + plen - 4, ".pfm") == 0) {
        /* linear float RGB; PFM stores rows bottom-to-top, the backbuffer's order */
        FILE* fp = fopen(ppm, "wb");
        if (!fp) return 1;
        fprintf(fp, "PF\n%d %d\n-1.0\n", w, h);   /* negative scale: little-endian */
        for (size_t i = 0; i < (size_t)w * h; ++i) fwrite(backbuffer + 4 * i, sizeof(float), 3, fp);
        fclose(fp);
    } else if (ppm) {
        FILE* fp = fopen(ppm, "wb");
        if (!fp) return 1;
        fprintf(fp, "P6\n%d %d\n255\n", w, h);
        for (int y = h - 1; y >= 0; --y) /* row 0 is the bottom (main.cpp:33 bottom-up DIB) */
            for (int x = 0; x < w; ++x) {
                const float* p = backbuffer + ((size_t)y * w + x) * 4;
                unsigned char rgb[3] = {(unsigned char)linear_to_srgb(p[0]), (unsigned char)linear_to_srgb(p[1]),
                                        (unsigned char)linear_to_srgb(p[2])};
                fwrite(rgb, 1, 3, fp);
            }
        fclose(fp);
    }
    lrt_host_free(backbuffer);
    lrt_shutdown();
    return 0;
}
