/* TEST INFRASTRUCTURE ONLY (SURVEY §5 "race detection": TSan on the CPU restatement).
 *
 * The reference's worker threads share one RNG state (`s_RndState`, maths.cpp:5,9-13),
 * a real data race; the restatement replaces it with per-pixel seeds and a shared row
 * cursor (lrt_oracle.c worker()). This driver is compiled together with lrt_oracle.c under
 * -fsanitize=thread (`make -C oracle tsan`) and renders one window with many threads and
 * with one: ThreadSanitizer reports any race on the job or the buffer, and the two images
 * and ray counts must be the same bits (the row order the threads take must not matter).
 *
 *   tsan_check SCENE.bin W H FRAMES DEPTH THREADS
 * SCENE.bin: int32 count, then count x 4 float32 spheres, then count x 9 float32 materials
 * (the layout of learnraytracing_amd.scene.scene_arrays). Exit 0 and "identical" on success.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lrt_oracle.h"

int main(int argc, char** argv) {
    if (argc != 7) {
        fprintf(stderr, "usage: %s SCENE.bin W H FRAMES DEPTH THREADS\n", argv[0]);
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 2; }
    int count = 0;
    if (fread(&count, sizeof(int), 1, f) != 1 || count < 0 || count > 4096) { fprintf(stderr, "bad scene\n"); return 2; }
    float* sph = (float*)malloc(sizeof(float) * 4 * (size_t)(count ? count : 1));
    float* mat = (float*)malloc(sizeof(float) * 9 * (size_t)(count ? count : 1));
    if (fread(sph, sizeof(float) * 4, (size_t)count, f) != (size_t)count ||
        fread(mat, sizeof(float) * 9, (size_t)count, f) != (size_t)count) { fprintf(stderr, "short scene\n"); return 2; }
    fclose(f);
    const int w = atoi(argv[2]), h = atoi(argv[3]), frames = atoi(argv[4]), depth = atoi(argv[5]);
    const int threads = atoi(argv[6]);
    if (w <= 0 || h <= 0 || frames <= 0 || threads <= 0) { fprintf(stderr, "bad size\n"); return 2; }
    const size_t n = (size_t)w * h * 4;
    float* a = (float*)calloc(n, sizeof(float));
    float* b = (float*)calloc(n, sizeof(float));
    const long long ra = orc_render_p(sph, mat, count, NULL, w, h, 0, w, 0, h, 0, frames, depth, a, threads);
    const long long rb = orc_render_p(sph, mat, count, NULL, w, h, 0, w, 0, h, 0, frames, depth, b, 1);
    const int same = ra == rb && memcmp(a, b, n * sizeof(float)) == 0;
    printf("%s rays %lld %lld\n", same ? "identical" : "DIFFERENT", ra, rb);
    free(a); free(b); free(sph); free(mat);
    return same ? 0 : 1;
}
