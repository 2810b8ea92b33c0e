/* TEST INFRASTRUCTURE ONLY — the CPU oracle for the path tracer hot path.
 *
 * A plain-C restatement of the reference's src/cpu renderer (maths.h, maths.cpp,
 * parallel.cpp of Sefaice/LearnRayTracing), operation for operation, so that it is
 * bit-identical to the reference compiled with clang (left-to-right argument order).
 * It differs from the reference only where the reference cannot be used as an
 * oracle: the scene is a runtime array of any length (the reference's is a
 * 9-element static, parallel.cpp:15-51) and the RNG state is an explicit per-pixel
 * variable (the reference's is one global, maths.cpp:5), which makes it thread-safe.
 *
 * Transcendentals come from glibc's libm (sinf, cosf, powf, tanf) — the very
 * functions the reference calls — so this oracle is pinned to the reference
 * through the golden fixtures in tests/golden/ and, where oracle/_ref/libref.so
 * is built, live (tests/test_oracle_vs_ref.py).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 */
#ifndef LRT_ORACLE_H
#define LRT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* sphere: cx, cy, cz, radius (maths.h:156-163)
 * material: type, albedo xyz, emissive xyz, roughness, ri as 9 floats
 *           (parallel.cpp:29-37; type 0 Lambert, 1 Metal, 2 Dielectric)
 * camera: 22 floats: origin, a, u, r, lowerLeftCorner, horizontalVec, verticalVec,
 *         lensRadius (maths.h:217-224)                                           */

uint32_t orc_xorshift32(uint32_t* state);
float orc_random01(uint32_t* state);
void orc_default_camera(int w, int h, float* cam22);
void orc_make_camera(const float* from, const float* at, const float* up, float vfov,
                     float aspect, float aperture, float focus, float* cam22);
int orc_hit_sphere(const float* o, const float* d, const float* sph, float tMin, float tMax,
                   float* out7);

/* Mode P / F: render frames [frame0, frame0+frames) of the window
 * [x0, x0+xc) x [y0, y0+yc) of a w x h image into buf (xc*yc*4 floats, RGBA stride,
 * alpha untouched). depth = number of allowed scatter events (D). threads <= 0: all
 * online CPUs. cam22 == NULL: DrawTest's camera. Returns the counted rays. */
long long orc_render_p(const float* spheres, const float* mats, int count, const float* cam22,
                       int w, int h, int x0, int xc, int y0, int yc, int frame0, int frames,
                       int depth, float* buf, int threads);

/* orc_render_p plus the GL path's opt-in features (fragmentShader.fs.glsl):
 * flags & ORC_NO_DOUBLE_LIGHT: doMaterialE rule (:430,456-457) on the CPU recursion;
 * feats[6] (NULL: none; entries may be NULL): first-hit normal, world position and
 * albedo running means, and running std-devs of colour, normal and world position
 * (:444-451, :494-568), each xc*yc*4 floats like buf, updated for frames
 * f <= max_frame (GL: 4; < 0: all). */
#define ORC_NO_DOUBLE_LIGHT 64
long long orc_render_p_ex(const float* spheres, const float* mats, int count, const float* cam22,
                          int w, int h, int x0, int xc, int y0, int yc, int frame0, int frames,
                          int depth, int flags, float* buf, float* const* feats, int max_frame,
                          int threads);

/* Mode R: the reference stream (one RNG from *state, rows in order). */
long long orc_render_r(const float* spheres, const float* mats, int count, int w, int h,
                       int frame0, int frames, int depth, uint32_t* state, float* buf);

/* glibc sinf/cosf/powf in bulk (kind 0 sinf, 1 cosf, 2 powf(x,5), 3 powf(x,0.416666667f)). */
void orc_libm_eval(int kind, const float* in, float* out, long long n);

#ifdef __cplusplus
}
#endif
#endif
