/* liblrt_hip diagnostics: checks of the renderer's parts (the libm restatement, the closest-hit
 * structures, Scatter) that the tests and tools call. Not part of the renderer API (lrt.h);
 * nothing on a render path uses them. Exported by the same library. */
#ifndef LRT_DIAG_H
#define LRT_DIAG_H
#include "lrt.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- diagnostics (libm restatement, lrt_libm.h) --------------------------- */
/* kind 0: sinf, 1: cosf, 2: powf(x, 5), 3: powf(x, 0.416666667f) (LinearToSRGB),
 * 4: sqrtf, 5: 1.0f / x (the device evaluates the path's short correctly rounded sequences),
 * 6 / 7: the sine / cosine results of the path's sincosf (one shared reduction).
 * Host evaluation of the restatement. */
int lrt_libm_eval_host(int kind, const float* in, float* out, long long n);
/* Device evaluation of the same restatement (device pointers, blocking). */
int lrt_libm_eval_device(int kind, const float* d_in, float* d_out, long long n);

/* BVH diagnostics (host only, no GPU): build the BVH of the given scene and trace n rays
 * (6 floats each: origin, direction) with the device traversal code. out[7]: mean nodes
 * visited, mean spheres tested, max nodes, max spheres, mismatches per ray against the
 * linear scan (0 by construction: closest hit (id and t), the bounded shadow-ray traversal
 * for the scan's winner and for one other sphere per ray, the two-query loop), the deepest
 * traversal-stack entry any of those traversals wrote, and the entries the device's LDS
 * stack holds for this scene (the first must not exceed the second). */
int lrt_bvh_stats(const lrt_sphere* spheres, int count, const float* rays, int n, double* out);
/* Diagnostic (host only, no GPU): the uniform grid (lrt_grid.h) of the given scene, built as
 * lrt_set_scene would, traced for n rays (o.xyz, d.xyz; d normalised as the Ray ctor does) by
 * the device's walk compiled for the host. out[0..9]: mean cells visited, mean spheres tested,
 * max (cells + spheres) of one ray, fraction of rays whose closest (id, t), bounded shadow answer
 * or two-query result differs from the linear scan (must be 0), fraction of rays that took the
 * fallback scan, cells per axis (3), spheres tested first by every ray, and 1 when the library
 * would pick the grid for this scene (LRT_ACCEL=auto). */
int lrt_grid_stats(const lrt_sphere* spheres, int count, const float* rays, int n, double* out);
/* Closest hit of n rays (6 floats each; d normalised as the Ray ctor does) through one
 * accelerated structure of the given scene, built as lrt_set_scene builds it: ids[i] (-1:
 * miss) and ts[i]. accel 1: the BVH, 2: the uniform grid. mode 0: host build of the device
 * traversal; 1: the same on the current device (one thread per ray); 2 (BVH only): the
 * device's packet (wave-coherent) traversal over each wave's 64 rays. Host pointers; blocking. */
int lrt_accel_eval(const lrt_sphere* spheres, int count, const float* rays, int n, int accel, int mode, int* ids,
                   float* ts);

/* Scatter probe (no render): the device Scatter in the reference's shape (lrt_trace.h;
 * parallel.cpp:78-196 `bool Scatter(mat, r_in, rec, attenuation, scattered, outLightE,
 * inoutRayCount)`, RNG state explicit) over the given scene, n cases. Case i: material
 * ids[i] scatters the ray rays[6i..6i+5] (origin, direction; normalised as the Ray ctor
 * does) at the hit recs[7i..7i+6] (pos, normal, t) from RNG state seeds[i]. Outputs:
 * out[12i..] = attenuation, scattered origin, scattered direction, outLightE; ret[i] =
 * Scatter's result (0: absorbed); counted[i] = shadow rays counted; state[i] = the RNG
 * state after. Scenes above 16 spheres trace shadow rays through the BVH. on_device = 0
 * runs the host build of the same code, 1 one thread per case on the current device, 2
 * the same with the packet (wave-coherent) shadow traversal. Host pointers; blocking. */
int lrt_scatter_eval(const lrt_sphere* spheres, const lrt_material* materials, int count,
                     const int* ids, const float* rays, const float* recs, const uint32_t* seeds,
                     int n, float* out, int* ret, int* counted, uint32_t* state, int on_device);

/* ---- kernel timing (bench.py's launch-alone leg) ------------------------------- */
/* on != 0: every later render kernel launch (the pool kernel and v0), on whichever device it
 * runs, is bracketed by two HIP events of that device recorded on its own stream, right before
 * and after the kernel -- no other stream command in between; on = 0 stops and discards them. lrt_kernel_times waits
 * for the recorded launches and writes up to max_n durations (ms) in launch order to ms, their
 * number to *n, then forgets them. */
int lrt_kernel_timing(int on);
int lrt_kernel_times(float* ms, int max_n, int* n);

#ifdef __cplusplus
}
#endif
#endif /* LRT_DIAG_H */
