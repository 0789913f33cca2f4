/*
 * oracle.h -- CPU oracle for the wololo hot path.  TEST INFRASTRUCTURE ONLY:
 * linked by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
 * never by the product library (csgrenderer_amd/lib/libwololo.so).
 *
 * Two restatements:
 *   oracle_ubershader_*  -- the reference fragment shader
 *                           src/wololo/renderer/ubershader1.frag:19-163 in IEEE
 *                           fp32, op order of its SPIR-V;
 *                           pinned by the survey's KATs (tests/golden/).
 *   oracle_pathtrace_*   -- the CSG path tracer's semantics (wo_scene.h program,
 *                           RTIOW materials).  The reference has no such code:
 *                           parity against the reference is UNPINNED here; the
 *                           oracle pins the HIP kernels to this definition.
 */
#ifndef WOLOLO_ORACLE_H
#define WOLOLO_ORACLE_H

#include <stdint.h>

#include "wololo/wo_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One pixel of ubershader1.frag.  mode: WO_MODE_UBERSHADER_RT1 or WO_MODE_DEBUG_ST. */
void oracle_ubershader_pixel(float out[4], uint32_t x, uint32_t y, uint32_t width, uint32_t height,
                             float time_sec, uint32_t mode);
/* Whole frame, row 0 = top, RGBA float. */
void oracle_ubershader_frame(float* out, uint32_t width, uint32_t height, float time_sec, uint32_t mode,
                             int nthreads);

/* Path-trace (or NORMALS-shade) a list of pixels of the full frame described by
 * `fr` (tile fields ignored).  out: npix*4 floats.  *segments (optional) gets the
 * number of traced segments.  Returns 0 on success. */
int oracle_pathtrace_pixels(WoRec const* prog, uint32_t n_recs, WoMaterial const* mats, uint32_t n_mats,
                            WoFrame const* fr, uint32_t const* xs, uint32_t const* ys, uint32_t npix, float* out,
                            uint64_t* segments, int nthreads);
/* Rows [row0, row0+nrows) of the frame; out: nrows*width*4 floats. */
int oracle_pathtrace_rows(WoRec const* prog, uint32_t n_recs, WoMaterial const* mats, uint32_t n_mats,
                          WoFrame const* fr, uint32_t row0, uint32_t nrows, float* out, uint64_t* segments,
                          int nthreads);

/* Single nearest-hit query (for unit tests): returns 1 on hit. */
int oracle_trace(WoRec const* prog, uint32_t n_recs, float const o[3], float const d[3], float* t, uint32_t* prim,
                 uint32_t* type, uint32_t* member, uint32_t* root_after);

/* sin/cos of 2*pi*u as the kernels compute it (polynomial, no libm). */
void oracle_sincos_turn(float u, float* s, float* c);

/* RNG known answers. */
uint32_t oracle_pcg_hash(uint32_t v);
uint32_t oracle_rng_next(uint32_t* state);

#ifdef __cplusplus
}
#endif

#endif /* WOLOLO_ORACLE_H */
