/*
 * wo_dev.h -- internal C ABI between the C host library (renderer.c) and the
 * HIP backend (trace_kernels.hip).  Replaces the reference's Vulkan backend
 * surface (renderer.c:394-1810 init, 2085-2219 per-frame dispatch).
 * Not installed; public entry points are in include/wololo/.
 */
#ifndef WOLOLO_WO_DEV_H
#define WOLOLO_WO_DEV_H

#include <stddef.h>
#include <stdint.h>

#include "wololo/wo_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct WoDev WoDev;

/* Number of HIP devices (0 on error / no driver). */
int wo_dev_count(void);
/* Currently selected HIP device, or -1. */
int wo_dev_current(void);
/* Create per-renderer device state on `device` (streams, buffers). */
int wo_dev_create(int device, WoDev** out, char* err, size_t errlen);
void wo_dev_destroy(WoDev* dev);
/* Copy the compiled scene to HBM (blocking). */
int wo_dev_upload_scene(WoDev* dev, WoRec const* prog, uint32_t n_recs, uint32_t n_prims,
                        WoMaterial const* mats, uint32_t n_mats, char* err, size_t errlen);
/* Compile (hiprtc, cached per process) and load a scene-specialised path
 * tracer from `src` (scene_jit.c); NULL unloads it.  While loaded, PATHTRACE and
 * NORMALS frames launch it instead of the interpreter kernel. */
int wo_dev_set_jit(WoDev* dev, const char* src, char* err, size_t errlen);
int wo_dev_jit_active(WoDev* dev);
/* Lane traversal kernel (union-only programs, see trace_kernels.hip). */
int wo_dev_lanes_available(WoDev* dev);
void wo_dev_set_lanes(WoDev* dev, int on);
double wo_dev_jit_compile_sec(WoDev* dev);
/* Launch the frame's kernel for this rank's tiles into d_out on `stream` (async). */
int wo_dev_launch(WoDev* dev, WoFrame const* frame, void* d_out, void* stream,
                  unsigned long long* d_segments, char* err, size_t errlen);
/* Full frame into host memory (synchronous; owns a device frame buffer). */
int wo_dev_render_host(WoDev* dev, WoFrame const* frame, float* host_rgba, char* err, size_t errlen);
/* Un-interleave gathered rank buffers into a frame (async on `stream`). */
int wo_dev_assemble(void const* d_gathered, void* d_frame, uint32_t width, uint32_t height,
                    uint32_t tile_rows, uint32_t nranks, void* stream, char* err, size_t errlen);

#ifdef __cplusplus
}
#endif

#endif /* WOLOLO_WO_DEV_H */
