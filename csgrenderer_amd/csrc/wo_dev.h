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

/* Frame slots of a device: the draw_frame pipeline's two (frame k renders while
 * k-1 is presented), the synchronous render's scratch slot (never presented, so
 * wo_renderer_last_frame keeps pointing at the last presented frame), and the
 * two slots device frames alternate over (wo_renderer_render_frame_device). */
enum { WO_SLOT_PIPE0 = 0, WO_SLOT_PIPE1 = 1, WO_SLOT_SYNC = 2, WO_SLOT_DEV0 = 3, WO_SLOT_DEV1 = 4, WO_SLOTS = 5 };

/* How a non-root rank's share reaches the root (wo_dev_enable_peer):
 *   SAME    same HIP device: a device-to-device copy;
 *   DMA     peer access enabled: hipMemcpyPeerAsync over xGMI;
 *   STAGED  no peer path (hipDeviceCanAccessPeer = 0, or WOLOLO_PEER=staged):
 *           the share goes through a pinned host buffer, D2H on the rank's
 *           stream, H2D on the root's. */
enum { WO_PEER_SAME = 0, WO_PEER_DMA = 1, WO_PEER_STAGED = 2 };

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
/* 1 when the code object of `src` for the device's target is in this process's
 * cache or the disk cache (then loading it takes milliseconds), else 0. */
int wo_dev_jit_cached(WoDev* dev, const char* src);
/* A compile of `src` for dev's target on a background host thread, into the
 * process cache (and the disk cache): wo_dev_set_jit then loads it at once.
 * done: 1 once the compile has ended; finish joins the thread and frees the job
 * (0, or -1 with the compiler's message). */
typedef struct WoJitJob WoJitJob;
WoJitJob* wo_jit_job_start(WoDev* dev, const char* src);
int wo_jit_job_done(WoJitJob* job);
const char* wo_jit_job_source(WoJitJob* job);
int wo_jit_job_finish(WoJitJob* job, char* err, size_t errlen);
/* Lane traversal kernel (union-only programs, see trace_kernels.hip). */
int wo_dev_lanes_available(WoDev* dev);
void wo_dev_set_lanes(WoDev* dev, int on);
double wo_dev_jit_compile_sec(WoDev* dev);
/* Launch the frame's kernel for this rank's tiles into d_out on `stream` (async). */
int wo_dev_launch(WoDev* dev, WoFrame const* frame, void* d_out, void* stream,
                  unsigned long long* d_segments, char* err, size_t errlen);
/* wo_dev_launch with progressive accumulation (PATHTRACE frames): d_accum holds
 * 3 int64 fixed-point sums per pixel of the earlier samples (zeroed to start);
 * the launch adds this frame's samples and writes the mean over accum_spp (the
 * samples in d_accum afterwards).  NULL d_accum = wo_dev_launch. */
int wo_dev_launch_ex(WoDev* dev, WoFrame const* frame, void* d_out, void* stream,
                     unsigned long long* d_segments, long long* d_accum, uint32_t accum_spp, char* err,
                     size_t errlen);
/* Progressive accumulation buffer for one rank's share of a width x height
 * frame (row-cyclic tiles of tile_rows rows over nranks; 3 int64 per pixel),
 * zeroed (async, on the device stream) when `reset` or reallocated. */
int wo_dev_accum_prepare(WoDev* dev, uint32_t width, uint32_t height, uint32_t tile_rows, uint32_t nranks, int reset,
                         long long** d_accum, char* err, size_t errlen);
/* The draw_frame pipeline: render a whole frame into frame slot 0 or 1 (with
 * accumulation when d_accum) on the device stream; then, on the device's copy
 * stream once the render is done, encode it for present (sRGB, B8G8R8A8), copy
 * the encode (and the float frame when `map_float`) to the slot's pinned host
 * buffers and record the slot's event.  Asynchronous; the next frame's render
 * does not wait for the map-back. */
int wo_dev_frame_submit(WoDev* dev, WoFrame const* frame, int slot, long long* d_accum, uint32_t accum_spp,
                        int map_float, char* err, size_t errlen);
/* wo_dev_frame_submit over n ranks, devs[0] presenting: rank i renders its
 * row-cyclic 4-row tiles on devs[i] (d_accum[i]: its accumulation, or d_accum
 * NULL), ranks 1..n-1 copy their shares to devs[0] (peer DMA when the devices
 * differ), devs[0] assembles the frame into the slot.  Asynchronous; wait with
 * wo_dev_frame_wait(devs[0], slot, ...). */
int wo_dev_frame_submit_ranks(WoDev* const* devs, uint32_t n, WoFrame const* frame, int slot,
                              long long* const* d_accum, uint32_t accum_spp, int map_float, char* err,
                              size_t errlen);
/* A frame over n ranks rendered and assembled into the caller's device frame
 * d_frame (width x height float4, on devs[0]'s device), ordered on `stream`
 * (a stream of devs[0]'s device): the ranks render on their own streams once
 * the slot's previous assembly is done, and the assembly is queued on
 * `stream`.  `slot` is WO_SLOT_DEV0 or _DEV1 (consecutive frames
 * alternate, so frame k+1 renders while frame k is gathered).  Each rank adds
 * its traced segments to its own counter (wo_dev_take_segments). */
int wo_dev_frame_ranks_device(WoDev* const* devs, uint32_t n, WoFrame const* frame, int slot, void* d_frame,
                              void* stream, char* err, size_t errlen);
/* Segments traced by this rank's device frames since the last call (waits for
 * the device; the counter restarts at 0). */
int wo_dev_take_segments(WoDev* dev, unsigned long long* total, char* err, size_t errlen);
/* Set how `from`'s share reaches `to` (WO_PEER_*): peer access is enabled when
 * the devices differ and the pair has a peer path.  WOLOLO_PEER=staged forces
 * the host-staged path (also between ranks stacked on one device). */
int wo_dev_enable_peer(WoDev* from, WoDev* to, char* err, size_t errlen);
int wo_dev_peer_mode(WoDev* dev);
/* HIP device of a WoDev. */
int wo_dev_device(WoDev* dev);
/* Select a HIP device for the calling thread (restoring the caller's). */
int wo_dev_select(int device);
/* jit_cache.c: SHA-256 and the on-disk code-object cache of the specialised
 * kernels (keyed by the hex digest of everything that determines the object). */
typedef struct WoSha256 {
    uint32_t h[8];
    uint64_t len;
    uint8_t buf[64];
    uint32_t fill;
} WoSha256;
void wo_sha256_init(WoSha256* s);
void wo_sha256_update(WoSha256* s, const void* data, size_t n);
void wo_sha256_final(WoSha256* s, uint8_t out[32]);
void wo_sha256_hex(const uint8_t digest[32], char out[65]);
int wo_jit_cache_dir(char* out, size_t len);
/* 0 and a malloc'd copy of the object on a valid entry, else -1 */
int wo_jit_disk_load(const char* key_hex, void** code, size_t* size);
int wo_jit_disk_store(const char* key_hex, const void* code, size_t size);
/* wo_jit_code_object: renderer_ext.h */
/* Origin (as above; -1: no specialised kernel) and seconds of the object the
 * device's specialised kernel was loaded from. */
int wo_dev_jit_origin(WoDev* dev, double* seconds);
int wo_dev_lanes_info(WoDev* dev, uint32_t* out);
/* the last launch's path kernel: key (65 B), out[4] = kind, scratch B/lane, VGPRs, LDS */
int wo_dev_kernel_info(WoDev* dev, char* key_hex, uint32_t* out);
/* Wait for the slot's frame; *host = its pixels (RGBA float; NULL when the
 * submit did not map them back), *host_bgra8 (if non-NULL) = its present
 * encode; both valid until the slot is submitted again. */
int wo_dev_frame_wait(WoDev* dev, int slot, float const** host, uint32_t const** host_bgra8, char* err,
                      size_t errlen);
/* The float pixels of a waited-for slot, copied from the device now if the
 * submit left them there (synchronous). */
int wo_dev_frame_map_float(WoDev* dev, int slot, float const** host, char* err, size_t errlen);
/* Pipeline timestamps of present-slot frames (on: from now; see
 * wo_renderer_frame_stamps).  slot_stamps: the slot's last frame, ms after the
 * stamps were turned on: render begin, render end, map-back end; -1 if none. */
int wo_dev_set_stamps(WoDev* dev, int on, char* err, size_t errlen);
int wo_dev_slot_stamps(WoDev* dev, int slot, double out[3]);
/* Drain every stream of the device. */
int wo_dev_sync(WoDev* dev);
/* Present encode of `pixels` float4 pixels into B8G8R8A8 sRGB (present.c) on
 * the current device, async on `stream`. */
int wo_dev_srgb8(void const* d_rgba, void* d_bgra8, size_t pixels, void* stream, char* err, size_t errlen);
/* present.c: the encode's 255 thresholds (host) */
void wo_srgb8_thresholds(float out[255]);
/* One frame of this rank's tiles with the counting variant of its path kernel
 * (synchronous): counts[WO_WORK_KINDS] = lane counts of the work that ran. */
int wo_dev_count_work(WoDev* dev, WoFrame const* frame, unsigned long long* counts, char* err, size_t errlen);
/* Full frame into host memory (synchronous; owns a device frame buffer). */
int wo_dev_render_host(WoDev* dev, WoFrame const* frame, float* host_rgba, char* err, size_t errlen);
/* Un-interleave gathered rank buffers into a frame (async on `stream`). */
int wo_dev_assemble(void const* d_gathered, void* d_frame, uint32_t width, uint32_t height,
                    uint32_t tile_rows, uint32_t nranks, uint32_t band_cycle, uint32_t band_skip, void* stream,
                    char* err, size_t errlen);

#ifdef __cplusplus
}
#endif

#endif /* WOLOLO_WO_DEV_H */
