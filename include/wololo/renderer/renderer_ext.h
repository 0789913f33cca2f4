/*
 * wololo/renderer/renderer_ext.h -- headless / north-star extensions of the
 * renderer API.  New names only; nothing here changes renderer.h.
 *
 * The reference declares `Wo_Material` but never uses it (renderer.h:16) and has
 * no camera, sample-count or bounce controls; its per-frame inputs are the 12-byte
 * UBO {time, W, H} (renderer.c:72-80, 2133-2155).  These calls add them.
 *
 * Return convention for int-returning calls: 0 on success, negative on error;
 * wo_renderer_last_error() returns a thread-local message for the last failure.
 */
#ifndef WOLOLO_RENDERER_RENDERER_EXT_H
#define WOLOLO_RENDERER_RENDERER_EXT_H

#include <stddef.h>
#include <stdint.h>

#include "wololo/renderer/renderer.h"
#include "wololo/wo_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

#define WO_NODE_INVALID ((Wo_Node)0xFFFFFFFFu)
#define WO_MATERIAL_INVALID ((Wo_Material)0xFFFFFFFFu)

typedef enum Wo_ShadingMode {
    WO_SHADING_UBERSHADER_RT1 = WO_MODE_UBERSHADER_RT1, /* default: the reference's image */
    WO_SHADING_DEBUG_ST = WO_MODE_DEBUG_ST,
    WO_SHADING_PATHTRACE = WO_MODE_PATHTRACE,
    WO_SHADING_NORMALS = WO_MODE_NORMALS,
} Wo_ShadingMode;

typedef struct Wo_RenderParams {
    uint32_t width, height;  /* frame size in pixels */
    uint32_t spp;            /* samples per pixel (PATHTRACE) */
    uint32_t max_depth;      /* max segments per path (PATHTRACE) */
    uint32_t seed;           /* RNG stream selector */
    uint32_t mode;           /* Wo_ShadingMode */
    uint32_t sample_offset;  /* index of the first sample (progressive rendering) */
    float time_sec;          /* UBERSHADER_RT1: time_since_start_sec */
} Wo_RenderParams;

/* Defaults: 1280x720 (or the app window), 1 spp, 8 segments, seed 0, UBERSHADER_RT1. */
void wo_render_params_default(Wo_RenderParams* params);

/* ---- materials (leaf nodes carry one; the default, id 0, is lambertian 0.5 grey) ---- */
Wo_Material wo_renderer_add_lambertian_material(Wo_Renderer* r, Wo_Vec3 albedo);
Wo_Material wo_renderer_add_metal_material(Wo_Renderer* r, Wo_Vec3 albedo, Wo_Scalar fuzz);
Wo_Material wo_renderer_add_dielectric_material(Wo_Renderer* r, Wo_Scalar refraction_index);
/* Only sphere / half-space leaves take materials.  Returns false on a bad handle. */
bool wo_renderer_set_node_material(Wo_Renderer* r, Wo_Node leaf, Wo_Material material);

/* ---- camera (RTIOW "positionable camera" with defocus blur) ---- */
void wo_renderer_set_camera(Wo_Renderer* r, Wo_Vec3 look_from, Wo_Vec3 look_at, Wo_Vec3 view_up,
                            Wo_Scalar vertical_fov_deg, Wo_Scalar aperture, Wo_Scalar focus_dist);

/* Parameters used by wo_renderer_draw_frame(); time_sec is overridden by the
 * app clock unless `pin_time` is non-zero. */
void wo_renderer_set_draw_params(Wo_Renderer* r, Wo_RenderParams const* params, int pin_time);

/* Render a whole frame into a host buffer of width*height*4 floats (RGBA,
 * row 0 = top).  Synchronous.  Includes the device->host copy. */
int wo_renderer_render_f32(Wo_Renderer* r, Wo_RenderParams const* params, float* out_rgba);

/* Render this rank's row tiles into DEVICE memory `d_out`
 * (wo_rank_local_rows(height, tile_rows, nranks) * width float4s) on HIP stream
 * `stream` (NULL = default stream), asynchronously.  Tiles are `tile_rows` rows;
 * rank r owns tiles g with g % nranks == r, stored in increasing g.  If
 * `d_segment_counter` is non-NULL, the number of traced CSG ray segments is
 * atomically added to it (uint64, device memory). */
int wo_renderer_render_rows_device(Wo_Renderer* r, Wo_RenderParams const* params, void* d_out,
                                   uint32_t tile_rows, uint32_t rank, uint32_t nranks, void* stream,
                                   unsigned long long* d_segment_counter);

/* Executed-work counters: render this rank's tiles once (synchronously, into
 * scratch memory) with the counting variant of the path kernel the renderer
 * runs -- same image, same segments -- and fill counts[WO_WORK_KINDS]
 * (wo_scene.h: segments, sphere / half-space / BOUND tests, events stored,
 * events swept, re-collects, primary segments; lane counts).  A measurement
 * aid (the counting kernel is slower); PATHTRACE / NORMALS frames only. */
int wo_renderer_count_work(Wo_Renderer* r, Wo_RenderParams const* params, uint32_t tile_rows, uint32_t rank,
                           uint32_t nranks, unsigned long long* counts);

/* Un-interleave nranks gathered local buffers (rank-major, each
 * wo_rank_local_rows(...) * width float4s) into a width*height float4 frame. */
int wo_assemble_rows_device(void const* d_gathered, void* d_frame, uint32_t width, uint32_t height,
                            uint32_t tile_rows, uint32_t nranks, void* stream);
/* The same for row bands weighted by wo_renderer_set_band_weight (buffers of
 * wo_rank_local_rows_ex(..., band_cycle, band_skip) rows). */
int wo_assemble_rows_device_ex(void const* d_gathered, void* d_frame, uint32_t width, uint32_t height,
                               uint32_t tile_rows, uint32_t nranks, uint32_t band_cycle, uint32_t band_skip,
                               void* stream);
/* Row bands of the renderer's multi-rank frames (render_rows_device, count_work
 * with nranks > 1): in every band_cycle rounds of the ranks rank 0 sits out
 * band_skip (0 = a band per rank and round, the default), so the rank that also
 * gathers, assembles and presents renders less (wo_scene.h wo_band_global).
 * -1 if 0 < band_skip >= band_cycle. */
int wo_renderer_set_band_weight(Wo_Renderer* r, uint32_t band_cycle, uint32_t band_skip);

/* ---- several GPUs per renderer ----
 * The reference renders on physical device 0 only (renderer.c:519-520).  Here
 * one renderer can split every frame over n ranks: rank i renders the
 * row-cyclic 4-row tiles g with g % n == i on HIP device (d0 + i) mod
 * visible devices (d0 = wo_renderer_device), ranks 1..n-1 copy their share to
 * d0 (peer DMA over xGMI; through pinned host memory when the pair has no peer
 * path), and d0 assembles and presents the frame.  The image is the same bit
 * for bit for every n.  n above the device count stacks ranks on one device.
 * After set_devices(n), draw_frame, render_f32, render_accumulate and
 * render_frame_device use all n ranks; render_rows_device (the caller splits
 * the frame) uses d0 only.
 * Default: WOLOLO_DEVICES=N|all (n ranks, always), else, for a renderer created
 * with an app (the demo), every visible GPU with the rank count chosen per frame
 * by workload: the reference shader, the debug view and normals frames (a few
 * microseconds of kernel) stay on d0, and a path-traced frame takes one rank
 * per WOLOLO_RANK_MIN_SAMPLES (default 4 Mi) samples, up to all of them; a
 * renderer without an app gets one rank.  WOLOLO_DEVICES=auto (every GPU) or
 * auto:N (N ranks) applies the app's workload rule to any renderer.  Returns n,
 * or -1 (last_error; the
 * renderer then keeps one rank). */
int wo_renderer_set_devices(Wo_Renderer* r, int n);
/* Ranks a frame is split over (0 for a device-less renderer). */
int wo_renderer_device_count(Wo_Renderer* r);
/* Ranks a frame with these parameters is split over (the workload rule above
 * for the app's default, else wo_renderer_device_count). */
int wo_renderer_frame_ranks(Wo_Renderer* r, Wo_RenderParams const* params);
/* How rank `rank`'s share reaches d0: 0 same device (device copy), 1 peer DMA,
 * 2 through pinned host memory (no peer path, or WOLOLO_PEER=staged); -1 for
 * rank 0 or a bad rank. */
int wo_renderer_peer_mode(Wo_Renderer* r, int rank);
/* Render a whole frame over the renderer's ranks into DEVICE memory d_frame
 * (width*height float4s on d0 = wo_renderer_device; row 0 = top), ordered on
 * HIP stream `stream` of d0 (NULL = its default stream): d_frame is written on
 * `stream` after the work queued on it before the call, and is complete when
 * `stream` reaches the point of the call's return.  The ranks render into the
 * library's own buffers on their own streams, so they may start earlier.
 * Asynchronous.  Consecutive calls alternate between two gather buffers, so
 * frame k+1 renders while frame k is gathered.  No present.  The traced CSG
 * segments are counted per rank (wo_renderer_take_segments). */
int wo_renderer_render_frame_device(Wo_Renderer* r, Wo_RenderParams const* params, void* d_frame, void* stream);
/* Segments traced by render_frame_device frames since the last call, summed
 * over the ranks (waits for their devices; the counters restart at 0). */
int wo_renderer_take_segments(Wo_Renderer* r, unsigned long long* total);

/* ---- frame pipeline and progressive rendering ----
 * The reference's draw_frame_with_renderer (renderer.c:2085-2219) ends every
 * frame with vkQueueWaitIdle (2212).  wo_renderer_draw_frame instead submits
 * frame k (asynchronous: the render on the device's render stream; the map-back
 * -- present encode and its copy to pinned host memory -- on a copy stream once
 * the render is done, so frame k+1's render never waits for frame k's copies)
 * and then waits for and presents frame k-1: the GPU renders while the host
 * presents, one frame of latency.  Presenting = the last frame below, plus a PPM
 * dump when WOLOLO_OUTPUT names a file. */
/* Wait for and present every submitted frame.  0, or -1 (last_error). */
int wo_renderer_finish(Wo_Renderer* r);
/* Host pixels of the last presented frame (RGBA float, row 0 = top; NULL
 * before the first), valid until the next draw_frame / finish.  The float frame
 * is copied from the device on the first call after a present (unless
 * wo_renderer_set_map_float asks for every frame), so a caller that only
 * presents never pays for its 16 bytes per pixel of map-back. */
float const* wo_renderer_last_frame(Wo_Renderer* r, uint32_t* width, uint32_t* height);
/* every_frame != 0: map each presented frame's float pixels back with its
 * present encode (asynchronously, on the copy stream); 0 (default): on demand. */
void wo_renderer_set_map_float(Wo_Renderer* r, int every_frame);
/* Pipeline timestamps (diagnostics): while on, each frame draw_frame presents
 * logs three times in ms after the call that turned them on -- render begin,
 * render end (both on the render stream) and map-back end (copy stream).
 * set: 0 or -1 (drains the pipeline first); frame_stamps copies up to
 * max_frames logged frames (oldest first, 3 doubles each) into out, empties the
 * log and returns how many, or -1.  The log holds 256 frames. */
int wo_renderer_set_frame_stamps(Wo_Renderer* r, int on);
int wo_renderer_frame_stamps(Wo_Renderer* r, double* out, int max_frames);
/* Present encode of the last presented frame: B8G8R8A8 sRGB, one uint32 per
 * pixel (B in the low byte) -- the reference's preferred swapchain format
 * (renderer.c:813-832) -- made on the GPU by wo_srgb8_encode_device.  Same
 * lifetime as wo_renderer_last_frame. */
uint32_t const* wo_renderer_last_frame_bgra8(Wo_Renderer* r, uint32_t* width, uint32_t* height);
/* The sRGB present encode (what the reference's B8G8R8A8_SRGB attachment does in
 * fixed function): per channel code = round-half-up(255 * srgb(clamp(v, 0, 1)))
 * with the IEC 61966-2-1 transfer function (NaN -> 0); alpha is linear.
 * wo_srgb8_thresholds gives the 255 floats the code counts (code(v) = number of
 * thresholds <= v); the device and host encodes use the same table, so they
 * agree bit for bit. */
void wo_srgb8_thresholds(float out[255]);
int wo_srgb8_encode_device(void const* d_rgba, void* d_bgra8, size_t pixels, void* stream);
void wo_srgb8_encode_host(float const* rgba, uint32_t* bgra8, size_t pixels);

/* Progressive accumulation for draw_frame (off by default): while on,
 * consecutive PATHTRACE frames with the same scene, camera and draw
 * parameters add params.spp new samples each (the sample index continues) and
 * present the mean over all of them -- bit for bit one render of that many
 * samples.  Any change starts over. */
void wo_renderer_set_progressive(Wo_Renderer* r, int on);
/* Samples per pixel in the current accumulation (0: none). */
uint32_t wo_renderer_accumulated_spp(Wo_Renderer* r);
/* Synchronous form: render params->spp more samples into the accumulation
 * (reset != 0, or different parameters / scene: start over) and write the mean
 * over all accumulated samples to out_rgba (width*height*4 floats, may be
 * NULL).  Returns the accumulated samples per pixel, or -1. */
int wo_renderer_render_accumulate(Wo_Renderer* r, Wo_RenderParams const* params, float* out_rgba, int reset);

/* Compile the node tables into the flattened program (done lazily by every
 * render call; exposed for tests).  Returns the number of records. */
int wo_renderer_compile(Wo_Renderer* r);
/* Host views of the compiled scene (valid until the next node/material change). */
WoRec const* wo_renderer_program(Wo_Renderer* r, uint32_t* n_recs, uint32_t* n_prims);
WoMaterial const* wo_renderer_materials(Wo_Renderer* r, uint32_t* n_materials);
/* Fill a WoFrame exactly as the kernels receive it (camera resolved for params). */
int wo_renderer_frame_desc(Wo_Renderer* r, Wo_RenderParams const* params, uint32_t tile_rows,
                           uint32_t rank, uint32_t nranks, WoFrame* out);

/* Path-tracer kernel selection (results are identical; only speed differs).
 *   AUTO         union-only scenes of more than WOLOLO_LANES_MIN_PRIMS (256)
 *                primitives -> LANES; else scenes of up to WOLOLO_JIT_MAX_PRIMS
 *                (256) primitives -> JIT; else INTERPRETER.
 *   INTERPRETER  the postfix-program interpreter kernel.
 *   JIT          the scene-specialised kernel, compiled with hiprtc at scene
 *                upload, for scenes of up to WOLOLO_JIT_MAX_PRIMS primitives
 *                (else, or if compilation fails, the interpreter).
 *   LANES        per-lane BOUND traversal, for union-only scenes (others fall
 *                back to AUTO's choice).
 * Environment: WOLOLO_TRACER=auto|interpreter|jit|lanes sets the initial value.
 * Takes effect at the next render. */
typedef enum Wo_Tracer {
    WO_TRACER_AUTO = 0,
    WO_TRACER_INTERPRETER = 1,
    WO_TRACER_JIT = 2,
    WO_TRACER_LANES = 3,
} Wo_Tracer;
void wo_renderer_set_tracer(Wo_Renderer* r, Wo_Tracer tracer);
/* Compatibility form: 0 = INTERPRETER, anything else = AUTO. */
void wo_renderer_set_jit(Wo_Renderer* r, int mode);
/* Which path kernel the last render used: "jit", "lanes", "interpreter" or "none". */
char const* wo_renderer_trace_path(Wo_Renderer* r);
/* Scene edits do not stall draw_frame (on by default; WOLOLO_JIT_ASYNC=0 turns it
 * off): when the specialised kernel of the edited scene is in neither code-object
 * cache, draw_frame starts its hiprtc compile on a background host thread and
 * renders with the interpreter -- the same image bit for bit -- until the compile
 * has ended; the first draw_frame after that switches to it.  render_f32,
 * render_accumulate, render_rows_device, render_frame_device and count_work wait
 * for a compile in flight (batch renders get the specialised kernel) -- except
 * under WO_TRACER_AUTO for a general tree above 256 primitives (1-2 minutes of
 * hiprtc), which the lane tracer renders meanwhile in batch renders too.  The
 * nodes are added incrementally as in the reference (renderer.c:2232-2275). */
void wo_renderer_set_jit_async(Wo_Renderer* r, int on);
/* 1 while a background compile of the current scene's kernel is in flight. */
int wo_renderer_jit_pending(Wo_Renderer* r);
/* Compile, upload and load the current scene's kernels now, waiting for any
 * background compile (a benchmark's set-up: the timed frames then run the
 * kernel AUTO settles on).  Extends the reference's per-frame scene upload
 * (renderer.c:2085-2219 records it into every frame); 0, or -1 on failure. */
int wo_renderer_prepare(Wo_Renderer* r);

/* HIP source of the scene-specialised kernel for the current scene (NULL if
 * the scene has no primitives); release with wo_free(). */
char* wo_renderer_jit_source(Wo_Renderer* r);
/* Compile `src` with hiprtc for `arch` (e.g. "gfx950") without loading it --
 * needs no GPU.  Returns 0, or -1 with the compiler log in err. */
int wo_jit_compile_check(char const* src, char const* arch, char* err, size_t errlen);
/* Code object of the specialised kernel `src` for `arch`, as a render would get
 * it: from this process's cache, else the on-disk cache (WOLOLO_JIT_CACHE =
 * directory, "0" = off; default $XDG_CACHE_HOME/wololo/jit or
 * ~/.cache/wololo/jit; entries keyed by the SHA-256 of source, headers,
 * target, options and hiprtc version), else compiled with hiprtc and stored.
 * *origin: 0 process cache, 1 disk cache, 2 compiled; *seconds: time taken;
 * key_hex (65 bytes or NULL): the key.  Returns the object's size or -1 (err).
 * Needs no GPU. */
long long wo_jit_code_object(char const* src, char const* arch, int* origin, double* seconds, char* key_hex,
                             char* err, size_t errlen);
/* The specialised kernel's resources as its code object states them (its AMDHSA
 * kernel descriptor, as wo_renderer_kernel_info reports them): out[0] scratch bytes
 * per lane (the private segment), out[1] static LDS bytes per workgroup (the group
 * segment).  Compiles (or takes from the caches) like wo_jit_code_object.  Returns 0,
 * or -1 (err).  Needs no GPU. */
int wo_jit_code_resources(char const* src, char const* arch, uint32_t* out, char* err, size_t errlen);
/* Where the renderer's specialised kernel came from (origin as above; -1: the
 * renderer does not run one) and the seconds it took (compile or load). */
int wo_renderer_jit_info(Wo_Renderer* r, double* seconds);
/* The lane tracer's BVH (union-only scenes): out[0] internal nodes, out[1] its
 * depth in internal levels (= the per-lane LDS stack entries; at most 24),
 * out[2] top nodes staged in LDS, out[3] primitives tested on every query (no
 * box), out[4] the kernel form of the last path launch (0-14 the lane tracer's
 * forms, 11-14 the resumable walk; trace_kernels.hip PathKind).  `out` holds 5
 * entries.  Returns 0, or -1 when the renderer does not run the lane tracer. */
int wo_renderer_lanes_info(Wo_Renderer* r, uint32_t* out);
/* The path kernel of the last launch as the runtime loaded it: key_hex (65 bytes)
 * gets the specialised kernel's code-object key (SHA-256 of source, options and
 * toolchain) or "static:<kind>:<40 hex digits of the library kernels' source hash>"; out[0] = kind (as lanes_info's), out[1] = private
 * (scratch) bytes per lane, out[2] = VGPRs, out[3] = static LDS bytes.  Profile
 * sessions record it beside their counters.  0, or -1 before any path launch. */
int wo_renderer_kernel_info(Wo_Renderer* r, char* key_hex, uint32_t* out);
void wo_free(void* p);

size_t wo_renderer_node_count(Wo_Renderer* r);
char const* wo_renderer_name(Wo_Renderer* r);
/* HIP device ordinal the renderer runs on; -1 for a device-less renderer. */
int wo_renderer_device(Wo_Renderer* r);
char const* wo_renderer_last_error(void);
/* Empty this thread's last-error message (so a caller can tell a new failure). */
void wo_renderer_clear_error(void);

/* ---- library-level ---- */
/* sizeof(type) (field NULL) or offsetof(type, field) as this library was
 * compiled, for the value types of the C ABI (Wo_Vec3, Wo_Quaternion,
 * Wo_Node_Argument, Wo_RenderParams, WoRec, WoMaterial, WoCamera, WoFrame);
 * (size_t)-1 for an unknown name.  Bindings check their mirrors with it. */
size_t wo_abi_layout(char const* type, char const* field);
/* Device self-check of the path tracer's fast correctly rounded square root
 * (which = 0) or reciprocal (1) against the IEEE expansions, over every float
 * bit pattern in [lo_bits, hi_bits] (on the current HIP device, synchronous).
 * 0 and the mismatch count / smallest mismatching pattern, or -1. */
int wo_fastmath_check(int which, uint32_t lo_bits, uint32_t hi_bits, unsigned long long* mismatches,
                      uint32_t* first_mismatch);
char const* wo_version(void);
/* Number of visible HIP devices (0 when none / no driver). */
int wo_hip_device_count(void);
/* Version of the HIP runtime this process uses (hipRuntimeGetVersion, e.g.
 * 70226015), or -1.  The scene-specialised kernels are compiled by the hiprtc of
 * the same installation: whichever libamdhip64.so.7 / libhiprtc.so.7 the process
 * loaded first (a PyTorch wheel bundles its own). */
int wo_hip_runtime_version(void);

#ifdef __cplusplus
}
#endif

#endif /* WOLOLO_RENDERER_RENDERER_EXT_H */
