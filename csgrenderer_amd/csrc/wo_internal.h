/*
 * wo_internal.h -- private structures of the host library.
 *
 * The node store mirrors the reference's (renderer.c:180-217): a type per node,
 * a parameter record per node, and a non-root bitset; handles are sequential.
 * The reference packs everything into one calloc slab (allocate_renderer,
 * renderer.c:338-393); here the tables are separate allocations owned by the
 * renderer, sized once from max_node_count.
 */
#ifndef WOLOLO_WO_INTERNAL_H
#define WOLOLO_WO_INTERNAL_H

#include <stddef.h>
#include <stdint.h>

#include "wololo/config.h"
#include "wololo/renderer/renderer_ext.h"
#include "wololo/wo_scene.h"
#include "wo_dev.h"

#define WO_MAX_DEVICES 16

/* Node kinds: same order as the reference's NodeType (renderer.c:182-188). */
enum {
    WO_NODE_SPHERE = 0,
    WO_NODE_HALFSPACE = 1,
    WO_NODE_UNION = 2,
    WO_NODE_INTERSECTION = 3,
    WO_NODE_DIFFERENCE = 4,
};

typedef struct WoNodeInfo {
    uint32_t kind;
    Wo_Material material;  /* leaves only */
    Wo_Scalar radius;      /* sphere */
    Wo_Vec3 normal;        /* half-space outward normal (as given) */
    Wo_Node_Argument left, right;  /* binops */
} WoNodeInfo;

typedef struct WoCameraDesc {
    Wo_Vec3 look_from, look_at, view_up;
    double vfov_deg, aperture, focus_dist;
} WoCameraDesc;

struct Wo_Renderer {
    size_t max_node_count;
    size_t node_count;
    WoNodeInfo* nodes;
    uint64_t* nonroot;  /* bitset, ceil(max/64) words */
    char* name;
    Wo_App* app;

    WoMaterial* mats;
    uint32_t n_mats, cap_mats;

    WoCameraDesc camera;

    Wo_RenderParams draw;
    int pin_time;
    double t0;  /* creation time (seconds, monotonic) when there is no app */

    /* compiled program (host copy) */
    WoRec* prog;
    uint32_t n_recs, n_prims, cap_recs;
    int dirty;          /* nodes/materials changed since the last compile */
    int dev_stale;      /* device copy out of date */

    int device;         /* -1: device-less (tests only) */
    WoDev* dev;         /* rank 0: uploads, presents (== devs[0]) */
    uint32_t ndevs;     /* ranks a frame is split over (wo_renderer_set_devices) */
    WoDev* devs[WO_MAX_DEVICES];
    int ranks_auto;     /* the app's default: ranks per frame chosen by workload */
    uint64_t dframe_seq;  /* render_frame_device calls (alternating gather slots) */

    int tracer;         /* Wo_Tracer */
    int jit_loaded;     /* the device runs the scene-specialised kernel */
    /* background compile (draw_frame): frames use the interpreter until it ends */
    WoJitJob* jit_job;      /* compiling jit_want */
    char* jit_want;         /* the current scene's specialised source, while deferred */
    WoJitJob* jit_old[8];   /* compiles of scenes edited since (joined when done) */
    uint32_t n_jit_old;
    int jit_async;          /* draw_frame may defer the compile (default; WOLOLO_JIT_ASYNC=0: off) */
    int lanes_loaded;   /* the device runs the lane-traversal kernel */

    uint64_t frames_drawn;
    uint64_t view_version;  /* bumped by every scene / material / camera change */

    /* progressive accumulation (draw_frame when `progressive`, render_accumulate) */
    int progressive;
    int acc_valid;
    uint32_t acc_spp;          /* samples per pixel in the accumulation */
    Wo_RenderParams acc_params;
    uint64_t acc_view;
    uint32_t acc_ranks;        /* ranks the accumulation is split over (per-rank sums) */

    /* draw_frame pipeline: frame k renders while frame k-1 is presented */
    int pending[2];
    uint32_t pend_w[2], pend_h[2];
    uint64_t frame_seq;
    float const* last_frame;     /* NULL until mapped back (lazily, wo_renderer_last_frame) */
    uint32_t const* last_bgra8;  /* its present encode (B8G8R8A8 sRGB) */
    uint32_t last_w, last_h;
    int last_slot;               /* the presented frame's slot (-1: none) */
    int map_float;               /* copy every presented float frame to the host (else on demand) */
    uint32_t band_cycle, band_skip; /* weighted row bands of a multi-rank frame (wo_renderer_set_band_weight) */
    /* pipeline timestamps (wo_renderer_set_frame_stamps): per presented frame,
     * render begin / render end / map-back end in ms */
    int stamps;
    uint32_t n_stamps;
    double stamp_log[256][3];
};

/* scene_compile.c */
int wo_compile_scene(Wo_Renderer* r, char* err, size_t errlen);
void wo_resolve_camera(WoCameraDesc const* desc, uint32_t width, uint32_t height, WoCamera* out);

/* scene_jit.c: HIP source of the scene-specialised trace kernel (malloc'd) */
char* wo_generate_jit_source(WoRec const* prog, uint32_t n_recs, uint32_t n_prims);

/* present.c: binary PPM (RGB) of a B8G8R8A8 frame; 0 or -1 (last_error) */
int wo_write_ppm_bgra8(char const* path, uint32_t const* bgra8, uint32_t w, uint32_t h);

/* renderer.c */
void wo_set_error(char const* fmt, ...);
double wo_monotonic_sec(void);

#endif /* WOLOLO_WO_INTERNAL_H */
