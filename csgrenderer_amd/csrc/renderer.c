/*
 * renderer.c -- the wololo renderer C API on HIP.
 *
 * Replaces src/wololo/renderer/renderer.c of the reference:
 *   - node store: same semantics as allocate_node / set_nonroot_node /
 *     add_*_node / wo_renderer_isroot (ref renderer.c:2220-2313), but the node
 *     is allocated OUTSIDE assert() (the reference's allocation vanishes under
 *     NDEBUG, renderer.c:2234) and a full store returns WO_NODE_INVALID;
 *   - Vulkan init (renderer.c:394-1810) -> one WoDev (HIP device + stream);
 *   - draw_frame_with_renderer (renderer.c:2085-2219): UBO {time, W, H} ->
 *     WoFrame, vkQueueSubmit -> kernel launch, present -> optional image dump.
 */
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "wo_internal.h"

static _Thread_local char g_err[512];

void wo_set_error(char const* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

char const* wo_renderer_last_error(void) { return g_err; }

void wo_renderer_clear_error(void) { g_err[0] = '\0'; }

char const* wo_version(void) { return "wololo-mi355x 0.1 (gfx950)"; }

double wo_monotonic_sec(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int wo_hip_device_count(void) { return wo_dev_count(); }

void wo_render_params_default(Wo_RenderParams* p) {
    memset(p, 0, sizeof *p);
    p->width = 1280;
    p->height = 720;
    p->spp = 1;
    p->max_depth = 8;
    p->seed = 0;
    p->mode = WO_SHADING_UBERSHADER_RT1;
    p->sample_offset = 0;
    p->time_sec = 0.0f;
}

static int env_flag(const char* name) {
    const char* v = getenv(name);
    return v && *v && strcmp(v, "0") != 0;
}

static void jit_old_reap(Wo_Renderer* r, int wait);

/* ---------------------------------------------------------------- lifecycle */

Wo_Renderer* wo_renderer_new(Wo_App* app, char const* name, size_t max_node_count) {
    Wo_Renderer* r = (Wo_Renderer*)calloc(1, sizeof(Wo_Renderer));
    if (!r) {
        fprintf(stderr, WO_LOG_PREFIX " Failed to allocate Wo_Renderer.\n");
        return NULL;
    }
    r->max_node_count = max_node_count;
    size_t words = max_node_count / 64 + 1;
    r->nodes = (WoNodeInfo*)calloc(max_node_count ? max_node_count : 1, sizeof(WoNodeInfo));
    r->nonroot = (uint64_t*)calloc(words, sizeof(uint64_t));
    r->cap_mats = 16;
    r->mats = (WoMaterial*)calloc(r->cap_mats, sizeof(WoMaterial));
    if (!r->nodes || !r->nonroot || !r->mats) {
        fprintf(stderr, WO_LOG_PREFIX " Failed to allocate node tables for %zu nodes.\n", max_node_count);
        wo_renderer_del(r);
        return NULL;
    }
    /* name: copied; empty -> NULL (ref allocate_renderer, renderer.c:344-351, 384-391) */
    if (name && name[0]) {
        size_t n = strlen(name);
        r->name = (char*)malloc(n + 1);
        if (r->name) memcpy(r->name, name, n + 1);
    }
    r->app = app;
    r->last_slot = -1;
    /* material 0: default lambertian grey */
    r->mats[0].kind = WO_MAT_LAMBERTIAN;
    r->mats[0].albedo[0] = r->mats[0].albedo[1] = r->mats[0].albedo[2] = 0.5f;
    r->n_mats = 1;
    r->camera.look_from = wo_vec3_make(0.0, 0.0, 0.0);
    r->camera.look_at = wo_vec3_make(0.0, 0.0, -1.0);
    r->camera.view_up = wo_vec3_make(0.0, 1.0, 0.0);
    r->camera.vfov_deg = 90.0;
    r->camera.aperture = 0.0;
    r->camera.focus_dist = 1.0;
    wo_render_params_default(&r->draw);
    if (app) {
        r->draw.width = wo_app_window_width(app);
        r->draw.height = wo_app_window_height(app);
    }
    r->t0 = wo_monotonic_sec();
    r->dirty = 1;
    r->view_version++;
    {
        const char* t = getenv("WOLOLO_TRACER");
        r->tracer = WO_TRACER_AUTO;
        if (t && strcmp(t, "interpreter") == 0) r->tracer = WO_TRACER_INTERPRETER;
        if (t && strcmp(t, "jit") == 0) r->tracer = WO_TRACER_JIT;
        if (t && strcmp(t, "lanes") == 0) r->tracer = WO_TRACER_LANES;
    }
    r->device = -1;
    r->jit_async = !(getenv("WOLOLO_JIT_ASYNC") && strcmp(getenv("WOLOLO_JIT_ASYNC"), "0") == 0);

    char err[256] = {0};
    int ndev = wo_dev_count();
    if (ndev <= 0) {
        if (env_flag("WOLOLO_ALLOW_NO_DEVICE")) {
            /* node store only (host tests); every render call fails loudly */
            return r;
        }
        fprintf(stderr, WO_LOG_PREFIX " No HIP device available; cannot create renderer.\n");
        wo_set_error("no HIP device available");
        wo_renderer_del(r);
        return NULL;
    }
    int dev = wo_dev_current();
    if (dev < 0) dev = 0;
    if (wo_dev_create(dev, &r->dev, err, sizeof err) != 0) {
        fprintf(stderr, WO_LOG_PREFIX " HIP init failed: %s\n", err);
        wo_set_error("HIP init failed: %s", err);
        wo_renderer_del(r);
        return NULL;
    }
    r->device = dev;
    r->devs[0] = r->dev;
    r->ndevs = 1;
    /* Ranks per frame: WOLOLO_DEVICES=N|all (always N), else every visible GPU
     * for a renderer of the app (the demo's, main.c:38) with the count chosen
     * per frame by workload (frame_ranks), and one for a library caller (one
     * process per GPU, e.g. bench.py under torchrun). */
    int want = 1, automatic = 0;
    const char* dv = getenv("WOLOLO_DEVICES");
    if (dv && strncmp(dv, "auto", 4) == 0) {
        /* the app's rule for any renderer; "auto:N" = N ranks (stacked when N
         * exceeds the GPUs: how the rule is tested on one GPU) */
        want = dv[4] == ':' ? atoi(dv + 5) : ndev;
        automatic = 1;
    } else if (dv && *dv) {
        want = strcmp(dv, "all") == 0 ? ndev : atoi(dv);
    } else if (app) {
        want = ndev;
        automatic = 1;
    }
    if (want > WO_MAX_DEVICES) want = WO_MAX_DEVICES;
    if (want > 1) {
        if (wo_renderer_set_devices(r, want) < 0)
            fprintf(stderr, WO_LOG_PREFIX " multi-GPU setup failed (%s); rendering on device %d only.\n",
                    wo_renderer_last_error(), dev);
        else
            r->ranks_auto = automatic;
    }
    return r;
}

/* Ranks a frame is split over.  Explicit (set_devices, WOLOLO_DEVICES): all of
 * them.  The app's default: the reference shader, the debug view and normals
 * frames are a few microseconds of kernel (C1 1080p: 0.019 ms), which n-1 share
 * copies, event waits and an assembly would only slow down, so they stay on
 * rank 0; a path-traced frame takes one rank per WOLOLO_RANK_MIN_SAMPLES
 * samples (default 4 Mi: about 0.1 ms of csg32 kernel per rank). */
static uint32_t frame_ranks(Wo_Renderer const* r, Wo_RenderParams const* p) {
    if (r->ndevs <= 1u || !r->ranks_auto) return r->ndevs ? r->ndevs : 1u;
    if (p->mode != WO_SHADING_PATHTRACE) return 1u;
    uint64_t per = 1ull << 22;
    const char* e = getenv("WOLOLO_RANK_MIN_SAMPLES");
    if (e && *e) per = strtoull(e, NULL, 10);
    if (per == 0) return r->ndevs;
    const uint64_t samples = (uint64_t)p->width * p->height * p->spp;
    uint64_t n = samples / per;
    if (n < 1) n = 1;
    return n < r->ndevs ? (uint32_t)n : r->ndevs;
}

int wo_renderer_frame_ranks(Wo_Renderer* r, Wo_RenderParams const* params) {
    if (!r || !r->dev || !params) return 0;
    return (int)frame_ranks(r, params);
}

int wo_renderer_peer_mode(Wo_Renderer* r, int rank) {
    if (!r || rank < 1 || (uint32_t)rank >= r->ndevs) return -1;
    return wo_dev_peer_mode(r->devs[rank]);
}

/* Row-cyclic frames over n ranks: rank i on HIP device (device + i) mod
 * visible devices, so n above the device count stacks ranks on one device
 * (each rank keeps its own stream and buffers). */
int wo_renderer_set_devices(Wo_Renderer* r, int n) {
    if (!r || !r->dev) {
        wo_set_error("renderer has no HIP device");
        return -1;
    }
    if (n < 1 || n > WO_MAX_DEVICES) {
        wo_set_error("device count %d out of range [1, %d]", n, WO_MAX_DEVICES);
        return -1;
    }
    if (wo_renderer_finish(r)) return -1;
    const int ndev = wo_dev_count();
    const int cur = wo_dev_current();
    r->ranks_auto = 0; /* an explicit count: every frame uses all n ranks */
    /* fault injection for the tests: rank k's set-up fails (WOLOLO_FAULT_RANK=k) */
    const char* fk = getenv("WOLOLO_FAULT_RANK");
    const int fault_rank = fk && *fk ? atoi(fk) : -1;
    /* the root's streams may still read the ranks' buffers (a device frame's
     * host-staged H2D from a rank's pinned copy): drain them first */
    if (r->ndevs > 1) (void)wo_dev_sync(r->dev);
    for (uint32_t i = 1; i < r->ndevs; ++i) {
        wo_dev_destroy(r->devs[i]);
        r->devs[i] = NULL;
    }
    r->ndevs = 1;
    r->dev_stale = 1; /* every rank needs the scene (and the kernel) */
    r->acc_valid = 0; /* accumulations are per rank */
    int rc = n;
    char err[256] = {0};
    for (int i = 1; i < n; ++i) {
        const int d = ndev > 0 ? (r->device + i) % ndev : r->device;
        if (i == fault_rank) {
            wo_set_error("rank %d on device %d: injected fault (WOLOLO_FAULT_RANK)", i, d);
            rc = -1;
            break;
        }
        if (wo_dev_create(d, &r->devs[i], err, sizeof err) != 0) {
            r->devs[i] = NULL;
            wo_set_error("rank %d on device %d: %s", i, d, err);
            rc = -1;
            break;
        }
        r->ndevs = (uint32_t)i + 1u;
        if (wo_dev_enable_peer(r->devs[i], r->dev, err, sizeof err) != 0) {
            wo_set_error("rank %d on device %d: %s", i, d, err);
            rc = -1;
            break;
        }
    }
    if (rc < 0) {
        for (uint32_t i = 1; i < r->ndevs; ++i) {
            wo_dev_destroy(r->devs[i]);
            r->devs[i] = NULL;
        }
        r->ndevs = 1;
    }
    if (cur >= 0) (void)wo_dev_select(cur);
    return rc;
}

int wo_renderer_device_count(Wo_Renderer* r) { return r && r->dev ? (int)r->ndevs : 0; }

void wo_renderer_del(Wo_Renderer* r) {
    if (!r) return;
    (void)wo_renderer_finish(r);
    if (r->jit_job) (void)wo_jit_job_finish(r->jit_job, NULL, 0);
    jit_old_reap(r, 1);
    free(r->jit_want);
    if (r->ndevs > 1) (void)wo_dev_sync(r->dev); /* as in set_devices */
    for (uint32_t i = 1; i < r->ndevs; ++i) wo_dev_destroy(r->devs[i]);
    if (r->dev) wo_dev_destroy(r->dev);
    free(r->nodes);
    free(r->nonroot);
    free(r->mats);
    free(r->prog);
    free(r->name);
    free(r);
}

/* ---------------------------------------------------------------- node store */

static Wo_Node alloc_node(Wo_Renderer* r, uint32_t kind) {
    if (r->node_count >= r->max_node_count) {
        fprintf(stderr, WO_LOG_PREFIX " Failed to allocate a new renderer node -- the store holds %zu nodes.\n",
                r->max_node_count);
        wo_set_error("node store full (%zu nodes)", r->max_node_count);
        return WO_NODE_INVALID;
    }
    Wo_Node n = (Wo_Node)r->node_count++;
    memset(&r->nodes[n], 0, sizeof(WoNodeInfo));
    r->nodes[n].kind = kind;
    r->nodes[n].material = 0;
    r->dirty = 1;
    r->view_version++;
    return n;
}

static void set_nonroot(Wo_Renderer* r, Wo_Node n) {
    if (n < r->max_node_count) r->nonroot[n / 64] |= 1ull << (n % 64);
}

Wo_Node wo_renderer_add_sphere_node(Wo_Renderer* r, Wo_Scalar radius) {
    Wo_Node n = alloc_node(r, WO_NODE_SPHERE);
    if (n != WO_NODE_INVALID) r->nodes[n].radius = radius;
    return n;
}

Wo_Node wo_renderer_add_infinite_planar_partition_node(Wo_Renderer* r, Wo_Vec3 outward_facing_normal) {
    Wo_Node n = alloc_node(r, WO_NODE_HALFSPACE);
    if (n != WO_NODE_INVALID) r->nodes[n].normal = outward_facing_normal;
    return n;
}

static Wo_Node add_binop(Wo_Renderer* r, uint32_t kind, Wo_Node_Argument left, Wo_Node_Argument right) {
    if (left.node >= r->node_count || right.node >= r->node_count) {
        fprintf(stderr, WO_LOG_PREFIX " binop operand refers to an unknown node (%u, %u of %zu).\n", left.node,
                right.node, r->node_count);
        wo_set_error("binop operand refers to an unknown node");
        return WO_NODE_INVALID;
    }
    Wo_Node n = alloc_node(r, kind);
    if (n == WO_NODE_INVALID) return n;
    r->nodes[n].left = left;
    r->nodes[n].right = right;
    set_nonroot(r, left.node);
    set_nonroot(r, right.node);
    return n;
}

Wo_Node wo_renderer_add_union_of_node(Wo_Renderer* r, Wo_Node_Argument left, Wo_Node_Argument right) {
    return add_binop(r, WO_NODE_UNION, left, right);
}

Wo_Node wo_renderer_add_intersection_of_node(Wo_Renderer* r, Wo_Node_Argument left, Wo_Node_Argument right) {
    return add_binop(r, WO_NODE_INTERSECTION, left, right);
}

Wo_Node wo_renderer_add_difference_of_node(Wo_Renderer* r, Wo_Node_Argument left, Wo_Node_Argument right) {
    return add_binop(r, WO_NODE_DIFFERENCE, left, right);
}

bool wo_renderer_isroot(Wo_Renderer* r, Wo_Node node) {
    if (node >= r->max_node_count) return false;
    return (r->nonroot[node / 64] & (1ull << (node % 64))) == 0;
}

size_t wo_renderer_node_count(Wo_Renderer* r) { return r->node_count; }
char const* wo_renderer_name(Wo_Renderer* r) { return r->name; }
int wo_renderer_device(Wo_Renderer* r) { return r->device; }

/* ---------------------------------------------------------------- materials */

static Wo_Material add_material(Wo_Renderer* r, WoMaterial const* m) {
    if (r->n_mats == r->cap_mats) {
        uint32_t nc = r->cap_mats * 2u;
        WoMaterial* nm = (WoMaterial*)realloc(r->mats, nc * sizeof(WoMaterial));
        if (!nm) {
            wo_set_error("out of host memory");
            return WO_MATERIAL_INVALID;
        }
        r->mats = nm;
        r->cap_mats = nc;
    }
    r->mats[r->n_mats] = *m;
    r->dirty = 1;
    r->view_version++;
    return r->n_mats++;
}

Wo_Material wo_renderer_add_lambertian_material(Wo_Renderer* r, Wo_Vec3 albedo) {
    WoMaterial m;
    memset(&m, 0, sizeof m);
    m.kind = WO_MAT_LAMBERTIAN;
    m.albedo[0] = (float)albedo.x;
    m.albedo[1] = (float)albedo.y;
    m.albedo[2] = (float)albedo.z;
    return add_material(r, &m);
}

Wo_Material wo_renderer_add_metal_material(Wo_Renderer* r, Wo_Vec3 albedo, Wo_Scalar fuzz) {
    WoMaterial m;
    memset(&m, 0, sizeof m);
    m.kind = WO_MAT_METAL;
    m.albedo[0] = (float)albedo.x;
    m.albedo[1] = (float)albedo.y;
    m.albedo[2] = (float)albedo.z;
    m.fuzz = (float)(fuzz < 1.0 ? (fuzz > 0.0 ? fuzz : 0.0) : 1.0);
    return add_material(r, &m);
}

Wo_Material wo_renderer_add_dielectric_material(Wo_Renderer* r, Wo_Scalar refraction_index) {
    WoMaterial m;
    memset(&m, 0, sizeof m);
    m.kind = WO_MAT_DIELECTRIC;
    m.albedo[0] = m.albedo[1] = m.albedo[2] = 1.0f;
    m.ior = (float)refraction_index;
    m.inv_ior = (float)(1.0 / refraction_index);
    const double q = (1.0 - refraction_index) / (1.0 + refraction_index);
    m.r0 = (float)(q * q);
    return add_material(r, &m);
}

bool wo_renderer_set_node_material(Wo_Renderer* r, Wo_Node leaf, Wo_Material material) {
    if (leaf >= r->node_count || material >= r->n_mats) return false;
    uint32_t k = r->nodes[leaf].kind;
    if (k != WO_NODE_SPHERE && k != WO_NODE_HALFSPACE) return false;
    r->nodes[leaf].material = material;
    r->dirty = 1;
    r->view_version++;
    return true;
}

void wo_renderer_set_camera(Wo_Renderer* r, Wo_Vec3 look_from, Wo_Vec3 look_at, Wo_Vec3 view_up,
                            Wo_Scalar vertical_fov_deg, Wo_Scalar aperture, Wo_Scalar focus_dist) {
    r->camera.look_from = look_from;
    r->camera.look_at = look_at;
    r->camera.view_up = view_up;
    r->camera.vfov_deg = vertical_fov_deg;
    r->camera.aperture = aperture;
    r->camera.focus_dist = focus_dist;
    r->view_version++;
}

void wo_renderer_set_draw_params(Wo_Renderer* r, Wo_RenderParams const* params, int pin_time) {
    r->draw = *params;
    r->pin_time = pin_time;
}

/* ---------------------------------------------------------------- compile / frame */

int wo_renderer_compile(Wo_Renderer* r) {
    if (r->dirty || !r->prog) {
        char err[256] = {0};
        if (wo_compile_scene(r, err, sizeof err) != 0) {
            wo_set_error("scene compile failed: %s", err);
            return -1;
        }
    }
    return (int)r->n_recs;
}

WoRec const* wo_renderer_program(Wo_Renderer* r, uint32_t* n_recs, uint32_t* n_prims) {
    if (wo_renderer_compile(r) < 0) return NULL;
    if (n_recs) *n_recs = r->n_recs;
    if (n_prims) *n_prims = r->n_prims;
    return r->prog;
}

WoMaterial const* wo_renderer_materials(Wo_Renderer* r, uint32_t* n_materials) {
    if (n_materials) *n_materials = r->n_mats;
    return r->mats;
}

/* Host float -> the ubershader's sphere height: amplitude * sin(omega * time),
 * omega = fp32(2 * 3.1415 / 4) = 0x3fc90e56 (ubershader1.frag:101-103, folded). */
static float ubershader_sphere_y(float time_sec) {
    const float omega = 1.57075f;
    return 2.0f * sinf(omega * time_sec);
}

int wo_renderer_frame_desc(Wo_Renderer* r, Wo_RenderParams const* p, uint32_t tile_rows, uint32_t rank,
                           uint32_t nranks, WoFrame* out) {
    if (wo_renderer_compile(r) < 0) return -1;
    memset(out, 0, sizeof *out);
    out->width = p->width;
    out->height = p->height;
    out->spp = p->spp;
    out->max_depth = p->max_depth;
    out->seed = p->seed;
    out->mode = p->mode;
    out->sample_offset = p->sample_offset;
    out->tile_rows = tile_rows;
    out->rank = rank;
    out->nranks = nranks;
    if (nranks > 1u) {
        out->band_cycle = r->band_cycle;
        out->band_skip = r->band_skip;
    }
    out->n_recs = r->n_recs;
    out->n_prims = r->n_prims;
    out->time_sec = p->time_sec;
    out->sphere_y = ubershader_sphere_y(p->time_sec);
    out->inv_width = p->width ? 1.0f / (float)p->width : 0.0f;
    out->inv_height = p->height ? 1.0f / (float)p->height : 0.0f;
    wo_resolve_camera(&r->camera, p->width, p->height, &out->cam);
    return 0;
}

/* ---- background compiles of the specialised kernel ----
 * A scene edit used to stall draw_frame for the hiprtc compile (csg32 ~1 s, csg256
 * ~4 s on the box).  draw_frame now starts the compile on a host thread when the
 * code object is in neither cache and renders with the interpreter (the same
 * image bit for bit) until it has ended; the next frame after that loads it.
 * Batch renders (render_f32, render_rows_device, ...) wait for it instead. */

static void jit_old_reap(Wo_Renderer* r, int wait) {
    uint32_t k = 0;
    for (uint32_t i = 0; i < r->n_jit_old; ++i) {
        if (wait || wo_jit_job_done(r->jit_old[i]))
            (void)wo_jit_job_finish(r->jit_old[i], NULL, 0); /* an edited scene's object: cached, unused */
        else
            r->jit_old[k++] = r->jit_old[i];
    }
    r->n_jit_old = k;
}

/* Load the current scene's specialised kernel on every rank once its background
 * compile has ended (`wait`: wait for it). */
static void jit_job_poll(Wo_Renderer* r, int wait) {
    jit_old_reap(r, 0);
    if (!r->jit_job || (!wait && !wo_jit_job_done(r->jit_job))) return;
    char err[512] = {0};
    const int rc = wo_jit_job_finish(r->jit_job, err, sizeof err);
    r->jit_job = NULL;
    char* src = r->jit_want;
    r->jit_want = NULL;
    if (rc) {
        fprintf(stderr, WO_LOG_PREFIX " scene specialisation failed (%s); using the %s\n", err,
                r->lanes_loaded ? "lane tracer" : "interpreter kernel");
    } else if (src && !r->dev_stale) {
        const int cur = r->ndevs > 1 ? wo_dev_current() : -1;
        int ok = 1;
        for (uint32_t i = 0; i < r->ndevs && ok; ++i) /* the process cache has it now */
            if (wo_dev_set_jit(r->devs[i], src, err, sizeof err) != 0) {
                fprintf(stderr, WO_LOG_PREFIX " loading the specialised kernel failed (%s)\n", err);
                ok = 0;
            }
        if (!ok)
            for (uint32_t i = 0; i < r->ndevs; ++i) (void)wo_dev_set_jit(r->devs[i], NULL, err, sizeof err);
        r->jit_loaded = ok;
        if (ok && r->lanes_loaded) { /* the lanes ran while it compiled (sync_device_ex) */
            for (uint32_t i = 0; i < r->ndevs; ++i) wo_dev_set_lanes(r->devs[i], 0);
            r->lanes_loaded = 0;
        }
        if (cur >= 0) (void)wo_dev_select(cur);
    }
    free(src);
}

/* The compile in flight belongs to an edited scene: let it finish on its own. */
static void jit_job_orphan(Wo_Renderer* r) {
    if (!r->jit_job) return;
    if (r->n_jit_old == sizeof r->jit_old / sizeof r->jit_old[0]) jit_old_reap(r, 1);
    r->jit_old[r->n_jit_old++] = r->jit_job;
    r->jit_job = NULL;
    free(r->jit_want);
    r->jit_want = NULL;
}

int wo_renderer_jit_pending(Wo_Renderer* r) { return r && r->jit_job ? 1 : 0; }

/* `may_defer`: the caller renders with the interpreter rather than wait for a
 * compile (draw_frame). */
static int sync_device_ex(Wo_Renderer* r, int may_defer) {
    if (!r->dev) {
        wo_set_error("renderer has no HIP device (created with WOLOLO_ALLOW_NO_DEVICE)");
        fprintf(stderr, WO_LOG_PREFIX " render called on a device-less renderer.\n");
        return -1;
    }
    if (wo_renderer_compile(r) < 0) return -1;
    /* a batch render waits for a pending compile unless the lanes render meanwhile
     * (AUTO; an explicit WO_TRACER_JIT asks for the specialised kernel itself) */
    if (!r->dev_stale) jit_job_poll(r, !may_defer && !(r->lanes_loaded && r->tracer == WO_TRACER_AUTO));
    if (r->dev_stale) {
        jit_job_orphan(r);
        char err[256] = {0};
        /* The pipeline may still hold a frame of the old scene on the device
         * stream (draw_frame returns with one in flight): retire it first, so it
         * is presented in order and finishes before its program, traversal table
         * and kernel module are replaced.  wo_dev_upload_scene then drains every
         * other stream of the device (render_rows_device on a caller's stream). */
        if (wo_renderer_finish(r)) return -1;
        const int cur = r->ndevs > 1 ? wo_dev_current() : -1;
        for (uint32_t i = 0; i < r->ndevs; ++i) {
            if (wo_dev_upload_scene(r->devs[i], r->prog, r->n_recs, r->n_prims, r->mats, r->n_mats, err,
                                    sizeof err)) {
                wo_set_error("scene upload failed (rank %u): %s", i, err);
                if (cur >= 0) (void)wo_dev_select(cur); /* the caller's device, on every exit */
                return -1;
            }
        }
        r->dev_stale = 0;
        r->jit_loaded = 0;
        r->lanes_loaded = 0;
        /* lanes only where the specialised kernel is not built: on union-only scenes it
         * wins up to 128 primitives at least (csg256_balanced_union 16.2 vs 24.8 ms) */
        uint32_t max_prims = 256, lanes_min = 256;
        const char* mp = getenv("WOLOLO_JIT_MAX_PRIMS");
        if (mp && *mp) max_prims = (uint32_t)strtoul(mp, NULL, 10);
        const char* lm = getenv("WOLOLO_LANES_MIN_PRIMS");
        if (lm && *lm) lanes_min = (uint32_t)strtoul(lm, NULL, 10);
        int lanes_ok = wo_dev_lanes_available(r->dev);
        /* an explicit JIT request on a scene above max_prims takes the lanes too
         * (faster than the interpreter wherever they apply) */
        int want_lanes = lanes_ok && (r->tracer == WO_TRACER_LANES ||
                                      (r->tracer == WO_TRACER_AUTO && r->n_prims > lanes_min) ||
                                      (r->tracer == WO_TRACER_JIT && r->n_prims > max_prims));
        /* A general tree above max_prims whose root the levelled truth tables
         * evaluate (scene_jit.c hlut_plan; not a union of terms or of primitives,
         * which the lane tracer's union count and term mode take): the specialised
         * kernel, with the lanes only while it compiles in the background
         * (csg360_nested 201.6 ms against the lanes' general walk, 324.4).
         * WOLOLO_JIT_GENERAL=0 keeps such scenes on the lanes. */
        char* pre_src = NULL;
        const char* jg = getenv("WOLOLO_JIT_GENERAL");
        if (r->tracer != WO_TRACER_INTERPRETER && r->tracer != WO_TRACER_LANES && r->n_prims > max_prims &&
            r->n_prims <= 1023u && !(jg && strcmp(jg, "0") == 0)) {
            pre_src = wo_generate_jit_source(r->prog, r->n_recs, r->n_prims);
            if (pre_src && !strstr(pre_src, "#define WO_JIT_HLUT 1\n")) {
                free(pre_src);
                pre_src = NULL;
            }
        }
        const int lanes_meanwhile = pre_src != NULL && want_lanes;
        if (pre_src) want_lanes = 0;
        int want_jit = !want_lanes && r->tracer != WO_TRACER_INTERPRETER && r->n_prims > 0 &&
                       (r->n_prims <= max_prims || pre_src != NULL);
        for (uint32_t i = 0; i < r->ndevs; ++i) wo_dev_set_lanes(r->devs[i], want_lanes);
        r->lanes_loaded = want_lanes;
        int deferred = 0;
        if (want_jit) {
            char* src = pre_src ? pre_src : wo_generate_jit_source(r->prog, r->n_recs, r->n_prims);
            pre_src = NULL;
            if (!src) {
                fprintf(stderr, WO_LOG_PREFIX " scene specialisation: source generation failed; using the interpreter\n");
            } else if ((may_defer || (lanes_meanwhile && r->tracer == WO_TRACER_AUTO)) && !wo_dev_jit_cached(r->dev, src) &&
                       (r->jit_job = wo_jit_job_start(r->dev, src))) {
                /* A batch render of such a scene (AUTO) does not wait for the 1-2 minute
                 * compile of a big general tree either: the lanes render it meanwhile,
                 * the same image bit for bit (wo_renderer_prepare waits for the kernel). */
                r->jit_want = src; /* compiling in the background; the interpreter (or the lanes) meanwhile */
                src = NULL;
                deferred = 1;
                if (lanes_meanwhile) { /* a loaded specialised kernel takes precedence (wo_dev_launch_ex) */
                    for (uint32_t i = 0; i < r->ndevs; ++i) wo_dev_set_lanes(r->devs[i], 1);
                    r->lanes_loaded = 1;
                }
            } else {
                /* compiled once (code-object cache), loaded on every rank's device */
                int ok = 1;
                for (uint32_t i = 0; i < r->ndevs && ok; ++i) {
                    if (wo_dev_set_jit(r->devs[i], src, err, sizeof err) != 0) {
                        fprintf(stderr, WO_LOG_PREFIX " scene specialisation failed (%s); using the %s\n", err,
                                lanes_meanwhile ? "lane tracer" : "interpreter kernel");
                        ok = 0;
                    }
                }
                r->jit_loaded = ok;
                if (!ok && lanes_meanwhile) { /* the lanes this scene qualified for, not the interpreter */
                    for (uint32_t i = 0; i < r->ndevs; ++i) wo_dev_set_lanes(r->devs[i], 1);
                    r->lanes_loaded = 1;
                }
            }
            free(src);
        }
        if (!r->jit_loaded)
            for (uint32_t i = 0; i < r->ndevs; ++i) (void)wo_dev_set_jit(r->devs[i], NULL, err, sizeof err);
        if (cur >= 0) (void)wo_dev_select(cur);
        (void)deferred;
    }
    return 0;
}

static int sync_device(Wo_Renderer* r) { return sync_device_ex(r, 0); }

int wo_renderer_prepare(Wo_Renderer* r) {
    if (!r) return -1;
    if (sync_device(r)) return -1;
    const int cur = r->ndevs > 1 ? wo_dev_current() : -1;
    jit_job_poll(r, 1);
    if (cur >= 0) (void)wo_dev_select(cur);
    return 0;
}

void wo_renderer_set_tracer(Wo_Renderer* r, Wo_Tracer tracer) {
    if (r->tracer != (int)tracer) {
        r->tracer = (int)tracer;
        r->dev_stale = 1;
    }
}

void wo_renderer_set_jit(Wo_Renderer* r, int mode) {
    wo_renderer_set_tracer(r, mode ? WO_TRACER_AUTO : WO_TRACER_INTERPRETER);
}

char* wo_renderer_jit_source(Wo_Renderer* r) {
    if (wo_renderer_compile(r) < 0 || r->n_prims == 0) return NULL;
    return wo_generate_jit_source(r->prog, r->n_recs, r->n_prims);
}

void wo_free(void* p) { free(p); }

int wo_renderer_jit_info(Wo_Renderer* r, double* seconds) {
    if (!r || !r->dev || !r->jit_loaded) return -1;
    return wo_dev_jit_origin(r->dev, seconds);
}

int wo_renderer_lanes_info(Wo_Renderer* r, uint32_t* out) {
    if (!r || !r->dev || !r->lanes_loaded || !out) return -1;
    return wo_dev_lanes_info(r->dev, out);
}

int wo_renderer_kernel_info(Wo_Renderer* r, char* key_hex, uint32_t* out) {
    if (!r || !r->dev || !out) return -1;
    return wo_dev_kernel_info(r->dev, key_hex, out);
}

char const* wo_renderer_trace_path(Wo_Renderer* r) {
    if (!r->dev) return "none";
    return r->jit_loaded ? "jit" : r->lanes_loaded ? "lanes" : "interpreter";
}

static int render_sync(Wo_Renderer* r, Wo_RenderParams const* params, float* out_rgba, int accumulate, int reset);

int wo_renderer_render_f32(Wo_Renderer* r, Wo_RenderParams const* params, float* out_rgba) {
    if (r && r->dev && frame_ranks(r, params) > 1u) return render_sync(r, params, out_rgba, 0, 0) < 0 ? -1 : 0;
    if (sync_device(r)) return -1;
    WoFrame fr;
    if (wo_renderer_frame_desc(r, params, 16, 0, 1, &fr)) return -1;
    char err[256] = {0};
    if (wo_dev_render_host(r->dev, &fr, out_rgba, err, sizeof err)) {
        wo_set_error("render failed: %s", err);
        return -1;
    }
    return 0;
}

int wo_renderer_render_rows_device(Wo_Renderer* r, Wo_RenderParams const* params, void* d_out, uint32_t tile_rows,
                                   uint32_t rank, uint32_t nranks, void* stream,
                                   unsigned long long* d_segment_counter) {
    if (sync_device(r)) return -1;
    WoFrame fr;
    if (wo_renderer_frame_desc(r, params, tile_rows, rank, nranks, &fr)) return -1;
    char err[256] = {0};
    if (wo_dev_launch(r->dev, &fr, d_out, stream, d_segment_counter, err, sizeof err)) {
        wo_set_error("launch failed: %s", err);
        return -1;
    }
    return 0;
}

int wo_renderer_count_work(Wo_Renderer* r, Wo_RenderParams const* params, uint32_t tile_rows, uint32_t rank,
                           uint32_t nranks, unsigned long long* counts) {
    if (sync_device(r)) return -1;
    WoFrame fr;
    if (wo_renderer_frame_desc(r, params, tile_rows, rank, nranks, &fr)) return -1;
    char err[256] = {0};
    if (wo_dev_count_work(r->dev, &fr, counts, err, sizeof err)) {
        wo_set_error("counting launch failed: %s", err);
        return -1;
    }
    return 0;
}

int wo_assemble_rows_device_ex(void const* d_gathered, void* d_frame, uint32_t width, uint32_t height,
                               uint32_t tile_rows, uint32_t nranks, uint32_t band_cycle, uint32_t band_skip,
                               void* stream) {
    char err[256] = {0};
    if (wo_dev_assemble(d_gathered, d_frame, width, height, tile_rows, nranks, band_cycle, band_skip, stream, err,
                        sizeof err)) {
        wo_set_error("%s", err);
        return -1;
    }
    return 0;
}

int wo_assemble_rows_device(void const* d_gathered, void* d_frame, uint32_t width, uint32_t height,
                            uint32_t tile_rows, uint32_t nranks, void* stream) {
    return wo_assemble_rows_device_ex(d_gathered, d_frame, width, height, tile_rows, nranks, 0u, 0u, stream);
}

int wo_renderer_set_band_weight(Wo_Renderer* r, uint32_t band_cycle, uint32_t band_skip) {
    if (!r) return -1;
    if (band_skip != 0u && band_skip >= band_cycle) {
        wo_set_error("band weight: skip %u must be below the cycle %u (or 0)", band_skip, band_cycle);
        return -1;
    }
    /* the band arithmetic forms cycle * nranks (<= 16 ranks) in 32 bits */
    if (band_skip != 0u && band_cycle > WO_BAND_CYCLE_MAX) {
        wo_set_error("band weight: cycle %u exceeds %u", band_cycle, (unsigned)WO_BAND_CYCLE_MAX);
        return -1;
    }
    r->band_cycle = band_skip ? band_cycle : 0u;
    r->band_skip = band_skip;
    return 0;
}

/* ---------------------------------------------------------------- draw_frame */

/* Present a finished frame: keep it (float and its B8G8R8A8 sRGB encode, made
 * on the GPU: present.c) as the last frame, and dump it as a binary PPM when
 * WOLOLO_OUTPUT names a file (the headless stand-in for the swapchain,
 * ref renderer.c:2160-2211). */
static void present(Wo_Renderer* r, int slot, float const* px, uint32_t const* bgra8, uint32_t w, uint32_t h) {
    r->last_slot = slot;
    if (r->stamps && r->n_stamps < sizeof r->stamp_log / sizeof r->stamp_log[0] &&
        wo_dev_slot_stamps(r->dev, slot, r->stamp_log[r->n_stamps]) == 0)
        r->n_stamps++;
    r->last_frame = px;
    r->last_bgra8 = bgra8;
    r->last_w = w;
    r->last_h = h;
    r->frames_drawn++;
    const char* out = getenv("WOLOLO_OUTPUT");
    if (out && *out && bgra8 && wo_write_ppm_bgra8(out, bgra8, w, h))
        fprintf(stderr, WO_LOG_PREFIX " present: %s\n", wo_renderer_last_error());
}

static int retire_slot(Wo_Renderer* r, int slot) {
    if (!r->pending[slot]) return 0;
    char err[256] = {0};
    float const* px = NULL;
    uint32_t const* bgra8 = NULL;
    r->pending[slot] = 0;
    if (wo_dev_frame_wait(r->dev, slot, &px, &bgra8, err, sizeof err)) {
        wo_set_error("frame wait failed: %s", err);
        return -1;
    }
    present(r, slot, px, bgra8, r->pend_w[slot], r->pend_h[slot]);
    return 0;
}

int wo_renderer_finish(Wo_Renderer* r) {
    if (!r || !r->dev) return 0;
    /* oldest first: the slot not used by the newest submission */
    int newest = (int)((r->frame_seq + 1u) & 1u);
    int rc = retire_slot(r, newest ^ 1);
    if (retire_slot(r, newest)) rc = -1;
    return rc;
}

/* Accumulation bookkeeping shared by draw_frame and render_accumulate: whether
 * this frame continues the accumulation, its sample offset and the total. */
static int acc_continues(Wo_Renderer* r, Wo_RenderParams const* p, uint32_t nranks) {
    Wo_RenderParams a = r->acc_params;
    return r->acc_valid && r->acc_view == r->view_version && r->acc_ranks == nranks && a.width == p->width &&
           a.height == p->height &&
           a.spp == p->spp && a.max_depth == p->max_depth && a.seed == p->seed && a.mode == p->mode &&
           a.sample_offset == p->sample_offset;
}

static int submit_frame(Wo_Renderer* r, Wo_RenderParams p, int slot, int accumulate, int reset) {
    char err[256] = {0};
    long long* d_acc[WO_MAX_DEVICES] = {NULL};
    int acc = 0;
    uint32_t total = 0;
    const uint32_t nr = frame_ranks(r, &p);
    if (accumulate && p.mode == WO_SHADING_PATHTRACE) {
        int cont = !reset && acc_continues(r, &p, nr);
        if (!cont) {
            r->acc_params = p;
            r->acc_view = r->view_version;
            r->acc_ranks = nr;
            r->acc_spp = 0;
            r->acc_valid = 1;
        }
        for (uint32_t i = 0; i < nr; ++i) {
            if (wo_dev_accum_prepare(r->devs[i], p.width, p.height, 4, nr, !cont, &d_acc[i], err, sizeof err)) {
                wo_set_error("accumulation buffer (rank %u): %s", i, err);
                return -1;
            }
        }
        acc = 1;
        uint64_t t = (uint64_t)r->acc_spp + p.spp;
        if (t > 0xFFFFFFFFull) {
            wo_set_error("accumulated samples overflow");
            return -1;
        }
        p.sample_offset = r->acc_params.sample_offset + r->acc_spp;
        total = (uint32_t)t;
        r->acc_spp = total;
    }
    WoFrame fr;
    if (wo_renderer_frame_desc(r, &p, 4, 0, nr, &fr)) return -1;
    const int cur = r->ndevs > 1 ? wo_dev_current() : -1;
    /* the synchronous render hands its float frame back; a presented frame maps
     * back its present encode, and the float pixels only on request */
    const int map_float = slot == WO_SLOT_SYNC || r->map_float;
    int rc = wo_dev_frame_submit_ranks(r->devs, nr, &fr, slot, acc ? d_acc : NULL, total, map_float, err, sizeof err);
    if (cur >= 0) (void)wo_dev_select(cur);
    if (rc) {
        wo_set_error("frame submit failed: %s", err);
        return -1;
    }
    if (slot <= WO_SLOT_PIPE1) {
        r->pending[slot] = 1;
        r->pend_w[slot] = p.width;
        r->pend_h[slot] = p.height;
    }
    return 0;
}

/* Reference draw_frame_with_renderer (renderer.c:2085-2219) waits for the queue
 * every frame (vkQueueWaitIdle, 2212).  Here frame k is submitted (render + copy
 * to pinned host memory, asynchronous) and then frame k-1 is waited for and
 * presented, so the GPU renders frame k while the host presents k-1. */
void wo_renderer_draw_frame(Wo_Renderer* r) {
    if (!r) return;
    Wo_RenderParams p = r->draw;
    if (!r->pin_time) p.time_sec = (float)(r->app ? wo_app_time_sec(r->app) : wo_monotonic_sec() - r->t0);
    if (sync_device_ex(r, r->jit_async)) {
        fprintf(stderr, WO_LOG_PREFIX " draw_frame failed: %s\n", wo_renderer_last_error());
        return;
    }
    int slot = (int)(r->frame_seq & 1u);
    if (retire_slot(r, slot) == 0 && submit_frame(r, p, slot, r->progressive, 0) == 0) {
        r->frame_seq++;
        if (retire_slot(r, slot ^ 1) == 0) return;
    }
    fprintf(stderr, WO_LOG_PREFIX " draw_frame failed: %s\n", wo_renderer_last_error());
}

void wo_renderer_set_progressive(Wo_Renderer* r, int on) {
    r->progressive = on != 0;
    if (!on) r->acc_valid = 0;
}

uint32_t wo_renderer_accumulated_spp(Wo_Renderer* r) { return r->acc_valid ? r->acc_spp : 0u; }

/* The presented frame's float pixels are mapped back when asked for: its slot
 * keeps the device frame until the next draw_frame submits into it. */
float const* wo_renderer_last_frame(Wo_Renderer* r, uint32_t* width, uint32_t* height) {
    if (!r->last_frame && r->last_bgra8 && r->dev && r->last_slot >= 0) {
        char err[256] = {0};
        float const* px = NULL;
        const int cur = wo_dev_current(); /* the map selects the root's device: restore the caller's */
        if (wo_dev_frame_map_float(r->dev, r->last_slot, &px, err, sizeof err) == 0)
            r->last_frame = px;
        else
            wo_set_error("last frame: %s", err);
        if (cur >= 0) (void)wo_dev_select(cur);
    }
    if (width) *width = r->last_frame ? r->last_w : 0u;
    if (height) *height = r->last_frame ? r->last_h : 0u;
    return r->last_frame;
}

uint32_t const* wo_renderer_last_frame_bgra8(Wo_Renderer* r, uint32_t* width, uint32_t* height) {
    if (width) *width = r->last_bgra8 ? r->last_w : 0u;
    if (height) *height = r->last_bgra8 ? r->last_h : 0u;
    return r->last_bgra8;
}

void wo_renderer_set_map_float(Wo_Renderer* r, int every_frame) {
    if (r) r->map_float = every_frame != 0;
}

int wo_renderer_set_frame_stamps(Wo_Renderer* r, int on) {
    if (!r || !r->dev) return -1;
    if (wo_renderer_finish(r)) return -1;
    char err[256] = {0};
    if (wo_dev_set_stamps(r->dev, on, err, sizeof err)) {
        wo_set_error("%s", err);
        return -1;
    }
    r->stamps = on != 0;
    r->n_stamps = 0;
    return 0;
}

int wo_renderer_frame_stamps(Wo_Renderer* r, double* out, int max_frames) {
    if (!r || !out || max_frames < 0) return -1;
    uint32_t n = r->n_stamps < (uint32_t)max_frames ? r->n_stamps : (uint32_t)max_frames;
    memcpy(out, r->stamp_log, (size_t)n * sizeof r->stamp_log[0]);
    r->n_stamps = 0;
    return (int)n;
}

int wo_srgb8_encode_device(void const* d_rgba, void* d_bgra8, size_t pixels, void* stream) {
    char err[256] = {0};
    if (wo_dev_srgb8(d_rgba, d_bgra8, pixels, stream, err, sizeof err)) {
        wo_set_error("%s", err);
        return -1;
    }
    return 0;
}

int wo_renderer_render_accumulate(Wo_Renderer* r, Wo_RenderParams const* params, float* out_rgba, int reset) {
    if (params->mode != WO_SHADING_PATHTRACE) {
        wo_set_error("render_accumulate needs WO_SHADING_PATHTRACE");
        return -1;
    }
    return render_sync(r, params, out_rgba, 1, reset);
}

/* One frame through the scratch slot (every rank), waited for.  Not presented:
 * wo_renderer_last_frame keeps pointing at the last presented frame, whose
 * pipeline slot this does not touch. */
static int render_sync(Wo_Renderer* r, Wo_RenderParams const* params, float* out_rgba, int accumulate, int reset) {
    if (wo_renderer_finish(r)) return -1; /* the pipeline's frames first (in order) */
    if (sync_device(r)) return -1;
    if (submit_frame(r, *params, WO_SLOT_SYNC, accumulate, reset)) return -1;
    char err[256] = {0};
    float const* px = NULL;
    if (wo_dev_frame_wait(r->dev, WO_SLOT_SYNC, &px, NULL, err, sizeof err)) {
        wo_set_error("frame wait failed: %s", err);
        return -1;
    }
    if (out_rgba) memcpy(out_rgba, px, (size_t)params->width * params->height * 4u * sizeof(float));
    return accumulate ? (int)r->acc_spp : 0;
}

/* ---------------------------------------------------------------- device frames */

int wo_renderer_render_frame_device(Wo_Renderer* r, Wo_RenderParams const* params, void* d_frame, void* stream) {
    if (!r || !params) return -1;
    if (sync_device(r)) return -1;
    const uint32_t nr = frame_ranks(r, params);
    WoFrame fr;
    if (wo_renderer_frame_desc(r, params, 4, 0, nr, &fr)) return -1;
    const int slot = (r->dframe_seq & 1u) ? WO_SLOT_DEV1 : WO_SLOT_DEV0;
    const int cur = r->ndevs > 1 ? wo_dev_current() : -1;
    char err[256] = {0};
    int rc = wo_dev_frame_ranks_device(r->devs, nr, &fr, slot, d_frame, stream, err, sizeof err);
    if (cur >= 0) (void)wo_dev_select(cur);
    if (rc) {
        wo_set_error("device frame failed: %s", err);
        return -1;
    }
    r->dframe_seq++;
    return 0;
}

int wo_renderer_take_segments(Wo_Renderer* r, unsigned long long* total) {
    if (!r || !r->dev || !total) return -1;
    *total = 0;
    const int cur = wo_dev_current();
    char err[256] = {0};
    int rc = 0;
    for (uint32_t i = 0; i < r->ndevs; ++i) {
        unsigned long long t = 0;
        if (wo_dev_take_segments(r->devs[i], &t, err, sizeof err)) {
            wo_set_error("rank %u: %s", i, err);
            rc = -1;
            break;
        }
        *total += t;
    }
    if (cur >= 0) (void)wo_dev_select(cur);
    return rc;
}

void wo_renderer_set_jit_async(Wo_Renderer* r, int on) {
    if (r) r->jit_async = on != 0;
}
