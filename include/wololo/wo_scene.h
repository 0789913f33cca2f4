/*
 * wololo/wo_scene.h -- the flattened scene ("CSG program") and per-frame
 * parameters as they sit in HBM / LDS.  This is a DATA contract: the host scene
 * compiler (csgrenderer_amd/csrc/scene_compile.c) writes it, the HIP kernels
 * (csrc/trace_kernels.hip) and the CPU oracle (oracle/oracle.c) read it.
 *
 * The reference never ships its node tables to the GPU: its
 * host tables are NodeType + NodeInfo (renderer.c:180-202).  Here they are
 * compiled into a postfix program over convex primitives:
 *
 *   WO_OP_PRIM   one convex primitive = intersection of `u0` member leaves,
 *                followed by exactly u0 WoRec leaf records (WO_LEAF_*).
 *                u1 = primitive ordinal (postfix order, dense from 0).
 *   WO_OP_UNION / _INTER / _DIFF / _RDIFF   pop B (top), pop A, push
 *                A|B, A&B, A&~B, B&~A.  (RDIFF lets the compiler emit the
 *                subtrahend first to keep the evaluation stack shallow.)
 *   WO_OP_BOUND  conservative bounding sphere (f[0..2] centre, f[3] R^2,
 *                f[4] R) of the subtree that starts at the next record and
 *                ends at record u0-1; u1 = leaves in that subtree.  A kernel MAY
 *                skip that subtree (value = empty set) when no ray of interest
 *                can touch the sphere; an evaluator that ignores BOUND (all of
 *                them, or the small ones) gets identical results.
 *
 * Every record is 32 bytes (8 dwords) so a wave reads one with two 16-byte
 * LDS broadcasts or one scalar s_load_dwordx8.
 */
#ifndef WOLOLO_WO_SCENE_H
#define WOLOLO_WO_SCENE_H

#if defined(__HIPCC_RTC__) /* hiprtc: no libc headers; take its internal fixed-width types */
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::uint64_t uint64_t;
#else
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

enum {
    WO_OP_PRIM = 1,
    WO_OP_UNION = 2,
    WO_OP_INTER = 3,
    WO_OP_DIFF = 4,
    WO_OP_RDIFF = 5,
    WO_OP_BOUND = 6,
};

enum {
    WO_LEAF_SPHERE = 16,     /* f: cx cy cz r^2 1/r */
    WO_LEAF_HALFSPACE = 17,  /* f: nx ny nz h   ({x : n.x <= h}, |n| = 1);
                              * u1 = 1 + a when n is exactly s*e_a (s = +-1, a = 0,1,2
                              * for x,y,z), else 0.  Such a half-space is intersected
                              * as t = (h - s*o_a) * (s * (1/d_a)), the reciprocal taken
                              * once per ray, instead of (h - n.o) / (n.d). */
};

typedef struct WoRec {
    uint32_t op;   /* WO_OP_* or WO_LEAF_* */
    uint32_t u0;   /* PRIM: member count; BOUND: skip target; leaf: material id */
    uint32_t u1;   /* PRIM: primitive ordinal */
    float f[5];
} WoRec;

enum {
    WO_MAT_LAMBERTIAN = 0,
    WO_MAT_METAL = 1,
    WO_MAT_DIELECTRIC = 2,
};

typedef struct WoMaterial {
    uint32_t kind;
    float albedo[3];
    float fuzz;   /* metal */
    float ior;    /* dielectric refraction index */
    float inv_ior; /* dielectric: 1/ior, rounded from double on the host */
    float r0;      /* dielectric: Schlick's ((1-ior)/(1+ior))^2, rounded from double on the host */
} WoMaterial;

/* Shading modes (Wo_ShadingMode in renderer_ext.h uses the same values). */
enum {
    WO_MODE_UBERSHADER_RT1 = 0, /* reference ubershader1.frag ep_rt1_1 (animated sphere) */
    WO_MODE_DEBUG_ST = 1,       /* reference ep_debug_view_1: (st.x, st.y, 0, 1) */
    WO_MODE_PATHTRACE = 2,      /* CSG scene, materials, spp, bounces */
    WO_MODE_NORMALS = 3,        /* CSG scene, 1 primary ray at the pixel centre, 0.5*(n+1) */
};

/* Camera already resolved to floats for one frame size (RTIOW camera model). */
typedef struct WoCamera {
    float origin[3];
    float lower_left[3];
    float horizontal[3];
    float vertical[3];
    float u[3];
    float v[3];
    float lens_radius;
    float pad[3];
} WoCamera;

typedef struct WoFrame {
    uint32_t width, height;     /* full frame */
    uint32_t spp;               /* samples per pixel */
    uint32_t max_depth;         /* max traced segments per path */
    uint32_t seed;              /* frame seed */
    uint32_t mode;              /* WO_MODE_* */
    uint32_t sample_offset;     /* first sample index */
    uint32_t tile_rows;         /* row-cyclic tiling: tile height in rows */
    uint32_t rank, nranks;      /* this device renders row bands (tiles) of the frame: wo_band_global */
    uint32_t n_recs;            /* program length */
    uint32_t n_prims;           /* primitive count */
    float time_sec;             /* ubershader: UBO time_since_start_sec */
    float sphere_y;             /* ubershader: 2*sin(omega*time), hoisted to the host */
    float inv_width, inv_height; /* path tracer: 1/width, 1/height (fp32); sample position = (x + jitter) * inv_width */
    WoCamera cam;
    uint32_t band_cycle;        /* band weighting: in every band_cycle rounds of the ranks, rank 0 */
    uint32_t band_skip;         /* sits out band_skip rounds (0: every rank takes one band per round) */
} WoFrame;

/* Executed-work counters of a counting launch (wo_renderer_count_work): lane
 * counts of what the path kernels actually ran, for the executed-work roofline
 * (SURVEY.md 8(d) prices each kind). */
enum {
    WO_WORK_SEGMENTS = 0,        /* traced ray segments */
    WO_WORK_SPHERE_TESTS = 1,    /* ray-sphere leaf intersections */
    WO_WORK_HALFSPACE_TESTS = 2, /* ray-half-space leaf intersections */
    WO_WORK_BOUND_TESTS = 3,     /* bounding-sphere (BOUND) tests */
    WO_WORK_EVENTS = 4,          /* boundary events stored in the event window */
    WO_WORK_SWEEP_STEPS = 5,     /* events swept (membership toggle + root evaluation) */
    WO_WORK_RECOLLECTS = 6,      /* re-collect passes after a window overflow */
    WO_WORK_PRIMARY = 7,         /* segments that are primary (camera) rays */
    /* wave cycles per section of the path loop, summed over waves: only in a
     * counting build with -DWO_TIME_SECTIONS=1 (WOLOLO_JIT_FLAGS), else 0 */
    WO_WORK_CYC_TAKE = 8,        /* job queue + sample set-up */
    WO_WORK_CYC_COLLECT = 9,     /* trace: first pass (culling, intervals, events) */
    WO_WORK_CYC_SWEEP = 10,      /* trace: sweep + re-collects */
    WO_WORK_CYC_SHADE = 11,      /* hit shading, scatter, accumulation */
    WO_WORK_CYC_LOOP = 12,       /* whole loop iterations */
    /* lane occupancy (counting launches): */
    WO_WORK_IDLE_LANES = 13,     /* loop iterations of a lane with no path (queue drained) */
    WO_WORK_SWEEP_TRIPS = 14,    /* sweep loop trips of a wave (64 lane slots each) */
    WO_WORK_CYC_CAM = 15,        /* wave cycles of camera-ray iterations (WO_TIME_SECTIONS) */
    WO_WORK_KINDS = 16
};

/* Minimum ray parameter for every CSG segment (RTIOW's 0.001). */
#define WO_T_MIN (1.0e-3f)

/* Row bands of tile_rows frame rows go to the ranks in rounds: band g of a plain
 * partition (skip = 0) is rank g % n's local band g / n.  With weighting (0 < skip
 * < cycle, n >= 2), every cycle of `cycle` rounds holds cycle * n - skip bands:
 * rounds [0, cycle - skip) give one band to every rank in rank order, the last
 * `skip` rounds one to every rank but 0 -- rank 0, which also gathers, assembles
 * and presents the frame, renders (cycle - skip) / cycle of another rank's share.
 * (Mirrored by wo_device_common.h local_to_global_row and wololo.py global_row.) */
/* cycles longer than this are not weighted (cycle * n stays far inside 32 bits) */
#define WO_BAND_CYCLE_MAX 65536u
static inline int wo_band_weighted(uint32_t n, uint32_t cycle, uint32_t skip) {
    return n >= 2u && skip > 0u && skip < cycle && cycle <= WO_BAND_CYCLE_MAX;
}
/* the frame band of rank `rank`'s local band lb */
static inline uint32_t wo_band_global(uint32_t lb, uint32_t rank, uint32_t n, uint32_t cycle, uint32_t skip) {
    if (!wo_band_weighted(n, cycle, skip)) return lb * n + rank;
    const uint32_t full = cycle - skip, per = rank == 0u ? full : cycle;
    const uint32_t c = lb / per, j = lb - c * per;
    const uint32_t p = j < full ? j * n + rank : full * n + (j - full) * (n - 1u) + rank - 1u;
    return c * (cycle * n - skip) + p;
}
/* the rank and local band of frame band g */
static inline void wo_band_local(uint32_t g, uint32_t n, uint32_t cycle, uint32_t skip, uint32_t* rank,
                                 uint32_t* lb) {
    if (!wo_band_weighted(n, cycle, skip)) {
        *rank = g % n;
        *lb = g / n;
        return;
    }
    const uint32_t full = cycle - skip, len = cycle * n - skip, c = g / len, p = g - c * len;
    if (p < full * n) {
        const uint32_t j = p / n, r = p - j * n;
        *rank = r;
        *lb = c * (r == 0u ? full : cycle) + j;
    } else {
        const uint32_t q = p - full * n, j = full + q / (n - 1u), r = 1u + q % (n - 1u);
        *rank = r;
        *lb = c * cycle + j;
    }
}
/* Number of bands (tile rows) a rank owns for a frame of `height` rows. */
static inline uint32_t wo_rank_tile_count_ex(uint32_t height, uint32_t tile_rows, uint32_t rank, uint32_t nranks,
                                             uint32_t cycle, uint32_t skip) {
    const uint32_t tiles = (height + tile_rows - 1u) / tile_rows;
    if (!wo_band_weighted(nranks, cycle, skip)) return rank < tiles ? (tiles - rank + nranks - 1u) / nranks : 0u;
    const uint32_t full = cycle - skip, per = rank == 0u ? full : cycle, len = cycle * nranks - skip;
    const uint32_t c = tiles / len, rem = tiles - c * len;
    uint32_t cnt = c * per;
    for (uint32_t j = 0; j < per; ++j) cnt += wo_band_global(j, rank, nranks, cycle, skip) < rem ? 1u : 0u;
    return cnt;
}
static inline uint32_t wo_rank_tile_count(uint32_t height, uint32_t tile_rows, uint32_t rank, uint32_t nranks) {
    return wo_rank_tile_count_ex(height, tile_rows, rank, nranks, 0u, 0u);
}

/* Rows in one rank's local (gather) buffer: the same for every rank, the most any
 * rank owns (rank 0 or 1: a rank owns no more bands than a lower one but 0). */
static inline uint32_t wo_rank_local_rows_ex(uint32_t height, uint32_t tile_rows, uint32_t nranks, uint32_t cycle,
                                             uint32_t skip) {
    const uint32_t t0 = wo_rank_tile_count_ex(height, tile_rows, 0u, nranks, cycle, skip);
    const uint32_t t1 = nranks > 1u ? wo_rank_tile_count_ex(height, tile_rows, 1u, nranks, cycle, skip) : 0u;
    return (t0 > t1 ? t0 : t1) * tile_rows;
}
static inline uint32_t wo_rank_local_rows(uint32_t height, uint32_t tile_rows, uint32_t nranks) {
    return wo_rank_local_rows_ex(height, tile_rows, nranks, 0u, 0u);
}

#ifdef __cplusplus
}
#endif

#endif /* WOLOLO_WO_SCENE_H */
