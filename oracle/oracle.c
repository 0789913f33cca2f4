/*
 * oracle.c -- CPU oracle (TEST INFRASTRUCTURE; see oracle.h).
 *
 * Compiled with -ffp-contract=off -fno-fast-math on x86-64 (SSE scalar fp32:
 * every +,-,*,/,sqrtf is one correctly rounded IEEE op), so each function is a
 * bit-exact statement of the arithmetic it names.
 *
 * Structure is deliberately different from the HIP kernels: no culling, no
 * event window, no bit stack.  Every primitive is intersected, ALL boundary
 * events are sorted, and the CSG tree is re-evaluated from scratch with an
 * explicit stack after every event.  Only the semantics are shared.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* Analysis builds (tools/trace_stats.c) observe every trace: events collected,
 * events swept up to the hit, hit or miss.  No-op in the oracle proper. */
#ifndef ORACLE_TRACE_HOOK
#define ORACLE_TRACE_HOOK(scratch, n_events, n_swept, hit) ((void)0)
#endif
#ifndef ORACLE_DEPTH_HOOK
#define ORACLE_DEPTH_HOOK(depth) ((void)0)
#endif

/* ======================================================================== */
/* Reference shader: src/wololo/renderer/ubershader1.frag                   */
/* ======================================================================== */

/* frag:101-103 -- omega = 2 * 3.1415 / 4 folded by glslc to fp32 0x3fc90e56;
 * y = amplitude(2) * sin(omega * time).  sin is evaluated once per frame on the
 * host (libm sinf), exactly as the HIP path does. */
static float sphere_height(float time_sec) {
    union {
        uint32_t u;
        float f;
    } omega = {0x3fc90e56u};
    return 2.0f * sinf(omega.f * time_sec);
}

static void shade_reference(float out[4], uint32_t x, uint32_t y, uint32_t width, uint32_t height, float sy,
                            uint32_t mode) {
    /* frag:19-20 */
    float res_x = (float)width;
    float res_y = (float)height;
    float aspect = res_x / res_y;
    /* frag:26-29 -- gl_FragCoord = pixel centre, origin upper-left */
    float frag_x = (float)x + 0.5f;
    float frag_y = (float)y + 0.5f;
    float st_x = frag_x / res_x;
    float st_y = 1.0f - frag_y / res_y;
    if (mode == WO_MODE_DEBUG_ST) { /* frag:133-138 */
        out[0] = st_x;
        out[1] = st_y;
        out[2] = 0.0f;
        out[3] = 1.0f;
        return;
    }
    /* frag:52-60: origin 0, horizontal (aspect,0,0), vertical (0,1,0),
     * lower_left = origin - h/2 - v/2 - (0,0,1) */
    float half_h = aspect / 2.0f;
    float llc[3] = {((0.0f - half_h) - 0.0f) - 0.0f, ((0.0f - 0.0f) - 0.5f) - 0.0f, ((0.0f - 0.0f) - 0.0f) - 1.0f};
    /* frag:74-82: dir = llc + st.x*h + st.y*v - origin (no normalisation) */
    float hx = st_x * aspect, hy = st_x * 0.0f, hz = st_x * 0.0f;
    float vx = st_y * 0.0f, vy = st_y * 1.0f, vz = st_y * 0.0f;
    float dir[3] = {((llc[0] + hx) + vx) - 0.0f, ((llc[1] + hy) + vy) - 0.0f, ((llc[2] + hz) + vz) - 0.0f};
    /* frag:100-105 */
    float center[3] = {0.0f, sy, -1.0f - 10.0f};
    float radius = 0.5f;
    /* frag:84-95 hit_sphere; dot(u,v) = (u.x v.x + u.y v.y) + u.z v.z */
    float oc[3] = {0.0f - center[0], 0.0f - center[1], 0.0f - center[2]};
    float a = (dir[0] * dir[0] + dir[1] * dir[1]) + dir[2] * dir[2];
    float b = 2.0f * ((oc[0] * dir[0] + oc[1] * dir[1]) + oc[2] * dir[2]);
    float c = ((oc[0] * oc[0] + oc[1] * oc[1]) + oc[2] * oc[2]) - radius * radius;
    float disc = b * b - (4.0f * a) * c;
    float t;
    if (disc < 0.0f)
        t = -1.0f;
    else
        t = (-b - sqrtf(disc)) / (2.0f * a);
    if (t > 0.0f) { /* frag:107-111: normal = normalize(dir*t - centre) = v / length(v) */
        float v[3] = {dir[0] * t - center[0], dir[1] * t - center[1], dir[2] * t - center[2]};
        float len = sqrtf((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
        for (int i = 0; i < 3; ++i) out[i] = 0.5f * (v[i] / len + 1.0f);
    } else { /* frag:116-122 */
        float len = sqrtf((dir[0] * dir[0] + dir[1] * dir[1]) + dir[2] * dir[2]);
        float u = dir[1] / len;
        float sky[3] = {0.5f, 0.7f, 1.0f};
        for (int i = 0; i < 3; ++i) out[i] = (1.0f - u) * 1.0f + u * sky[i];
    }
    out[3] = 1.0f;
}

void oracle_ubershader_pixel(float out[4], uint32_t x, uint32_t y, uint32_t width, uint32_t height, float time_sec,
                             uint32_t mode) {
    shade_reference(out, x, y, width, height, sphere_height(time_sec), mode);
}

void oracle_ubershader_frame(float* out, uint32_t width, uint32_t height, float time_sec, uint32_t mode,
                             int nthreads) {
    float sy = sphere_height(time_sec);
    (void)nthreads;
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (long y = 0; y < (long)height; ++y)
        for (uint32_t x = 0; x < width; ++x)
            shade_reference(out + ((size_t)y * width + x) * 4, x, (uint32_t)y, width, height, sy, mode);
}

/* ======================================================================== */
/* CSG path tracer semantics                                                */
/* ======================================================================== */

uint32_t oracle_pcg_hash(uint32_t v) {
    uint32_t state = v * 747796405u + 2891336453u;
    uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}

uint32_t oracle_rng_next(uint32_t* state) {
    *state = *state * 747796405u + 2891336453u;
    uint32_t word = ((*state >> ((*state >> 28u) + 4u)) ^ *state) * 277803737u;
    return (word >> 22u) ^ word;
}

static float rng_float(uint32_t* state) { return (float)(oracle_rng_next(state) >> 8) * (1.0f / 16777216.0f); }

static float dot3(const float a[3], const float b[3]) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
/* The path tracer's square root: sqrtf of max(x, 2^-96) (wo_device_common.h
 * sqrt_pt; the kernels' correctly rounded sequence is exact from 2^-96 up). */
static float sqrt_pt(float x) { return sqrtf(fmaxf(x, 0x1p-96f)); }
/* Exported for tests/test_oracle.py: the clamp must leave IEEE sqrtf untouched on [2^-96, inf]
 * (keep the oracle tied to IEEE behaviour, not to the kernel). */
void oracle_sqrt_pt_array(const float* in, float* out, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) out[i] = sqrt_pt(in[i]);
}

static void normalize3(float v[3]) {
    float inv = 1.0f / sqrt_pt(dot3(v, v));
    v[0] = v[0] * inv;
    v[1] = v[1] * inv;
    v[2] = v[2] * inv;
}

/* sin and cos of the angle 2*pi*u: reduce to the nearest quarter turn, then
 * fp32 minimax polynomials (Cephes sinf/cosf coefficients) on [-pi/4, pi/4],
 * one rounding per written operation. */
static void sincos_turn(float u, float* s, float* c) {
    float quarter_turns = u * 4.0f;
    float q = rintf(quarter_turns); /* round half to even, as v_rndne_f32 */
    float x = (quarter_turns - q) * 1.57079637f;
    float xx = x * x;
    float ps = -1.9515295891e-4f * xx;
    ps = ps + 8.3321608736e-3f;
    ps = ps * xx;
    ps = ps - 1.6666654611e-1f;
    ps = ps * xx;
    ps = ps * x;
    float sin_x = x + ps;
    float pc = 2.443315711809948e-5f * xx;
    pc = pc - 1.388731625493765e-3f;
    pc = pc * xx;
    pc = pc + 4.166664568298827e-2f;
    pc = pc * xx;
    pc = pc * xx;
    float cos_x = (1.0f - 0.5f * xx) + pc;
    switch ((unsigned)(int)q & 3u) {
    case 0: *s = sin_x; *c = cos_x; break;
    case 1: *s = cos_x; *c = -sin_x; break;
    case 2: *s = -sin_x; *c = -cos_x; break;
    default: *s = -cos_x; *c = sin_x; break;
    }
}

/* Uniform unit vector: z uniform in [-1, 1], azimuth uniform. */
static void rand_unit_vector(uint32_t* rng, float p[3]) {
    float z = 1.0f - 2.0f * rng_float(rng);
    float r = sqrt_pt(1.0f - z * z);
    float s, c;
    sincos_turn(rng_float(rng), &s, &c);
    p[0] = r * c;
    p[1] = r * s;
    p[2] = z;
}

/* Ray interval of one leaf; empty = [+inf, -inf]. */
static void leaf_span(const WoRec* L, const float o[3], const float d[3], float* lo, float* hi) {
    if (L->op == WO_LEAF_SPHERE) {
        /* |o + t d - c|^2 = r^2 with |d| = 1, via the perpendicular foot l */
        /* single-rounding fused multiply-adds in this order (fmaf) */
        float f[3] = {o[0] - L->f[0], o[1] - L->f[1], o[2] - L->f[2]};
        float b = fmaf(f[2], d[2], fmaf(f[1], d[1], f[0] * d[0]));
        float l[3] = {fmaf(-b, d[0], f[0]), fmaf(-b, d[1], f[1]), fmaf(-b, d[2], f[2])};
        float disc = L->f[3] - fmaf(l[2], l[2], fmaf(l[1], l[1], l[0] * l[0]));
        if (disc < 0.0f) {
            *lo = INFINITY;
            *hi = -INFINITY;
            return;
        }
        float s = sqrt_pt(disc);
        *lo = -b - s;
        *hi = -b + s;
        return;
    }
    /* half-space {x : n.x <= h} */
    float n[3] = {L->f[0], L->f[1], L->f[2]};
    float den, dist;
    if (L->u1 != 0u) {
        /* axis-aligned n = s*e_a (wo_scene.h): t = (h - s*o_a) * (s*(1/d_a)) */
        uint32_t a = L->u1 - 1u;
        float s = n[a];
        den = s * d[a];
        dist = L->f[3] - s * o[a];
        if (den != 0.0f) {
            float t = dist * (s * (1.0f / d[a]));
            *lo = den > 0.0f ? -INFINITY : t;
            *hi = den > 0.0f ? t : INFINITY;
            return;
        }
    } else {
        den = dot3(n, d);
        dist = L->f[3] - dot3(n, o);
    }
    if (den == 0.0f) {
        if (dist >= 0.0f) {
            *lo = -INFINITY;
            *hi = INFINITY;
        } else {
            *lo = INFINITY;
            *hi = -INFINITY;
        }
        return;
    }
    float t = dist / den;
    if (den > 0.0f) {
        *lo = -INFINITY;
        *hi = t;
    } else {
        *lo = t;
        *hi = INFINITY;
    }
}

typedef struct Prim {
    uint32_t pc, count;
} Prim;

typedef struct Event {
    uint64_t key; /* t bits | ordinal | type | member */
} Event;

typedef struct Scratch {
    Prim* prims;
    uint32_t nprims;
    Event* ev;
    unsigned char* inside;
    unsigned char* stack;
} Scratch;

static int scratch_init(Scratch* s, const WoRec* prog, uint32_t n) {
    memset(s, 0, sizeof *s);
    uint32_t np = 0;
    for (uint32_t pc = 0; pc < n;) {
        if (prog[pc].op == WO_OP_PRIM) {
            ++np;
            pc += 1u + prog[pc].u0;
        } else {
            ++pc;
        }
    }
    s->prims = (Prim*)malloc(sizeof(Prim) * (np + 1));
    s->ev = (Event*)malloc(sizeof(Event) * (2 * np + 1));
    s->inside = (unsigned char*)malloc(np + 1);
    s->stack = (unsigned char*)malloc(n + 1);
    if (!s->prims || !s->ev || !s->inside || !s->stack) return -1;
    for (uint32_t pc = 0; pc < n;) {
        if (prog[pc].op == WO_OP_PRIM) {
            s->prims[s->nprims].pc = pc;
            s->prims[s->nprims].count = prog[pc].u0;
            ++s->nprims;
            pc += 1u + prog[pc].u0;
        } else {
            ++pc;
        }
    }
    return 0;
}

static void scratch_free(Scratch* s) {
    free(s->prims);
    free(s->ev);
    free(s->inside);
    free(s->stack);
}

/* Postfix evaluation with an explicit stack; BOUND records are ignored. */
static int eval_tree(const WoRec* prog, uint32_t n, const unsigned char* inside, unsigned char* stack) {
    int sp = 0;
    uint32_t ord = 0;
    for (uint32_t pc = 0; pc < n;) {
        uint32_t op = prog[pc].op;
        if (op == WO_OP_PRIM) {
            stack[sp++] = inside[ord++];
            pc += 1u + prog[pc].u0;
            continue;
        }
        if (op == WO_OP_BOUND) {
            ++pc;
            continue;
        }
        int B = stack[--sp];
        int A = stack[--sp];
        int r;
        switch (op) {
        case WO_OP_UNION: r = A || B; break;
        case WO_OP_INTER: r = A && B; break;
        case WO_OP_DIFF: r = A && !B; break;
        default: r = B && !A; break; /* WO_OP_RDIFF */
        }
        stack[sp++] = (unsigned char)r;
        ++pc;
    }
    return sp > 0 ? stack[sp - 1] : 0;
}

static int cmp_event(const void* a, const void* b) {
    uint64_t x = ((const Event*)a)->key, y = ((const Event*)b)->key;
    return x < y ? -1 : x > y ? 1 : 0;
}

static uint64_t make_key(float t, uint32_t ord, uint32_t type, uint32_t member) {
    union {
        float f;
        uint32_t u;
    } tb;
    tb.f = t;
    return ((uint64_t)tb.u << 32) | (uint64_t)((ord << 12) | (type << 11) | member);
}

typedef struct OHit {
    float t;
    uint32_t ord, type, member, root_after;
} OHit;

/* First change of the root's membership along o + t d, t > WO_T_MIN. */
static int trace_ray(const WoRec* prog, uint32_t n, Scratch* s, const float o[3], const float d[3], OHit* hit) {
    const float tmin = WO_T_MIN;
    uint32_t nev = 0;
    for (uint32_t k = 0; k < s->nprims; ++k) {
        /* convex primitive: intersection of the member spans, starting from the
         * first member's span; the first member attaining the extreme wins */
        float lo, hi;
        uint32_t mlo = 0, mhi = 0;
        leaf_span(&prog[s->prims[k].pc + 1u], o, d, &lo, &hi);
        for (uint32_t m = 1; m < s->prims[k].count; ++m) {
            float a, b;
            leaf_span(&prog[s->prims[k].pc + 1u + m], o, d, &a, &b);
            if (a > lo) {
                lo = a;
                mlo = m;
            }
            if (b < hi) {
                hi = b;
                mhi = m;
            }
        }
        s->inside[k] = 0;
        if (lo > hi) continue; /* empty */
        s->inside[k] = (lo <= tmin && hi > tmin) ? 1 : 0;
        if (lo > tmin) s->ev[nev++].key = make_key(lo, k, 0u, mlo);
        if (hi > tmin && hi < INFINITY) s->ev[nev++].key = make_key(hi, k, 1u, mhi);
    }
    if (nev == 0) {
        ORACLE_TRACE_HOOK(s, 0u, 0u, 0);
        return 0;
    }
    qsort(s->ev, nev, sizeof(Event), cmp_event);
    int root = eval_tree(prog, n, s->inside, s->stack);
    for (uint32_t i = 0; i < nev; ++i) {
        uint32_t lo32 = (uint32_t)s->ev[i].key;
        uint32_t ord = lo32 >> 12;
        s->inside[ord] ^= 1u;
        int r = eval_tree(prog, n, s->inside, s->stack);
        if (r != root) {
            union {
                uint32_t u;
                float f;
            } tb;
            tb.u = (uint32_t)(s->ev[i].key >> 32);
            hit->t = tb.f;
            hit->ord = ord;
            hit->type = (lo32 >> 11) & 1u;
            hit->member = lo32 & 2047u;
            hit->root_after = (uint32_t)r;
            ORACLE_TRACE_HOOK(s, nev, i + 1u, 1);
            return 1;
        }
        root = r;
    }
    ORACLE_TRACE_HOOK(s, nev, nev, 0);
    return 0;
}

int oracle_trace(WoRec const* prog, uint32_t n_recs, float const o[3], float const d[3], float* t, uint32_t* prim,
                 uint32_t* type, uint32_t* member, uint32_t* root_after) {
    Scratch s;
    if (scratch_init(&s, prog, n_recs)) {
        scratch_free(&s);
        return -1;
    }
    OHit h;
    int found = trace_ray(prog, n_recs, &s, o, d, &h);
    if (found) {
        *t = h.t;
        *prim = h.ord;
        *type = h.type;
        *member = h.member;
        *root_after = h.root_after;
    }
    scratch_free(&s);
    return found;
}

/* RTIOW sky gradient */
static void sky_color(const float d[3], float c[3]) {
    float t = 0.5f * (d[1] + 1.0f);
    float s = 1.0f - t;
    c[0] = s + t * 0.5f;
    c[1] = s + t * 0.7f;
    c[2] = s + t * 1.0f;
}

/* Samples are summed as exact 32.32 fixed point, so a pixel's sum does not depend
 * on the order its samples are added in (the GPU hands samples to whichever lane
 * is free).  |r| >= 2^20 and NaN contribute 0. */
static int64_t quantize_radiance(float r) { return fabsf(r) < 1048576.0f ? (int64_t)((double)r * 4294967296.0) : 0; }
static float mean_radiance(int64_t sum, uint32_t spp) {
    return (float)(((double)sum * (1.0 / 4294967296.0)) / (double)spp);
}

/* One pixel: spp samples of up to max_depth segments each. */
static void shade_pixel(const WoRec* prog, uint32_t n, const WoMaterial* mats, uint32_t n_mats, const WoFrame* fr,
                        Scratch* s, uint32_t x, uint32_t y, float out[4], uint64_t* segs) {
    const WoCamera* cam = &fr->cam;
    const int normals = fr->mode == WO_MODE_NORMALS;
    const uint32_t spp = normals ? 1u : fr->spp;
    const uint32_t max_depth = normals ? 1u : fr->max_depth;
    const uint32_t W = fr->width, H = fr->height;
    const uint32_t pixel = y * W + x;
    int64_t sum[3] = {0, 0, 0};
    if (spp == 0 || max_depth == 0) {
        for (int i = 0; i < 3; ++i) out[i] = mean_radiance(0, spp);
        out[3] = 1.0f;
        return;
    }
    for (uint32_t smp = 0; smp < spp; ++smp) {
        uint32_t rng = oracle_pcg_hash(pixel ^ oracle_pcg_hash((fr->sample_offset + smp) ^ oracle_pcg_hash(fr->seed)));
        float u, v;
        if (normals) {
            u = ((float)x + 0.5f) * fr->inv_width;
            v = ((float)(H - 1u - y) + 0.5f) * fr->inv_height;
        } else {
            float jx = rng_float(&rng);
            float jy = rng_float(&rng);
            u = ((float)x + jx) * fr->inv_width;
            v = ((float)(H - 1u - y) + jy) * fr->inv_height;
        }
        float off[3] = {0.0f, 0.0f, 0.0f};
        if (cam->lens_radius > 0.0f && !normals) {
            /* point on the unit disk: radius sqrt(u), angle 2*pi*v */
            float rad = sqrt_pt(rng_float(&rng));
            float s, c;
            sincos_turn(rng_float(&rng), &s, &c);
            float px = rad * c, py = rad * s;
            float rx = cam->lens_radius * px, ry = cam->lens_radius * py;
            for (int i = 0; i < 3; ++i) off[i] = cam->u[i] * rx + cam->v[i] * ry;
        }
        float o[3], d[3];
        for (int i = 0; i < 3; ++i) {
            o[i] = cam->origin[i] + off[i];
            d[i] = ((cam->lower_left[i] + u * cam->horizontal[i]) + v * cam->vertical[i]) - cam->origin[i] - off[i];
        }
        normalize3(d);
        float thr[3] = {1.0f, 1.0f, 1.0f};
        float rad[3] = {0.0f, 0.0f, 0.0f};
        for (uint32_t depth = 0; depth < max_depth; ++depth) {
            OHit h;
            ++*segs;
            ORACLE_DEPTH_HOOK(depth);
            if (!trace_ray(prog, n, s, o, d, &h)) {
                float sk[3];
                sky_color(d, sk);
                for (int i = 0; i < 3; ++i) rad[i] = thr[i] * sk[i];
                break;
            }
            const WoRec* L = &prog[s->prims[h.ord].pc + 1u + h.member];
            float P[3] = {o[0] + h.t * d[0], o[1] + h.t * d[1], o[2] + h.t * d[2]};
            float nl[3];
            if (L->op == WO_LEAF_SPHERE) {
                for (int i = 0; i < 3; ++i) nl[i] = (P[i] - L->f[i]) * L->f[4];
            } else {
                for (int i = 0; i < 3; ++i) nl[i] = L->f[i];
            }
            /* normal facing the incoming ray: the leaf's outward normal when the
             * event enters the leaf, its negation when it leaves it */
            float N[3];
            for (int i = 0; i < 3; ++i) N[i] = h.type == 0u ? nl[i] : -nl[i];
            int front = h.root_after != 0u; /* ray enters the CSG solid */
            if (normals) {
                for (int i = 0; i < 3; ++i) {
                    float ns = front ? N[i] : -N[i];
                    rad[i] = 0.5f * (ns + 1.0f);
                }
                break;
            }
            uint32_t mid = L->u0 < n_mats ? L->u0 : 0u;
            const WoMaterial* m = &mats[mid];
            float nd[3], att[3];
            if (m->kind == WO_MAT_LAMBERTIAN) {
                float ru[3];
                rand_unit_vector(&rng, ru);
                float sd[3] = {N[0] + ru[0], N[1] + ru[1], N[2] + ru[2]};
                if (fabsf(sd[0]) < 1e-8f && fabsf(sd[1]) < 1e-8f && fabsf(sd[2]) < 1e-8f) {
                    sd[0] = N[0];
                    sd[1] = N[1];
                    sd[2] = N[2];
                }
                memcpy(nd, sd, sizeof nd);
                normalize3(nd);
                for (int i = 0; i < 3; ++i) att[i] = m->albedo[i];
            } else if (m->kind == WO_MAT_METAL) {
                float k = 2.0f * dot3(d, N);
                float rs[3];
                rand_unit_vector(&rng, rs); /* RTIOW v4 fuzz: unit vector */
                float sc[3];
                for (int i = 0; i < 3; ++i) sc[i] = (d[i] - k * N[i]) + m->fuzz * rs[i];
                if (!(dot3(sc, N) > 0.0f)) break; /* absorbed */
                memcpy(nd, sc, sizeof nd);
                normalize3(nd);
                for (int i = 0; i < 3; ++i) att[i] = m->albedo[i];
            } else {
                float ri = front ? m->inv_ior : m->ior;
                float nd0[3] = {-d[0], -d[1], -d[2]};
                float ct = dot3(nd0, N);
                if (!(ct < 1.0f)) ct = 1.0f;
                float st = sqrt_pt(1.0f - ct * ct);
                int reflect = ri * st > 1.0f;
                if (!reflect) {
                    const float r0 = m->r0; /* Schlick base, symmetric in ri and 1/ri */
                    float q = 1.0f - ct;
                    float q5 = (((q * q) * q) * q) * q;
                    reflect = r0 + (1.0f - r0) * q5 > rng_float(&rng);
                }
                float sc[3];
                if (reflect) {
                    float k = 2.0f * dot3(d, N);
                    for (int i = 0; i < 3; ++i) sc[i] = d[i] - k * N[i];
                } else {
                    float perp[3];
                    for (int i = 0; i < 3; ++i) perp[i] = ri * (d[i] + ct * N[i]);
                    float par = -sqrt_pt(fabsf(1.0f - dot3(perp, perp)));
                    for (int i = 0; i < 3; ++i) sc[i] = perp[i] + par * N[i];
                }
                memcpy(nd, sc, sizeof nd);
                normalize3(nd);
                att[0] = att[1] = att[2] = 1.0f;
            }
            for (int i = 0; i < 3; ++i) {
                thr[i] = thr[i] * att[i];
                o[i] = P[i];
                d[i] = nd[i];
            }
        }
        for (int i = 0; i < 3; ++i) sum[i] += quantize_radiance(rad[i]);
    }
    for (int i = 0; i < 3; ++i) out[i] = mean_radiance(sum[i], spp);
    out[3] = 1.0f;
}

int oracle_pathtrace_pixels(WoRec const* prog, uint32_t n_recs, WoMaterial const* mats, uint32_t n_mats,
                            WoFrame const* fr, uint32_t const* xs, uint32_t const* ys, uint32_t npix, float* out,
                            uint64_t* segments, int nthreads) {
    uint64_t total = 0;
    int fail = 0;
    (void)nthreads;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : total) reduction(| : fail)
#endif
    {
        Scratch s;
        if (scratch_init(&s, prog, n_recs)) {
            fail = 1;
        } else {
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 16)
#endif
            for (long i = 0; i < (long)npix; ++i) {
                uint64_t segs = 0;
                shade_pixel(prog, n_recs, mats, n_mats, fr, &s, xs[i], ys[i], out + (size_t)i * 4, &segs);
                total += segs;
            }
        }
        scratch_free(&s);
    }
    if (segments) *segments = total;
    return fail ? -1 : 0;
}

int oracle_pathtrace_rows(WoRec const* prog, uint32_t n_recs, WoMaterial const* mats, uint32_t n_mats,
                          WoFrame const* fr, uint32_t row0, uint32_t nrows, float* out, uint64_t* segments,
                          int nthreads) {
    uint64_t total = 0;
    int fail = 0;
    const uint32_t W = fr->width;
    (void)nthreads;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : total) reduction(| : fail)
#endif
    {
        Scratch s;
        if (scratch_init(&s, prog, n_recs)) {
            fail = 1;
        } else {
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 16)
#endif
            for (long i = 0; i < (long)nrows * W; ++i) {
                uint32_t y = row0 + (uint32_t)(i / W), x = (uint32_t)(i % W);
                uint64_t segs = 0;
                shade_pixel(prog, n_recs, mats, n_mats, fr, &s, x, y, out + (size_t)i * 4, &segs);
                total += segs;
            }
        }
        scratch_free(&s);
    }
    if (segments) *segments = total;
    return fail ? -1 : 0;
}

void oracle_sincos_turn(float u, float* s, float* c) { sincos_turn(u, s, c); }
