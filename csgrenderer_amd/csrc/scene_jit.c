/*
 * scene_jit.c -- generates a scene-specialised HIP trace kernel from the
 * compiled CSG program (wo_scene.h).  The source is compiled at scene upload by
 * hiprtc (trace_kernels.hip: wo_dev_upload_scene), the way a Vulkan renderer
 * builds a pipeline for its shaders (ref renderer.c:1135-1280 loads the SPIR-V
 * and builds the pipeline at init).
 *
 * What specialisation buys over the interpreter kernel:
 *   - leaf parameters become fp32 literals (no LDS/global reads, no VGPRs);
 *   - BOUND culling becomes a scalar branch around the subtree's code, its
 *     ballot result kept in an SGPR for the later evaluations;
 *   - the CSG evaluation becomes straight-line masked compares of the membership
 *     words (one per literal set, gen_eval_flat) instead of a decoded postfix walk.
 * The arithmetic, event order and tie-breaking are exactly the interpreter's
 * (wo_device_common.h), so both paths agree bit-for-bit with the oracle.
 */
#include <inttypes.h>
#include <stdarg.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "wo_internal.h"

typedef struct Buf {
    char* s;
    size_t n, cap;
    int oom;
} Buf;

static void bput(Buf* b, const char* fmt, ...) {
    if (b->oom) return;
    for (;;) {
        va_list ap;
        va_start(ap, fmt);
        size_t room = b->cap - b->n;
        int k = vsnprintf(b->s ? b->s + b->n : NULL, b->s ? room : 0, fmt, ap);
        va_end(ap);
        if (k < 0) {
            b->oom = 1;
            return;
        }
        if (b->s && (size_t)k < room) {
            b->n += (size_t)k;
            return;
        }
        size_t nc = b->cap ? b->cap * 2 : 1 << 16;
        while (nc < b->n + (size_t)k + 1) nc *= 2;
        char* ns = (char*)realloc(b->s, nc);
        if (!ns) {
            b->oom = 1;
            return;
        }
        b->s = ns;
        b->cap = nc;
    }
}

static uint32_t fbits(float v) {
    uint32_t u;
    memcpy(&u, &v, sizeof u);
    return u;
}

/* Scene constants are materialised by a volatile s_mov_b32 AT THEIR USE: every
 * trace runs inside the sample loop, and plain literals are loop-invariant, so
 * the compiler would hoist hundreds of them into registers for the whole kernel
 * (measured: 210 VGPRs, 160 SGPR spills for csg32).  One SALU op per constant
 * keeps them in short-lived SGPRs.  `names` are the declared float variables. */
static void emit_consts(Buf* b, int indent, const char* type, const char* names[], const uint32_t* vals, int n) {
    bput(b, "%*s%s %s", indent, "", type, names[0]);
    for (int i = 1; i < n; ++i) bput(b, ", %s", names[i]);
    bput(b, ";\n%*sasm volatile(\"", indent, "");
    for (int i = 0; i < n; ++i) bput(b, "%ss_mov_b32 %%%d, 0x%08x", i ? "\\n\\t" : "", i, vals[i]);
    bput(b, "\" : ");
    for (int i = 0; i < n; ++i) bput(b, "%s\"=s\"(%s)", i ? ", " : "", names[i]);
    bput(b, ");\n");
}

typedef struct Gen {
    const WoRec* prog;
    uint32_t n;
    uint32_t bound_min_leaves; /* smaller BOUND records are not tested (inlined) */
    int lds_events;            /* event window: LDS list (LdsWindow) or registers (Window) */
    Buf* b;
    uint32_t nbound;  /* BOUND counter (cull flag names) */
    int first_pass;   /* gen_collect: the first pass (cull tests, bits at t_min) or a re-collect */
    uint32_t nval;    /* value counter (eval temporaries) */
    int first_event;  /* the first event of waves that start outside every primitive from a constant table */
    int term_mode;    /* root a union of <= 2-literal conjunctions: term transitions, no event window (gen_term) */
    int spatial;      /* collect grouped by a spatial hierarchy over the primitives (gen_spatial) */
    uint32_t spatial_leaf; /* most primitives in a leaf group of that hierarchy */
    int cull_barrier;      /* cull[] through an opaque move in re-collects */
    uint32_t ncw;          /* words of cull[] */
    struct SPrim* sprims;  /* the bounded primitives it groups */
    uint32_t nsprims;
    struct SPrim* tunb;    /* term mode: terms without a bounding sphere (tested first, ungrouped) */
    uint32_t ntunb;
    const struct RTree* rtree; /* collect over the CSG tree with relevance-box culls (gen_rtree), or NULL */
    struct DList* dls; /* decision-list pool (ids are 1-based; 0 = none) */
    uint32_t ndl, dl_cap;
    int err;
} Gen;

/* A BOUND record gets a wave-level test when its subtree has enough leaves and
 * holds more than one primitive: a lone convex primitive's own first member,
 * with the member skip, is the cheaper test (csg32 4.87 -> 4.82 ms). */
static int bound_tested(const Gen* g, uint32_t pc) {
    const WoRec* r = &g->prog[pc];
    if (g->spatial) return 0; /* the spatial hierarchy culls instead (gen_spatial) */
    if (r->u1 < g->bound_min_leaves) return 0;
    if (pc + 1u < g->n && g->prog[pc + 1u].op == WO_OP_PRIM &&
        pc + 2u + g->prog[pc + 1u].u0 == r->u0)
        return 0;
    return 1;
}

/* ---- collect: intersect every primitive of [start, end), fill the window ---- */
static void gen_lone_sphere(Gen* g, const WoRec* L, uint32_t ord, int indent);

/* The members of the convex primitive at pc (cnt leaves) met into `iv`
 * (declared by the caller with `float la, lb;`): the wave-level member skip,
 * fused slab face pairs, literal constants. */
static void gen_members(Gen* g, uint32_t pc, uint32_t cnt, int indent) {
    static const char* nl[4] = {"c0", "c1", "c2", "c3"};
    int open_skips = 0;
    for (uint32_t m = 0; m < cnt; ++m) {
        const WoRec* L = &g->prog[pc + 1 + m];
        uint32_t vl[4];
        for (int i = 0; i < 4; ++i) vl[i] = fbits(L->f[i]);
        if (m > 0) /* empty on every lane: the other members cannot widen it */
            bput(g->b, "%*s  if (__ballot(!(iv.a > iv.b)) != 0ull) {\n", indent, ""), ++open_skips;
        bput(g->b, "%*s  {\n", indent, "");
        const WoRec* L2 = m + 1u < cnt ? &g->prog[pc + 2 + m] : NULL;
        if (L->op == WO_LEAF_HALFSPACE && L->u1 != 0u && L2 && L2->op == WO_LEAF_HALFSPACE &&
            L2->u1 == L->u1 && (L->f[L->u1 - 1u] > 0.0f) != (L2->f[L2->u1 - 1u] > 0.0f)) {
            /* two faces of a slab: one entry, one exit (axis_pair_meet) */
            static const char axis[3] = {'x', 'y', 'z'};
            const char ax = axis[L->u1 - 1u];
            const int pos = L->f[L->u1 - 1u] > 0.0f; /* s1 = +1 */
            uint32_t vh[2] = {vl[3], fbits(L2->f[3])};
            bput(g->b, "%*s    WO_WK_N(WO_WORK_HALFSPACE_TESTS, 2u);\n", indent, "");
            if (m == 0) bput(g->b, "%*s    wodev::ivl_open(iv);\n", indent, "");
            /* dist1 = h1 - s1*oa, dist2 = h2 + s1*oa with h as a literal operand */
            bput(g->b,
                 "%*s    float dist1, dist2;\n"
                 "%*s    asm(\"%s %%0, 0x%08x, %%1\" : \"=v\"(dist1) : \"v\"(o.%c));\n"
                 "%*s    asm(\"%s %%0, 0x%08x, %%1\" : \"=v\"(dist2) : \"v\"(o.%c));\n"
                 "%*s    wodev::axis_pair_meet_d(iv, %s, dist1, dist2, d.%c, iv%c, %uu, %uu);\n%*s  }\n",
                 indent, "", indent, "", pos ? "v_sub_f32_e32" : "v_add_f32_e32", vh[0], ax, indent, "",
                 pos ? "v_add_f32_e32" : "v_sub_f32_e32", vh[1], ax, indent, "", pos ? "1.0f" : "-1.0f", ax,
                 ax, m, m + 1u, indent, "");
            ++m;
            continue;
        }
        bput(g->b, "%*s    WO_WK(%s);\n", indent, "",
             L->op == WO_LEAF_SPHERE ? "WO_WORK_SPHERE_TESTS" : "WO_WORK_HALFSPACE_TESTS");
        if (L->op == WO_LEAF_HALFSPACE && L->u1 != 0u) {
            /* axis-aligned: s = +-1 stays a literal (inline constant), h a literal operand */
            static const char axis[3] = {'x', 'y', 'z'};
            char ax = axis[L->u1 - 1u];
            const int pos = L->f[L->u1 - 1u] > 0.0f;
            bput(g->b,
                 "%*s    float dist;\n"
                 "%*s    asm(\"%s %%0, 0x%08x, %%1\" : \"=v\"(dist) : \"v\"(o.%c));\n"
                 "%*s    wodev::halfspace_axis_dist(%s, dist, d.%c, iv%c, la, lb);\n",
                 indent, "", indent, "", pos ? "v_sub_f32_e32" : "v_add_f32_e32", vl[3], ax, indent, "",
                 pos ? "1.0f" : "-1.0f", ax, ax);
        } else if (L->op == WO_LEAF_SPHERE) {
            /* the centre and r^2 as VALU literal operands: o - c and r^2 - ll
             * are single VOP2 operations (the constant needs no scalar move) */
            bput(g->b,
                 "%*s    float fx, fy, fz, b, ll, disc;\n"
                 "%*s    asm(\"v_subrev_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(fx) : \"v\"(o.x));\n"
                 "%*s    asm(\"v_subrev_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(fy) : \"v\"(o.y));\n"
                 "%*s    asm(\"v_subrev_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(fz) : \"v\"(o.z));\n"
                 "%*s    wodev::sphere_fbl(fx, fy, fz, d, b, ll);\n"
                 "%*s    asm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(disc) : \"v\"(ll));\n"
                 "%*s    wodev::sphere_interval_bd(b, disc, la, lb);\n",
                 indent, "", indent, "", vl[0], indent, "", vl[1], indent, "", vl[2], indent, "", indent, "",
                 vl[3], indent, "");
        } else { /* a general half-space: its constants by scalar moves */
            emit_consts(g->b, indent + 4, "float", nl, vl, 4);
            bput(g->b, "%*s    wodev::halfspace_interval(c0, c1, c2, c3, o, d, la, lb);\n", indent, "");
        }
        if (m == 0)
            bput(g->b, "%*s    wodev::ivl_first(iv, la, lb);\n", indent, "");
        else
            bput(g->b, "%*s    wodev::ivl_meet(iv, la, lb, %uu);\n", indent, "", m);
        bput(g->b, "%*s  }\n", indent, "");
    }
    for (; open_skips > 0; --open_skips) bput(g->b, "%*s  }\n", indent, "");
}

static void gen_collect(Gen* g, uint32_t start, uint32_t end, int indent) {
    uint32_t pc = start;
    while (pc < end && !g->err) {
        const WoRec* r = &g->prog[pc];
        if (r->op == WO_OP_BOUND && !bound_tested(g, pc)) {
            ++pc; /* too small to pay for a wave-level test: the subtree is emitted inline */
        } else if (r->op == WO_OP_BOUND) {
            uint32_t vb[5];
            for (int i = 0; i < 5; ++i) vb[i] = fbits(r->f[i]);
            uint32_t k = g->nbound++;
            if (g->first_pass) { /* the wave's cull decision; re-collects reuse it */
                bput(g->b, "%*s{  // BOUND %u\n%*s  WO_WK(WO_WORK_BOUND_TESTS);\n", indent, "", k, indent, "");
                /* c - o and tca + R with the constants as VALU literal operands; R^2
                 * (an FMA addend) in an SGPR */
                static const char* nr[1] = {"bc3"};
                emit_consts(g->b, indent + 2, "float", nr, &vb[3], 1);
                bput(g->b,
                     "%*s  float ox, oy, oz, tca, d2, tr;\n"
                     "%*s  asm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(ox) : \"v\"(o.x));\n"
                     "%*s  asm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(oy) : \"v\"(o.y));\n"
                     "%*s  asm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(oz) : \"v\"(o.z));\n"
                     "%*s  wodev::bound_tca_d2(ox, oy, oz, d, tca, d2);\n"
                     "%*s  asm(\"v_add_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(tr) : \"v\"(tca));\n"
                     "%*s  const bool miss = (d2 > __builtin_fmaf(4e-6f * tca, tca, bc3)) | (tr < 0.0f);\n"
                     "%*s  if (__ballot(!miss) == 0ull) cull[%u] |= %uu;\n"
                     "%*s}\n",
                     indent, "", indent, "", vb[0], indent, "", vb[1], indent, "", vb[2], indent, "", indent, "",
                     vb[4], indent, "", indent, "", k / 32, 1u << (k % 32), indent, "");
            }
            bput(g->b, "%*sif (!(cull[%u] & %uu)) {\n", indent, "", k / 32, 1u << (k % 32));
            gen_collect(g, pc + 1, r->u0, indent + 2);
            bput(g->b, "%*s}\n", indent, "");
            pc = r->u0;
        } else if (r->op == WO_OP_PRIM) {
            uint32_t ord = r->u1, cnt = r->u0;
            static const char* nk[2] = {"ka", "kb"};
            bput(g->b, "%*s{  // primitive %u (%u leaves)\n", indent, "", ord, cnt);
            if (cnt == 1u && g->prog[pc + 1].op == WO_LEAF_SPHERE) {
                gen_lone_sphere(g, &g->prog[pc + 1], ord, indent);
                pc += 2;
                continue;
            }
            bput(g->b, "%*s  wodev::Ivl iv; float la, lb;\n", indent, "");
            gen_members(g, pc, cnt, indent);
            uint32_t vk[2] = {ord << 12, (ord << 12) | (1u << 11)};
            bput(g->b, "%*s  if (!(iv.a > iv.b)) {\n", indent, "");
            emit_consts(g->b, indent + 4, "uint32_t", nk, vk, 2);
            /* one lane branch per event.  The first pass also sets the membership
             * bit at t_min; a re-collect keeps only the events after `after`. */
            if (g->first_pass)
                bput(g->b,
                     "%*s    bits[%u] |= ((iv.a <= tmin) & (iv.b > tmin) ? 1u : 0u) << %u;\n"
                     "%*s    { const bool c = iv.a > tmin; WO_WK_IF(c, WO_WORK_EVENTS); win.insert_if(c, wodev::event_key_lo(iv.a, ka | iv.ma)); }\n"
                     "%*s    { const bool c = (iv.b > tmin) & (iv.b < wodev::kInf); WO_WK_IF(c, WO_WORK_EVENTS); win.insert_if(c, wodev::event_key_lo(iv.b, kb | iv.mb)); }\n"
                     "%*s  }\n%*s}\n",
                     indent, "", ord / 32, ord % 32, indent, "", indent, "", indent, "", indent, "");
            else
                bput(g->b,
                     "%*s    uint64_t k0 = wodev::event_key_lo(iv.a, ka | iv.ma), k1 = wodev::event_key_lo(iv.b, kb | iv.mb);\n"
                     "%*s    { const bool c = (iv.a > tmin) & (k0 > after); WO_WK_IF(c, WO_WORK_EVENTS); win.insert_if(c, k0); }\n"
                     "%*s    { const bool c = (iv.b > tmin) & (iv.b < wodev::kInf) & (k1 > after); WO_WK_IF(c, WO_WORK_EVENTS); win.insert_if(c, k1); }\n"
                     "%*s  }\n%*s}\n",
                     indent, "", indent, "", indent, "", indent, "", indent, "");
            pc += 1 + cnt;
        } else {
            ++pc; /* binops: nothing to collect */
        }
    }
}

/* A primitive that is one sphere: its interval is [-b - s, -b + s] exactly when
 * disc >= 0, so the membership bit and the events are set inside the branch that
 * computes s (the lanes that skip it have an empty interval, as in
 * sphere_interval_bd: same bits and events) and no empty interval is formed.
 * Member index 0 (ivl_first). */
static void gen_lone_sphere(Gen* g, const WoRec* L, uint32_t ord, int indent) {
    uint32_t vl[4];
    for (int i = 0; i < 4; ++i) vl[i] = fbits(L->f[i]);
    bput(g->b,
         "%*s  WO_WK(WO_WORK_SPHERE_TESTS);\n"
         "%*s  float fx, fy, fz, b, ll, disc;\n"
         "%*s  asm(\"v_subrev_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(fx) : \"v\"(o.x));\n"
         "%*s  asm(\"v_subrev_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(fy) : \"v\"(o.y));\n"
         "%*s  asm(\"v_subrev_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(fz) : \"v\"(o.z));\n"
         "%*s  wodev::sphere_fbl(fx, fy, fz, d, b, ll);\n"
         "%*s  asm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(disc) : \"v\"(ll));\n"
         "%*s  if (__ballot(wodev::sphere_need(b, disc)) != 0ull) {\n"
         "%*s    asm volatile(\"\");\n"
         "#if WO_LONE_SEL_EV  // every lane of the wave forms the interval; hd masks the bit and the events\n"
         "%*s    {\n"
         "%*s      const bool hd = !(disc < 0.0f);\n"
         "#else\n"
         "%*s    if (!(disc < 0.0f)) {\n"
         "%*s      const bool hd = true;\n"
         "#endif\n"
         "%*s      const float s = wodev::sqrt_pt(disc), nb = -b, la = nb - s, lb = nb + s;\n"
         "%*s      uint32_t ka, kb;\n"
         "%*s      asm volatile(\"s_mov_b32 %%0, 0x%08x\\n\\ts_mov_b32 %%1, 0x%08x\" : \"=s\"(ka), \"=s\"(kb));\n",
         indent, "", indent, "", indent, "", vl[0], indent, "", vl[1], indent, "", vl[2], indent, "", indent, "", vl[3],
         indent, "", indent, "", indent, "", indent, "", indent, "", indent, "", indent, "", indent, "", indent, "",
         ord << 12, (ord << 12) | (1u << 11));
    if (g->first_pass)
        bput(g->b,
             "%*s      bits[%u] |= (hd & (la <= tmin) & (lb > tmin) ? 1u : 0u) << %u;\n"
             "%*s      { const bool c = hd & (la > tmin); WO_WK_IF(c, WO_WORK_EVENTS); win.insert_if(c, wodev::event_key_lo(la, ka)); }\n"
             "%*s      { const bool c = hd & (lb > tmin) & (lb < wodev::kInf); WO_WK_IF(c, WO_WORK_EVENTS); win.insert_if(c, wodev::event_key_lo(lb, kb)); }\n",
             indent, "", ord / 32, ord % 32, indent, "", indent, "");
    else
        bput(g->b,
             "%*s      const uint64_t k0 = wodev::event_key_lo(la, ka), k1 = wodev::event_key_lo(lb, kb);\n"
             "%*s      { const bool c = hd & (la > tmin) & (k0 > after); WO_WK_IF(c, WO_WORK_EVENTS); win.insert_if(c, k0); }\n"
             "%*s      { const bool c = hd & (lb > tmin) & (lb < wodev::kInf) & (k1 > after); WO_WK_IF(c, WO_WORK_EVENTS); win.insert_if(c, k1); }\n",
             indent, "", indent, "", indent, "");
    bput(g->b, "%*s    }\n%*s  }\n%*s}\n", indent, "", indent, "", indent, "");
}

/* ---- spatial collect ----
 * The collect pass is order-independent: each primitive sets its own membership
 * bit and adds its own events, and a primitive the ray does not reach keeps bit 0
 * and adds none -- its true state.  So any grouping of the primitives may cull,
 * not only the CSG tree's subtrees (BOUND records: a union cluster's hierarchy).
 * For a tree without such structure (csg256 chain: a left-deep chain whose
 * operands are scattered spheres) the primitives with a bounding sphere are
 * grouped by a median-split hierarchy and tested against the wave's rays group by
 * group; unbounded primitives (half-space-only convex primitives) are tested as
 * before.  The root evaluation then reads the bits alone (a culled primitive's
 * bits stay 0). */
#define SUNIT_MAX 8
typedef struct SPrim {
    double c[3], r;
    uint32_t pc;               /* a primitive's program counter ... */
    uint32_t npc;              /* ... or, for a unit of several primitives (npc > 0), theirs */
    uint32_t pcs[SUNIT_MAX];
    uint32_t negm;             /* term mode: bit k = pcs[k] is a complemented literal */
    int term;                  /* term mode: the unit is a term (gen_term) */
} SPrim;

/* a primitive's bounding sphere: its smallest sphere member (an intersection lies
 * inside each member); 0 when it has none */
static int prim_sphere(const WoRec* prog, uint32_t pc, SPrim* out) {
    const uint32_t cnt = prog[pc].u0;
    int found = 0;
    for (uint32_t m = 0; m < cnt; ++m) {
        const WoRec* L = &prog[pc + 1 + m];
        if (L->op != WO_LEAF_SPHERE) continue;
        const double r = sqrt((double)L->f[3]);
        if (!found || r < out->r) {
            out->c[0] = L->f[0], out->c[1] = L->f[1], out->c[2] = L->f[2], out->r = r;
            found = 1;
        }
    }
    out->pc = pc;
    out->npc = 0;
    out->negm = 0;
    out->term = 0;
    return found;
}

/* one comparator per axis (no shared state: scenes may be generated on several threads) */
#define SPRIM_CMP(A)                                                          \
    static int sprim_cmp##A(const void* a, const void* b) {                  \
        const double x = ((const SPrim*)a)->c[A], y = ((const SPrim*)b)->c[A]; \
        return x < y ? -1 : x > y;                                            \
    }
SPRIM_CMP(0)
SPRIM_CMP(1)
SPRIM_CMP(2)

/* the enclosing sphere of p[0..n), expanded as the scene compiler expands BOUNDs */
static void sprim_bound(const SPrim* p, uint32_t n, double c[3], double* R) {
    double lo[3], hi[3];
    for (int a = 0; a < 3; ++a) lo[a] = hi[a] = p[0].c[a];
    for (uint32_t i = 0; i < n; ++i)
        for (int a = 0; a < 3; ++a) {
            lo[a] = fmin(lo[a], p[i].c[a] - p[i].r);
            hi[a] = fmax(hi[a], p[i].c[a] + p[i].r);
        }
    for (int a = 0; a < 3; ++a) c[a] = 0.5 * (lo[a] + hi[a]);
    double r = 0.0;
    for (uint32_t i = 0; i < n; ++i) {
        const double dx = p[i].c[0] - c[0], dy = p[i].c[1] - c[1], dz = p[i].c[2] - c[2];
        r = fmax(r, sqrt(dx * dx + dy * dy + dz * dz) + p[i].r);
    }
    const double cn = sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    *R = r * (1.0 + 1e-4) + 1e-5 * (cn + r) + 1e-6;
}


static void gen_term(Gen* g, const SPrim* q, int indent);

static void gen_sprim(Gen* g, const SPrim* q, int indent) {
    if (q->term) {
        gen_term(g, q, indent);
        return;
    }
    if (!q->npc) {
        gen_collect(g, q->pc, q->pc + 1u + g->prog[q->pc].u0, indent);
        return;
    }
    for (uint32_t k = 0; k < q->npc; ++k) gen_collect(g, q->pcs[k], q->pcs[k] + 1u + g->prog[q->pcs[k]].u0, indent);
}

static void gen_spatial(Gen* g, SPrim* p, uint32_t n, int indent, int root) {
    if (n == 0u || g->err) return;
    if (n == 1u) {
        gen_sprim(g, &p[0], indent);
        return;
    }
    int inner = indent;
    if (!root) {
        double c[3], R;
        sprim_bound(p, n, c, &R);
        const uint32_t k = g->nbound++;
        if (g->first_pass) {
            const float fc[3] = {(float)c[0], (float)c[1], (float)c[2]};
            const float fR = (float)R, fR2 = (float)(R * R);
            uint32_t vr2 = fbits(fR2);
            static const char* nr[1] = {"bc3"};
            uint32_t nprim = 0;
            for (uint32_t i = 0; i < n; ++i) nprim += p[i].npc ? p[i].npc : 1u;
            bput(g->b, "%*s{  // group %u (%u primitives)\n%*s  WO_WK(WO_WORK_BOUND_TESTS);\n", indent, "", k, nprim,
                 indent, "");
            emit_consts(g->b, indent + 2, "float", nr, &vr2, 1);
            bput(g->b,
                 "%*s  float ox, oy, oz, tca, d2, tr;\n"
                 "%*s  asm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(ox) : \"v\"(o.x));\n"
                 "%*s  asm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(oy) : \"v\"(o.y));\n"
                 "%*s  asm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(oz) : \"v\"(o.z));\n"
                 "%*s  wodev::bound_tca_d2(ox, oy, oz, d, tca, d2);\n"
                 "%*s  asm(\"v_add_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(tr) : \"v\"(tca));\n"
                 "%*s  const bool miss = (d2 > __builtin_fmaf(4e-6f * tca, tca, bc3)) | (tr < 0.0f);\n"
                 "%*s  if (__ballot(!miss) == 0ull) cull[%u] |= %uu;\n",
                 indent, "", indent, "", fbits(fc[0]), indent, "", fbits(fc[1]), indent, "", fbits(fc[2]), indent, "",
                 indent, "", fbits(fR), indent, "", indent, "", k / 32, 1u << (k % 32));
            bput(g->b, "%*s}\n%*sif (!(cull[%u] & %uu)) {\n", indent, "", indent, "", k / 32, 1u << (k % 32));
        } else {
            bput(g->b, "%*sif (!(cull[%u] & %uu)) {\n", indent, "", k / 32, 1u << (k % 32));
        }
        inner = indent + 2;
    }
    if (n <= g->spatial_leaf) {
        for (uint32_t i = 0; i < n; ++i) gen_sprim(g, &p[i], inner);
    } else {
        /* surface-area split (csg32 3.716 -> 3.586 ms against median splits): over
         * the three axes (centres sorted) and every cut, the least R_left^2 * n_left
         * + R_right^2 * n_right of the enclosing spheres */
        uint32_t cut = n / 2u;
        int ax = 0;
        double best = -1.0;
        for (int a = 0; a < 3; ++a) {
            qsort(p, n, sizeof(SPrim), a == 0 ? sprim_cmp0 : a == 1 ? sprim_cmp1 : sprim_cmp2);
            for (uint32_t k = 1; k < n; ++k) {
                double cl[3], cr[3], rl, rr;
                sprim_bound(p, k, cl, &rl);
                sprim_bound(p + k, n - k, cr, &rr);
                const double cost = rl * rl * k + rr * rr * (n - k);
                if (best < 0.0 || cost < best) best = cost, ax = a, cut = k;
            }
        }
        qsort(p, n, sizeof(SPrim), ax == 0 ? sprim_cmp0 : ax == 1 ? sprim_cmp1 : sprim_cmp2);
        gen_spatial(g, p, cut, inner, 0);
        gen_spatial(g, p + cut, n - cut, inner, 0);
    }
    if (!root) bput(g->b, "%*s}\n", indent, "");
}

/* the collect of the whole program in spatial groups: unbounded primitives
 * first, in program order, then the hierarchy (same order in both passes) */
static void gen_collect_spatial(Gen* g, const SPrim* bounded, uint32_t nb, int indent) {
    for (uint32_t pc = 0; pc < g->n && !g->err;) {
        const WoRec* r = &g->prog[pc];
        if (r->op != WO_OP_PRIM) {
            ++pc;
            continue;
        }
        int grouped = 0;
        for (uint32_t i = 0; i < nb && !grouped; ++i) {
            if (!bounded[i].npc) grouped = bounded[i].pc == pc;
            for (uint32_t k = 0; k < bounded[i].npc && !grouped; ++k) grouped = bounded[i].pcs[k] == pc;
        }
        if (!grouped) gen_collect(g, pc, pc + 1u + r->u0, indent);
        pc += 1u + r->u0;
    }
    if (!nb) return;
    SPrim* p = (SPrim*)malloc(sizeof(SPrim) * nb);
    if (!p) {
        g->err = 1;
        return;
    }
    memcpy(p, bounded, sizeof(SPrim) * nb); /* gen_spatial sorts in place: the same order each pass */
    gen_spatial(g, p, nb, indent, 1);
    free(p);
}

/* term mode: the unbounded terms, then the spatial hierarchy over the others */
static void gen_collect_terms(Gen* g, int indent) {
    for (uint32_t i = 0; i < g->ntunb && !g->err; ++i) gen_term(g, &g->tunb[i], indent);
    if (!g->nsprims) return;
    SPrim* p = (SPrim*)malloc(sizeof(SPrim) * g->nsprims);
    if (!p) {
        g->err = 1;
        return;
    }
    memcpy(p, g->sprims, sizeof(SPrim) * g->nsprims); /* gen_spatial sorts in place: the same order each pass */
    gen_spatial(g, p, g->nsprims, indent, 1);
    free(p);
}

/* The cull words through an opaque move: the wave's cull bits are loop-invariant
 * in the sweep, and without it the compiler turns every bit the re-collect and
 * the root evaluation test into a 64-bit lane mask ahead of the sweep loop and
 * keeps them all live -- under SGPR pressure spilled to VGPR lanes (two
 * v_writelane per bit on every trace, csg256 chain: 60 per trace).  After the
 * move each test is an s_bitcmp where it is used.  The words are wave-uniform
 * (every active lane ran the same ballots), but a value carried through the
 * divergent sweep loop is not provably so: the first lane's copy (exact) puts it
 * in an SGPR for the move. */
static void gen_cull_barrier(Gen* g, int indent) {
    bput(g->b, "#if WO_JIT_CULL_BARRIER\n");
    for (uint32_t w = 0; w < g->ncw; ++w)
        bput(g->b,
             "%*s{ uint32_t cw = (uint32_t)__builtin_amdgcn_readfirstlane((int)cull[%u]); "
             "asm volatile(\"\" : \"+s\"(cw)); cull[%u] = cw; }\n",
             indent, "", w, w);
    bput(g->b, "#endif\n");
}

static void gen_rtree(Gen* g, int indent);

/* the collect of the whole program (either pass) */
static void gen_collect_all(Gen* g, int indent) {
    if (!g->first_pass) gen_cull_barrier(g, indent);
    g->nbound = 0;
    if (g->term_mode)
        gen_collect_terms(g, indent);
    else if (g->rtree)
        gen_rtree(g, indent);
    else if (g->spatial)
        gen_collect_spatial(g, g->sprims, g->nsprims, indent);
    else
        gen_collect(g, 0, g->n, indent);
}

/* ---- term mode ----
 * When the root is a union of TERMS -- conjunctions of one or two literals, a
 * literal being a primitive or its complement (a DIFF of one primitive by
 * another is a AND NOT b) -- and every primitive is in one term (csg32, csg256
 * balanced), a term changes value only at an event of one of its literals X, and
 * then exactly when the other literal holds at that key; it rises where X's
 * literal becomes true.  One key changes one term, so the root flips where the
 * count of true terms crosses 0.  The collect then keeps, per lane, only the
 * smallest term transition after `after` and whether it rises (wo_device_common.h
 * term_cands_of): no event list, no sweep; a ray that starts outside every term
 * hits at its first transition, others re-collect after each transition that does
 * not flip the root (rare: a ray inside one term meets its own exit first unless
 * another term begins before it).  The same rule as the lane tracer's term mode
 * (trace_kernels.hip extract_terms), bit for bit the general sweep's hit. */
#define JT_LITS 2
#define JT_NEG 0x80000000u
typedef struct JTerm {
    uint32_t n, lit[JT_LITS]; /* ordinal | JT_NEG for a complement */
} JTerm;

typedef struct JTSub {
    int kind;       /* 0 conjunction (t), 1 union of terms [start, start + count) of the term list, 2 neither */
    JTerm t;
    uint32_t start, count;
} JTSub;

/* Key constants of primitive `ord` as a term literal of polarity `pos`: the rise
 * flag (bit 10) on the event where the literal becomes true -- wodev::term_ka /
 * term_kb; JIT_TERM_MAX_MEMBERS = wodev::kTermMaxMembers. */
#define JIT_TERM_RISE (1u << 10)
#define JIT_TERM_MAX_MEMBERS JIT_TERM_RISE
static uint32_t term_ka(uint32_t ord, int pos) { return (ord << 12) | (pos ? JIT_TERM_RISE : 0u); }
static uint32_t term_kb(uint32_t ord, int pos) { return (ord << 12) | (1u << 11) | (pos ? 0u : JIT_TERM_RISE); }

/* The root's terms (malloc'd, *nt of them), or NULL when the root is not a union of
 * such conjunctions. */
static JTerm* jit_terms(const WoRec* prog, uint32_t n_recs, uint32_t n_prims, uint32_t* nt) {
    JTSub* st = (JTSub*)malloc(sizeof(JTSub) * (n_recs + 1u));
    JTerm* tl = (JTerm*)malloc(sizeof(JTerm) * (n_prims + 1u));
    uint32_t sp = 0, n = 0;
    int ok = st && tl;
    for (uint32_t pc = 0; pc < n_recs && ok;) {
        const WoRec* r = &prog[pc];
        if (r->op == WO_OP_PRIM) {
            if (r->u0 >= JIT_TERM_MAX_MEMBERS) { /* its member index would reach the rise flag */
                ok = 0;
                break;
            }
            JTSub x;
            memset(&x, 0, sizeof x);
            x.t.n = 1;
            x.t.lit[0] = r->u1;
            st[sp++] = x;
            pc += 1u + r->u0;
            continue;
        }
        ++pc;
        if (r->op == WO_OP_BOUND) continue;
        if (sp < 2u) {
            ok = 0;
            break;
        }
        JTSub b = st[--sp], a = st[--sp], out;
        memset(&out, 0, sizeof out);
        out.kind = 2;
        if (a.kind != 2 && b.kind != 2) {
            if (r->op == WO_OP_UNION) {
                /* the term list stays contiguous: a union child's terms were appended
                 * when it formed, a conjunction's are appended now */
                uint32_t start = a.kind == 1 ? a.start : (b.kind == 1 ? b.start : n);
                if (a.kind == 0 && n < n_prims) tl[n++] = a.t;
                if (b.kind == 0 && n < n_prims) tl[n++] = b.t;
                out.kind = 1;
                out.start = start;
                out.count = n - start;
            } else if (r->op == WO_OP_INTER && a.kind == 0 && b.kind == 0 && a.t.n + b.t.n <= JT_LITS) {
                out = a;
                for (uint32_t k = 0; k < b.t.n; ++k) out.t.lit[out.t.n++] = b.t.lit[k];
            } else if (r->op == WO_OP_DIFF || r->op == WO_OP_RDIFF) {
                const JTSub* keep = r->op == WO_OP_DIFF ? &a : &b; /* DIFF: a AND NOT b; RDIFF: b AND NOT a */
                const JTSub* sub = r->op == WO_OP_DIFF ? &b : &a;
                JTerm t = keep->t;
                int good = keep->kind == 0;
                if (good && sub->kind == 0) {
                    good = sub->t.n == 1u && !(sub->t.lit[0] & JT_NEG) && t.n < JT_LITS;
                    if (good) t.lit[t.n++] = sub->t.lit[0] | JT_NEG;
                } else if (good && sub->kind == 1) {
                    for (uint32_t i = 0; i < sub->count && good; ++i) {
                        const JTerm* u = &tl[sub->start + i];
                        good = u->n == 1u && !(u->lit[0] & JT_NEG) && t.n < JT_LITS;
                        if (good) t.lit[t.n++] = u->lit[0] | JT_NEG;
                    }
                    if (good) n = sub->start; /* the subtrahend's terms were the last ones appended */
                }
                if (good) {
                    out.kind = 0;
                    out.t = t;
                }
            }
        }
        st[sp++] = out;
    }
    if (ok && sp == 1u && st[0].kind == 0 && n < n_prims + 1u) {
        tl[n++] = st[0].t;
    } else if (!(ok && sp == 1u && st[0].kind == 1)) {
        ok = 0;
    }
    if (ok) { /* every primitive in exactly one term */
        uint8_t* seen = (uint8_t*)calloc(n_prims ? n_prims : 1u, 1);
        ok = seen != NULL;
        uint32_t lits = 0;
        for (uint32_t i = 0; i < n && ok; ++i)
            for (uint32_t k = 0; k < tl[i].n && ok; ++k) {
                const uint32_t o = tl[i].lit[k] & ~JT_NEG;
                ok = o < n_prims && !seen[o];
                if (ok) seen[o] = 1, ++lits;
            }
        ok = ok && lits == n_prims;
        free(seen);
    }
    free(st);
    if (!ok) {
        free(tl);
        return NULL;
    }
    *nt = n;
    return tl;
}

/* The interval of the convex primitive at pc into `name` (declared by the caller). */
static void gen_term_ivl(Gen* g, uint32_t pc, const char* name, int indent) {
    bput(g->b, "%*s{\n%*s  wodev::Ivl iv; float la, lb;\n", indent, "", indent, "");
    gen_members(g, pc, g->prog[pc].u0, indent);
    bput(g->b, "%*s  %s = iv;\n%*s}\n", indent, "", name, indent, "");
}

/* One term: its transitions into best, and at t_min its value into cnt (first pass). */
static void gen_term(Gen* g, const SPrim* q, int indent) {
    const int first = g->first_pass;
    uint32_t pcs[2] = {q->pcs[0], q->npc > 1u ? q->pcs[1] : 0u};
    int pos[2] = {!(q->negm & 1u), !(q->negm & 2u)};
    if (q->npc > 1u && !pos[0] && pos[1]) { /* a positive literal first: it can skip the other */
        const uint32_t t = pcs[0];
        pcs[0] = pcs[1], pcs[1] = t;
        pos[0] = 1, pos[1] = 0;
    }
    const uint32_t o0 = g->prog[pcs[0]].u1;
    const char* after0 = first ? "" : " & (k0 > after)";
    const char* after1 = first ? "" : " & (k1 > after)";
    bput(g->b, "%*s{  // term: %sprimitive %u", indent, "", pos[0] ? "" : "NOT ", o0);
    if (q->npc > 1u) bput(g->b, " AND %sprimitive %u", pos[1] ? "" : "NOT ", g->prog[pcs[1]].u1);
    bput(g->b, "\n");
    const WoRec* P = &g->prog[pcs[0]];
    if (q->npc == 1u && pos[0] && P->u0 == 1u && g->prog[pcs[0] + 1u].op == WO_LEAF_SPHERE) {
        /* a lone sphere: its interval is [-b - s, -b + s] exactly when disc >= 0, so
         * its transitions are formed inside the branch that computes s */
        const WoRec* L = &g->prog[pcs[0] + 1u];
        uint32_t vl[4];
        for (int i = 0; i < 4; ++i) vl[i] = fbits(L->f[i]);
        bput(g->b,
             "%*s  WO_WK(WO_WORK_SPHERE_TESTS);\n"
             "%*s  float fx, fy, fz, b, ll, disc;\n"
             "%*s  asm(\"v_subrev_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(fx) : \"v\"(o.x));\n"
             "%*s  asm(\"v_subrev_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(fy) : \"v\"(o.y));\n"
             "%*s  asm(\"v_subrev_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(fz) : \"v\"(o.z));\n"
             "%*s  wodev::sphere_fbl(fx, fy, fz, d, b, ll);\n"
             "%*s  asm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(disc) : \"v\"(ll));\n"
             "%*s  if (__ballot(wodev::sphere_need(b, disc)) != 0ull) {\n"
             "%*s    asm volatile(\"\");\n"
             "#if WO_LONE_SEL  // every lane of the wave forms the interval; hd masks the candidates\n"
             "%*s    {\n"
             "%*s      const bool hd = !(disc < 0.0f);\n"
             "#else\n"
             "%*s    if (!(disc < 0.0f)) {\n"
             "%*s      const bool hd = true;\n"
             "#endif\n"
             "%*s      const float s = wodev::sqrt_pt(disc), nb = -b, la = nb - s, lb = nb + s;\n"
             "%*s      uint32_t ka, kb;\n"
             "%*s      asm volatile(\"s_mov_b32 %%0, 0x%08x\\n\\ts_mov_b32 %%1, 0x%08x\" : \"=s\"(ka), \"=s\"(kb));\n"
             "%*s      const uint64_t k0 = wodev::event_key_lo(la, ka), k1 = wodev::event_key_lo(lb, kb);\n",
             indent, "", indent, "", indent, "", vl[0], indent, "", vl[1], indent, "", vl[2], indent, "", indent, "",
             vl[3], indent, "", indent, "", indent, "", indent, "", indent, "", indent, "", indent, "", indent, "",
             indent, "", term_ka(o0, 1), term_kb(o0, 1), indent, "");
        if (first) bput(g->b, "%*s      cnt += (hd & (la <= tmin) & (lb > tmin)) ? 1u : 0u;\n", indent, "");
        bput(g->b,
             "%*s      WO_WK(WO_WORK_EVENTS);\n"
             "%*s      wodev::term_cand(k0, hd & (la > tmin)%s, best);\n"
             "%*s      wodev::term_cand(k1, hd & (lb > tmin) & (lb < wodev::kInf)%s, best);\n"
             "%*s    }\n%*s  }\n%*s}\n",
             indent, "", indent, "", after0, indent, "", after1, indent, "", indent, "", indent, "");
        return;
    }
    bput(g->b, "%*s  wodev::Ivl ia;\n", indent, "");
    gen_term_ivl(g, pcs[0], "ia", indent + 2);
    uint32_t vk[4] = {term_ka(o0, pos[0]), term_kb(o0, pos[0]), 0u, 0u};
    static const char* nk[4] = {"ka0", "kb0", "ka1", "kb1"};
    if (q->npc == 1u) {
        emit_consts(g->b, indent + 2, "uint32_t", nk, vk, 2);
        bput(g->b, "%*s  const wodev::TermLit x = wodev::term_lit(ia, ka0, kb0);\n", indent, "");
        if (first) bput(g->b, "%*s  cnt += %swodev::term_in0(x) ? 1u : 0u;\n", indent, "", pos[0] ? "" : "!");
        bput(g->b,
             "%*s  WO_WK(WO_WORK_EVENTS);\n"
             "%*s  wodev::term_cands1<%s>(x, after, best);\n%*s}\n",
             indent, "", indent, "", first ? "true" : "false", indent, "");
        return;
    }
    const uint32_t o1 = g->prog[pcs[1]].u1;
    vk[2] = term_ka(o1, pos[1]);
    vk[3] = term_kb(o1, pos[1]);
    /* a positive first literal empty along every lane's ray: the term is false throughout */
    if (pos[0])
        bput(g->b, "%*s  if (__ballot(!(ia.a > ia.b) & (ia.b > tmin)) != 0ull) {\n", indent, "");
    else
        bput(g->b, "%*s  {\n", indent, "");
    bput(g->b, "%*s    wodev::Ivl ib;\n", indent, "");
    gen_term_ivl(g, pcs[1], "ib", indent + 4);
    emit_consts(g->b, indent + 4, "uint32_t", nk, vk, 4);
    bput(g->b,
         "%*s    const wodev::TermLit x = wodev::term_lit(ia, ka0, kb0), y = wodev::term_lit(ib, ka1, kb1);\n",
         indent, "");
    if (first)
        bput(g->b, "%*s    cnt += (%swodev::term_in0(x) & %swodev::term_in0(y)) ? 1u : 0u;\n", indent, "",
             pos[0] ? "" : "!", pos[1] ? "" : "!");
    bput(g->b,
         "%*s    WO_WK(WO_WORK_EVENTS);\n"
         "%*s    wodev::term_cands_of<%s, %s, %s>(x, y, after, best);\n"
         "%*s    wodev::term_cands_of<%s, %s, %s>(y, x, after, best);\n"
         "%*s  }\n%*s}\n",
         indent, "", indent, "", pos[1] ? "true" : "false", first ? "true" : "false", o1 < o0 ? "true" : "false",
         indent, "", pos[0] ? "true" : "false", first ? "true" : "false", o0 < o1 ? "true" : "false", indent, "",
         indent, "");
}

/* ---- eval, flattened: literal sets as one masked compare ----
 * A conjunction of primitive literals (x and not-y terms, primitives of one bits
 * word) is true iff (bits & (P|N)) == P; a disjunction iff (bits & (P|N)) != N.
 * Unions / intersections / differences of such sets merge into one set, so a
 * union of k primitives costs one AND and one compare instead of 2k-1 bit ops;
 * the remaining combinations are bools, which the compiler keeps as wave lane
 * masks (SALU).  Same function of `bits` as gen_eval. */
typedef struct Term {
    /* kind 0: the named bool v; kind 1: v & conj(P, N); kind 2: v | disj(P, N),
     * v == kNoName meaning the literal set alone (an empty set is the identity).
     * dl: the same value as a decision list (1-based id, 0 = none); cost: the
     * rough VALU/SALU count of evaluating the term as written, for the choice
     * between the two forms when it is named. */
    int kind;
    uint32_t w, P, N, v;
    uint32_t dl, cost;
} Term;

enum { kNoName = 0xffffffffu };

/* ---- decision lists ----
 * A chain of set operations whose right operands are literal sets, e.g. the
 * left-deep ((((a u b) \ c) u d) \ e) ... of csg256_chain, is a decision list:
 * walking from the last operation down, a union operand that holds the point
 * decides "inside", a subtracted one "outside", an intersected one that does NOT
 * hold it "outside"; the first operand decides when nothing above it does.  When
 * the operands' primitive ordinals grow along the chain (postfix order does
 * that), the deciding entry is the highest set bit of
 * (bits ^ INV) & USED, and its value a bit of VAL at that position: one
 * count-leading-zeros and a shift per membership word instead of one mask
 * compare and one lane-mask operation per chain link. */
#define DL_WORDS 8
typedef struct DList {
    uint32_t used[DL_WORDS]; /* primitives in the list */
    uint32_t inv[DL_WORDS];  /* entry decides when its primitive does NOT hold the point */
    uint32_t val[DL_WORDS];  /* the value an entry decides */
    int dflt;                /* the value when no entry decides */
} DList;

static uint32_t dl_new(Gen* g) {
    if (g->ndl == g->dl_cap) {
        uint32_t cap = g->dl_cap ? 2u * g->dl_cap : 64u;
        DList* p = (DList*)realloc(g->dls, cap * sizeof(DList));
        if (!p) {
            g->err = 1;
            return 0;
        }
        g->dls = p;
        g->dl_cap = cap;
    }
    memset(&g->dls[g->ndl], 0, sizeof(DList));
    return ++g->ndl;
}

static int term_is_literal(const Term* t) {
    uint32_t m = t->P | t->N;
    return t->kind && t->v == kNoName && m && (m & (m - 1u)) == 0u;
}

/* t as a decision list for a join of `kind` (1 intersection, 2 union): its own,
 * or a literal set's (kind 2: any entry decides 1, else 0; kind 1: any entry
 * decides 0, else 1; a single literal takes the join's form) */
static uint32_t dl_of(Gen* g, const Term* t, int kind) {
    if (t->dl) return t->dl;
    if (!t->kind || t->v != kNoName || !(t->P | t->N) || t->w >= DL_WORDS) return 0;
    const int k = term_is_literal(t) ? kind : t->kind;
    uint32_t id = dl_new(g);
    if (!id) return 0;
    DList* d = &g->dls[id - 1u];
    d->used[t->w] = t->P | t->N;
    if (k == 2) {
        d->inv[t->w] = t->N;
        d->val[t->w] = t->P | t->N;
        d->dflt = 0;
    } else {
        d->inv[t->w] = t->P;
        d->dflt = 1;
    }
    return id;
}

/* the join of `kind` with `top` above `base`.  A union's top must be a plain
 * disjunction (every entry decides 1, default 0), an intersection's a plain
 * conjunction (every entry decides 0, default 1): then whenever an entry of top
 * decides, it decides the join.  Entries sit at their bit positions, so every
 * entry of base above the lowest of top's must already decide the same value
 * (their relative order then does not matter); otherwise no list. */
static uint32_t dl_merge(Gen* g, uint32_t base, uint32_t top, int kind) {
    if (!base || !top) return 0;
    const int v = kind == 2;
    const DList* t = &g->dls[top - 1u];
    const DList* b = &g->dls[base - 1u];
    if (t->dflt == v) return 0;
    uint32_t lo = 0xffffffffu;
    for (uint32_t w = 0; w < DL_WORDS; ++w) {
        if ((t->val[w] & t->used[w]) != (v ? t->used[w] : 0u)) return 0;
        if (b->used[w] & t->used[w]) return 0;
        if (t->used[w] && lo == 0xffffffffu) lo = 32u * w + (uint32_t)__builtin_ctz(t->used[w]);
    }
    if (lo == 0xffffffffu) return 0;
    for (uint32_t w = lo / 32u; w < DL_WORDS; ++w) {
        const uint32_t above = w > lo / 32u ? ~0u : (lo % 32u == 31u ? 0u : ~0u << (lo % 32u + 1u));
        if (b->used[w] & above & (v ? ~b->val[w] : b->val[w])) return 0;
    }
    uint32_t id = dl_new(g);
    if (!id) return 0;
    DList* d = &g->dls[id - 1u];
    *d = g->dls[base - 1u];
    t = &g->dls[top - 1u];
    for (uint32_t w = 0; w < DL_WORDS; ++w) {
        d->used[w] |= t->used[w];
        d->inv[w] |= t->inv[w];
        d->val[w] |= t->val[w];
    }
    return id;
}

static uint32_t dl_not(Gen* g, uint32_t id) {
    if (!id) return 0;
    uint32_t n = dl_new(g);
    if (!n) return 0;
    DList* d = &g->dls[n - 1u];
    *d = g->dls[id - 1u];
    for (uint32_t w = 0; w < DL_WORDS; ++w) d->val[w] ^= d->used[w];
    d->dflt ^= 1;
    return n;
}

static uint32_t dl_cost(const Gen* g, uint32_t id) {
    const DList* d = &g->dls[id - 1u];
    uint32_t c = 1;
    for (uint32_t w = 0; w < DL_WORDS; ++w)
        if (d->used[w]) c += 6u;
    return c;
}

/* the list as a named bool: words from the lowest (least priority) up, each
 * overriding the value where one of its entries decides */
static uint32_t dl_name(Gen* g, uint32_t id, int indent) {
    const DList* d = &g->dls[id - 1u];
    uint32_t v = g->nval++;
    bput(g->b, "%*sbool v%u = %s;  // decision list\n", indent, "", v, d->dflt ? "true" : "false");
    for (uint32_t w = 0; w < DL_WORDS; ++w) {
        const uint32_t u = d->used[w];
        if (!u) continue;
        char x[96];
        if (d->inv[w])
            snprintf(x, sizeof x, "((bits[%u] ^ 0x%08xu) & 0x%08xu)", w, d->inv[w], u);
        else if (u != ~0u)
            snprintf(x, sizeof x, "(bits[%u] & 0x%08xu)", w, u);
        else
            snprintf(x, sizeof x, "bits[%u]", w);
        const uint32_t vals = d->val[w] & u;
        if (vals == u)
            bput(g->b, "%*sv%u = v%u | (%s != 0u);\n", indent, "", v, v, x);
        else if (vals == 0u)
            bput(g->b, "%*sv%u = v%u & (%s == 0u);\n", indent, "", v, v, x);
        else
            bput(g->b,
                 "%*s{ const uint32_t dw = %s; v%u = dw != 0u ? (int)(0x%08xu << __builtin_clz(dw)) < 0 : v%u; }\n",
                 indent, "", x, v, vals, v);
    }
    return v;
}

/* the literal set of t (kind 1/2) as a named bool */
static uint32_t lits_name(Gen* g, const Term* t, int indent) {
    uint32_t v = g->nval++;
    bput(g->b, "%*sconst bool v%u = (bits[%u] & 0x%08xu) %s 0x%08xu;\n", indent, "", v, t->w, t->P | t->N,
         t->kind == 1 ? "==" : "!=", t->kind == 1 ? t->P : t->N);
    return v;
}

static uint32_t bool_op(Gen* g, uint32_t x, uint32_t y, int kind, int indent) {
    if (x == kNoName) return y;
    if (y == kNoName) return x;
    uint32_t v = g->nval++;
    bput(g->b, "%*sconst bool v%u = v%u %s v%u;\n", indent, "", v, x, kind == 1 ? "&" : "|", y);
    return v;
}

static uint32_t term_name(Gen* g, const Term* t, int indent) {
    if (t->kind == 0) return t->v;
    const uint32_t m = t->P | t->N;
    /* the decision list where it is cheaper than the term as written (a literal
     * set adds an AND, a compare and a lane-mask operation) */
    if (t->dl && dl_cost(g, t->dl) < t->cost + (m ? 3u : 0u)) return dl_name(g, t->dl, indent);
    if (m == 0u) {
        if (t->v != kNoName) return t->v;
        uint32_t v = g->nval++;
        bput(g->b, "%*sconst bool v%u = %s;\n", indent, "", v, t->kind == 1 ? "true" : "false");
        return v;
    }
    return bool_op(g, t->v, lits_name(g, t, indent), t->kind, indent);
}

/* not(v & C) = !v | not C; not(v | D) = !v & not D */
static Term term_not(Gen* g, Term t, int indent) {
    uint32_t nv = kNoName;
    if (t.v != kNoName) {
        nv = g->nval++;
        bput(g->b, "%*sconst bool v%u = !v%u;\n", indent, "", nv, t.v);
    }
    const uint32_t dl = dl_not(g, t.dl), cost = t.cost + (nv != kNoName);
    if (t.kind == 0) {
        Term r = {0, 0, 0, 0, nv, dl, cost};
        return r;
    }
    Term r = {t.kind == 1 ? 2 : 1, t.w, t.N, t.P, nv, dl, cost};
    return r;
}

/* kind 1: intersection, kind 2: union.  Literal sets of one bits word merge. */
static Term term_join(Gen* g, Term a, Term b, int kind, int indent) {
    /* the decision-list form: either operand as the list, the other (a literal
     * set) on top of it */
    const uint32_t da = dl_of(g, &a, kind), db = dl_of(g, &b, kind);
    uint32_t dl = dl_merge(g, da, db, kind);
    if (!dl) dl = dl_merge(g, db, da, kind);
    const uint32_t nval0 = g->nval;
    Term x[2] = {a, b};
    for (int i = 0; i < 2; ++i) {
        if (x[i].kind == kind) continue;
        if (term_is_literal(&x[i])) {
            x[i].kind = kind;
            continue;
        }
        uint32_t v = term_name(g, &x[i], indent);
        Term n = {kind, 0, 0, 0, v, 0, 0};
        x[i] = n;
    }
    Term r = {kind, x[0].w, x[0].P, x[0].N, kNoName, 0, 0};
    uint32_t m0 = x[0].P | x[0].N, m1 = x[1].P | x[1].N;
    uint32_t extra = kNoName;
    if (!m0) {
        r.w = x[1].w, r.P = x[1].P, r.N = x[1].N;
    } else if (m1 && (x[1].w != x[0].w || (m0 & m1))) {
        extra = lits_name(g, &x[1], indent);
    } else {
        r.P |= x[1].P, r.N |= x[1].N;
    }
    r.v = bool_op(g, bool_op(g, x[0].v, x[1].v, kind, indent), extra, kind, indent);
    r.dl = dl;
    r.cost = a.cost + b.cost + 2u * (g->nval - nval0);
    return r;
}

static Term gen_eval_flat(Gen* g, uint32_t start, uint32_t end, int indent) {
    Term stack[64], none = {0, 0, 0, 0, 0, 0, 0};
    int sp = 0;
    uint32_t pc = start;
    while (pc < end && !g->err) {
        const WoRec* r = &g->prog[pc];
        if (sp >= 64) {
            g->err = 1;
            return none;
        }
        if (r->op == WO_OP_BOUND && !bound_tested(g, pc)) {
            ++pc;
        } else if (r->op == WO_OP_BOUND) {
            uint32_t k = g->nbound++;
            Term t = {0, 0, 0, 0, g->nval++, 0, 1};
            bput(g->b, "%*sbool v%u = false;\n%*sif (!(cull[%u] & %uu)) {\n", indent, "", t.v, indent, "", k / 32,
                 1u << (k % 32));
            Term inner = gen_eval_flat(g, pc + 1, r->u0, indent + 2);
            {
                /* the cost of the form term_name picks, plus the cull test */
                const uint32_t lits = inner.kind && (inner.P | inner.N) ? 3u : 0u;
                const uint32_t dc = inner.dl ? dl_cost(g, inner.dl) : 0xffffffffu;
                t.cost = 1u + (dc < inner.cost + lits ? dc : inner.cost + lits);
            }
            uint32_t iv = term_name(g, &inner, indent + 2);
            bput(g->b, "%*s  v%u = v%u;\n%*s}\n", indent, "", t.v, iv, indent, "");
            stack[sp++] = t;
            pc = r->u0;
        } else if (r->op == WO_OP_PRIM) {
            Term t = {1, r->u1 / 32u, 1u << (r->u1 % 32u), 0u, kNoName, 0, 0};
            stack[sp++] = t;
            pc += 1 + r->u0;
        } else {
            if (sp < 2) {
                g->err = 1;
                return none;
            }
            Term B = stack[--sp], A = stack[--sp];
            if (r->op == WO_OP_UNION)
                stack[sp++] = term_join(g, A, B, 2, indent);
            else if (r->op == WO_OP_INTER)
                stack[sp++] = term_join(g, A, B, 1, indent);
            else if (r->op == WO_OP_DIFF)
                stack[sp++] = term_join(g, A, term_not(g, B, indent), 1, indent);
            else /* RDIFF: B & ~A */
                stack[sp++] = term_join(g, B, term_not(g, A, indent), 1, indent);
            ++pc;
        }
    }
    if (sp != 1) {
        g->err = 1;
        return none;
    }
    return stack[0];
}

/* ---- incremental union count ----
 * When the root is a union of literal sets (each a conjunction or disjunction of
 * primitive literals of one membership word), an event toggles one primitive,
 * and only the one term holding that primitive can change: the sweep keeps the
 * number of true terms and updates it from that term before and after the
 * toggle (a table lookup and two mask compares), instead of re-evaluating every
 * term per event.  The root is inside iff the count is > 0.  csg256_balanced's
 * union of 65 pair terms is the case this is for. */
typedef struct LSet {
    int type;        /* 0 other, 1 literal set, 2 union of terms */
    int kind;        /* literal set: 1 conj, 2 disj (a single literal is either) */
    uint32_t w;      /* literal set: first membership word of its 64-bit window */
    uint64_t P, N;   /* literal set: bit i = primitive 32 w + i */
} LSet;

typedef struct UTerm {
    uint32_t w, neg; /* true iff ((window(w) & m) == q) != neg, window(w) = bits[w] | bits[w + 1] << 32 */
    uint64_t m, q;
} UTerm;

static int lset_single(const LSet* a) {
    uint64_t m = a->P | a->N;
    return m && (m & (m - 1u)) == 0u;
}

static LSet lset_not(LSet a) {
    LSet r = a;
    r.kind = a.kind == 1 ? 2 : 1;
    r.P = a.N;
    r.N = a.P;
    return r;
}

static void uterm_add(UTerm* t, uint32_t* nt, uint32_t cap, const LSet* a, int* ok) {
    if (*nt >= cap) {
        *ok = 0;
        return;
    }
    UTerm u;
    u.w = a->w;
    u.m = a->P | a->N;
    if (a->kind == 1 || lset_single(a)) {
        u.q = a->P; /* conj: every P set, every N clear */
        u.neg = 0;
    } else {
        u.q = a->N; /* disj: not (every P clear and every N set) */
        u.neg = 1;
    }
    t[(*nt)++] = u;
}

/* join of two literal sets into one (kind 1 conj / 2 disj), when they fit one
 * 64-bit window of the membership words */
static int lset_merge(const LSet* a, const LSet* b, int kind, LSet* r) {
    if (a->type != 1 || b->type != 1) return 0;
    if ((a->kind != kind && !lset_single(a)) || (b->kind != kind && !lset_single(b))) return 0;
    const LSet* lo = a->w <= b->w ? a : b;
    const LSet* hi = a->w <= b->w ? b : a;
    const uint32_t sh = 32u * (hi->w - lo->w);
    if (sh > 32u || (sh && ((hi->P | hi->N) >> (64u - sh)) != 0u)) return 0;
    const uint64_t hp = hi->P << sh, hn = hi->N << sh;
    if ((lo->P | lo->N) & (hp | hn)) return 0;
    r->type = 1;
    r->kind = kind;
    r->w = lo->w;
    r->P = lo->P | hp;
    r->N = lo->N | hn;
    /* a set whose low word is empty moves its window up */
    if (r->w + 1u && ((r->P | r->N) & 0xffffffffull) == 0u) {
        r->w += 1u;
        r->P >>= 32;
        r->N >>= 32;
    }
    return 1;
}

/* the root's terms when it is a union of literal sets (0 terms otherwise) */
static uint32_t union_terms(const WoRec* prog, uint32_t n_recs, uint32_t n_prims, UTerm* terms, uint32_t cap) {
    LSet st[256];
    uint32_t sp = 0, nt = 0;
    int ok = 1;
    for (uint32_t pc = 0; pc < n_recs && ok;) {
        const WoRec* r = &prog[pc];
        if (r->op == WO_OP_BOUND) {
            ++pc;
            continue;
        }
        if (r->op == WO_OP_PRIM) {
            if (sp == 256u) return 0;
            LSet a = {1, 1, r->u1 / 32u, 1ull << (r->u1 % 32u), 0u};
            st[sp++] = a;
            pc += 1u + r->u0;
            continue;
        }
        if (sp < 2u) return 0;
        LSet b = st[--sp], a = st[--sp], res = {0, 0, 0, 0, 0};
        if (r->op == WO_OP_UNION) {
            if (!lset_merge(&a, &b, 2, &res)) {
                if (a.type == 0 || b.type == 0) {
                    res.type = 0;
                } else {
                    if (a.type == 1) uterm_add(terms, &nt, cap, &a, &ok);
                    if (b.type == 1) uterm_add(terms, &nt, cap, &b, &ok);
                    res.type = 2;
                }
            }
        } else if (a.type == 1 && b.type == 1) {
            LSet x = a, y = b;
            if (r->op == WO_OP_DIFF) y = lset_not(b);
            if (r->op == WO_OP_RDIFF) {
                x = b;
                y = lset_not(a);
            }
            if (!lset_merge(&x, &y, 1, &res)) res.type = 0;
        }
        st[sp++] = res;
        ++pc;
    }
    if (!ok || sp != 1u || st[0].type != 2) return 0;
    /* every primitive in exactly one term */
    uint32_t seen = 0;
    for (uint32_t i = 0; i < nt; ++i) seen += (uint32_t)__builtin_popcountll(terms[i].m);
    return seen == n_prims ? nt : 0u;
}

/* The root's membership when only primitive p holds the point: the postfix
 * program evaluated over bits = {p} (BOUND records do not change values). */
static int single_root(const WoRec* prog, uint32_t n_recs, uint32_t p) {
    uint8_t st[512];
    uint32_t sp = 0;
    for (uint32_t pc = 0; pc < n_recs;) {
        const WoRec* r = &prog[pc];
        if (r->op == WO_OP_PRIM) {
            if (sp == sizeof st) return -1;
            st[sp++] = r->u1 == p;
            pc += 1u + r->u0;
            continue;
        }
        if (r->op != WO_OP_BOUND) {
            if (sp < 2u) return -1;
            const uint8_t B = st[--sp], A = st[sp - 1u];
            st[sp - 1u] = r->op == WO_OP_UNION   ? (A | B)
                          : r->op == WO_OP_INTER ? (A & B)
                          : r->op == WO_OP_DIFF  ? (A & !B)
                                                 : (B & !A);
        }
        ++pc;
    }
    return sp == 1u ? st[0] : -1;
}

/* Depth of the CSG tree over primitives (a primitive is depth 0). */
static uint32_t tree_depth(const WoRec* prog, uint32_t n_recs) {
    uint32_t stack[256];
    uint32_t sp = 0, best = 0;
    for (uint32_t pc = 0; pc < n_recs;) {
        const WoRec* r = &prog[pc];
        if (r->op == WO_OP_PRIM) {
            if (sp == 256u) return 1000u; /* deeper than any window choice cares about */
            stack[sp++] = 0u;
            pc += 1u + r->u0;
        } else if (r->op == WO_OP_BOUND) {
            ++pc;
        } else {
            if (sp < 2u) return 0u;
            uint32_t b = stack[--sp], a = stack[sp - 1u];
            uint32_t d = 1u + (a > b ? a : b);
            stack[sp - 1u] = d;
            best = d > best ? d : best;
            ++pc;
        }
    }
    return best;
}

/* The sweep for a root that is a union of literal-set terms (union_terms): the
 * number of true terms at t_min (every term once; a culled BOUND's primitives
 * stay 0, their true membership along the ray), then per event the toggled
 * primitive's term before and after the toggle.  The root flips exactly when
 * the count moves between 0 and non-zero. */
static void gen_union_sweep(Gen* g, const UTerm* uterms, uint32_t n_uterms, uint32_t n_recs, uint32_t nw) {
    Buf* b = g->b;
    bput(b,
         "    int ucnt = 0;  // true terms of the root's union\n"
         "    if (!have) {\n"
         "      uint32_t r;\n"
         "      // WO_EVAL_BEGIN (the root's value from bits[] and cull[]; tests/test_jit.py compiles it on the host)\n"
         "      {\n"
         "        int c = 0;\n");
    /* terms that are one primitive: a population count per word (as separate
     * compares the compiler extracted every bit first and spilled them) */
    uint32_t single[64] = {0};
    for (uint32_t i = 0; i < n_uterms; ++i) {
        const UTerm* u = &uterms[i];
        if (u->m == u->q && (u->m & (u->m - 1u)) == 0u && !u->neg) {
            const uint32_t bit = 32u * u->w + (uint32_t)__builtin_ctzll(u->m);
            if (bit / 32u < 64u) single[bit / 32u] |= 1u << (bit % 32u);
        }
    }
    for (uint32_t w = 0; w < nw && w < 64u; ++w)
        if (single[w]) bput(b, "        c += __builtin_popcount(bits[%u] & 0x%08xu);\n", w, single[w]);
    for (uint32_t i = 0; i < n_uterms; ++i) {
        const UTerm* u = &uterms[i];
        if (u->m == u->q && (u->m & (u->m - 1u)) == 0u && !u->neg) {
            const uint32_t bit = 32u * u->w + (uint32_t)__builtin_ctzll(u->m);
            if (bit / 32u < 64u) continue;
        }
        const uint32_t mlo = (uint32_t)u->m, mhi = (uint32_t)(u->m >> 32);
        const uint32_t qlo = (uint32_t)u->q, qhi = (uint32_t)(u->q >> 32);
        if (!mhi)
            bput(b, "        c += (int)((bits[%u] & 0x%08xu) %s 0x%08xu);\n", u->w, mlo, u->neg ? "!=" : "==", qlo);
        else
            bput(b, "        c += (int)((((bits[%u] & 0x%08xu) == 0x%08xu) & ((bits[%u] & 0x%08xu) == 0x%08xu)) != %s);\n",
                 u->w, mlo, qlo, u->w + 1u, mhi, qhi, u->neg ? "true" : "false");
    }
    bput(b,
         "        ucnt = c;\n"
         "        r = c != 0 ? 1u : 0u;\n"
         "      }\n"
         "      // WO_EVAL_END\n"
         "      (void)r;\n"
         "    }\n"
         "    for (;;) {\n"
         "      if (!win.next(key)) {  // key keeps the last processed event\n"
         "        if (!win.dropped()) return false;\n"
         "        after = key;\n"
         "        WO_WK(WO_WORK_RECOLLECTS);\n"
         "        win.clear();\n"
         "        {\n");
    g->first_pass = 0;
    gen_collect_all(g, 10);
    bput(b,
         "        }\n"
         "        if (!win.next(key)) return false;\n"
         "      }\n"
         "      WO_WK(WO_WORK_SWEEP_STEPS);\n"
         "      WO_WK_WAVE(WO_WORK_SWEEP_TRIPS);\n"
         "      bool was;\n"
         "      // WO_TOGGLE_BEGIN (the event's membership toggle; tests/test_jit.py)\n"
         "      {\n"
         "        const uint32_t ord = ((uint32_t)key) >> 12;\n"
         "        const uint32_t w = ord >> 5, m = 1u << (ord & 31u);\n"
         "        const WoUTerm t = WO_UTERM[ord];\n");
    if (nw == 1u) {
        bput(b, "        const uint64_t cw = bits[0];\n");
    } else {
        bput(b, "        const uint32_t clo = ");
        for (uint32_t w = 0; w + 1u < nw; ++w) bput(b, "t.w == %uu ? bits[%u] : ", w, w);
        bput(b, "bits[%u];\n        const uint32_t chi = ", nw - 1u);
        for (uint32_t w = 0; w + 2u < nw; ++w) bput(b, "t.w == %uu ? bits[%u] : ", w, w + 1u);
        bput(b, "bits[%u];\n        const uint64_t cw = ((uint64_t)chi << 32) | clo;\n", nw - 1u);
    }
    bput(b,
         "        const uint64_t tm = 1ull << (ord - 32u * t.w);\n"
         "        const bool tb = ((cw & t.m) == t.q) != (t.neg != 0u);\n"
         "        const bool ta = (((cw ^ tm) & t.m) == t.q) != (t.neg != 0u);\n"
         "        was = ucnt != 0;\n"
         "        ucnt += (int)ta - (int)tb;\n");
    for (uint32_t w = 0; w < nw; ++w) bput(b, "        bits[%u] ^= w == %uu ? m : 0u;\n", w, w);
    bput(b,
         "      }\n"
         "      // WO_TOGGLE_END\n"
         "      if ((ucnt != 0) != was) { wodev::hit_from_key(key, ucnt != 0 ? 1u : 0u, hit); return true; }\n"
         "    }\n"
         "  }\n"
         "};\n");
}

/* ---- root evaluation by truth tables ----
 * A small general tree (no union count, no term mode) splits into K <= 4
 * subtrees of <= 12 primitives each, every one a contiguous ordinal range
 * (postfix order numbers a subtree's primitives consecutively).  A subtree's
 * value is one bit of its truth table (2^n bits, indexed by its range of the
 * membership words) and the root one bit of a 2^K-entry table over the K
 * subtree values: per event K table reads from LDS and a shift, instead of the
 * tree's masked compares and lane-mask operations (csg32_nested: two subtrees of
 * 9 and 10 primitives). */
#define LUT_MAX_BITS 12u
#define LUT_MAX_SUBS 4u
typedef struct TNode {
    int op; /* 0 primitive, else WO_OP_UNION / _INTER / _DIFF / _RDIFF */
    int l, r;
    uint32_t lo, n; /* ordinal range [lo, lo + n) */
} TNode;

typedef struct LutPlan {
    uint32_t k;                    /* subtrees */
    uint32_t lo[LUT_MAX_SUBS], n[LUT_MAX_SUBS], off[LUT_MAX_SUBS];
    int node[LUT_MAX_SUBS];
    uint32_t words;                /* table words in all */
    uint32_t top;                  /* bit j: the root when subtree s has value (j >> s) & 1 */
    uint32_t* table;
} LutPlan;

static int tn_eval(const TNode* t, int x, uint32_t lo, uint32_t idx, const LutPlan* pl, uint32_t j) {
    if (pl) /* a subtree of the plan: its value from j */
        for (uint32_t s = 0; s < pl->k; ++s)
            if (pl->node[s] == x) return (int)((j >> s) & 1u);
    const TNode* n = &t[x];
    if (n->op == 0) return (int)((idx >> (n->lo - lo)) & 1u);
    const int a = tn_eval(t, n->l, lo, idx, pl, j), b = tn_eval(t, n->r, lo, idx, pl, j);
    return n->op == WO_OP_UNION ? (a | b) : n->op == WO_OP_INTER ? (a & b) : n->op == WO_OP_DIFF ? (a & !b) : (b & !a);
}

static int lut_split(const TNode* t, int x, LutPlan* pl) {
    if (t[x].n <= LUT_MAX_BITS) {
        if (pl->k == LUT_MAX_SUBS) return 0;
        pl->node[pl->k] = x;
        pl->lo[pl->k] = t[x].lo;
        pl->n[pl->k] = t[x].n;
        ++pl->k;
        return 1;
    }
    return lut_split(t, t[x].l, pl) && lut_split(t, t[x].r, pl);
}

/* 1 with *pl filled (pl->table malloc'd), 0 when the tree does not split so */
static int lut_plan(const WoRec* prog, uint32_t n_recs, uint32_t n_prims, LutPlan* pl) {
    memset(pl, 0, sizeof *pl);
    if (n_prims == 0u || n_prims > 64u) return 0;
    TNode* t = (TNode*)malloc(sizeof(TNode) * (2u * n_prims));
    int* st = (int*)malloc(sizeof(int) * (n_prims + 1u));
    uint32_t nt = 0, sp = 0;
    int ok = t && st;
    for (uint32_t pc = 0; pc < n_recs && ok;) {
        const WoRec* r = &prog[pc];
        if (r->op == WO_OP_PRIM) {
            ok = nt < 2u * n_prims && sp <= n_prims;
            if (!ok) break;
            TNode x = {0, -1, -1, r->u1, 1u};
            t[nt] = x;
            st[sp++] = (int)nt++;
            pc += 1u + r->u0;
            continue;
        }
        ++pc;
        if (r->op == WO_OP_BOUND) continue;
        ok = sp >= 2u && nt < 2u * n_prims;
        if (!ok) break;
        const int b = st[--sp], a = st[--sp];
        TNode x = {(int)r->op, a, b, t[a].lo < t[b].lo ? t[a].lo : t[b].lo, t[a].n + t[b].n};
        ok = t[a].lo + t[a].n == t[b].lo || t[b].lo + t[b].n == t[a].lo; /* contiguous ranges */
        t[nt] = x;
        st[sp++] = (int)nt++;
    }
    ok = ok && sp == 1u && t[st[0]].lo == 0u && t[st[0]].n == n_prims && lut_split(t, st[0], pl) && pl->k >= 1u;
    for (uint32_t s = 0; ok && s < pl->k; ++s) {
        ok = (pl->lo[s] % 32u) + pl->n[s] <= 64u && pl->lo[s] / 32u + ((pl->lo[s] % 32u) + pl->n[s] > 32u) < 2u;
        pl->off[s] = pl->words;
        pl->words += pl->n[s] >= 5u ? 1u << (pl->n[s] - 5u) : 1u;
    }
    if (ok) {
        pl->table = (uint32_t*)calloc(pl->words, sizeof(uint32_t));
        ok = pl->table != NULL;
    }
    for (uint32_t s = 0; ok && s < pl->k; ++s)
        for (uint32_t idx = 0; idx < (1u << pl->n[s]); ++idx)
            if (tn_eval(t, pl->node[s], pl->lo[s], idx, NULL, 0u)) pl->table[pl->off[s] + (idx >> 5)] |= 1u << (idx & 31u);
    for (uint32_t j = 0; ok && j < (1u << pl->k); ++j)
        if (tn_eval(t, st[0], 0u, 0u, pl, j)) pl->top |= 1u << j;
    free(t);
    free(st);
    if (!ok) {
        free(pl->table);
        memset(pl, 0, sizeof *pl);
    }
    return ok;
}

/* the root's value r from bits[] through the tables (WO_LUT: the LDS copy) */
static void lut_emit_eval(Buf* b, const LutPlan* pl, int indent) {
    bput(b, "%*suint32_t lsub = 0u;\n", indent, "");
    for (uint32_t s = 0; s < pl->k; ++s) {
        const uint32_t w = pl->lo[s] / 32u, sh = pl->lo[s] % 32u, n = pl->n[s];
        char idx[160];
        if (sh + n <= 32u)
            snprintf(idx, sizeof idx, "(bits[%u] >> %u) & 0x%xu", w, sh, (1u << n) - 1u);
        else
            snprintf(idx, sizeof idx, "(uint32_t)((((uint64_t)bits[%u] << 32) | bits[%u]) >> %u) & 0x%xu", w + 1u, w, sh,
                     (1u << n) - 1u);
        if (n >= 5u)
            bput(b, "%*s{ const uint32_t i = %s; lsub |= ((WO_LUT[%uu + (i >> 5)] >> (i & 31u)) & 1u) << %u; }\n",
                 indent, "", idx, pl->off[s], s);
        else
            bput(b, "%*s{ const uint32_t i = %s; lsub |= ((0x%08xu >> i) & 1u) << %u; }\n", indent, "", idx,
                 pl->table[pl->off[s]], s);
    }
    bput(b, "%*sr = (0x%08xu >> lsub) & 1u;  // the root from the %u subtree values\n", indent, "", pl->top, pl->k);
}

/* ---- root evaluation by levels of truth tables (larger general trees) ----
 * A general tree too big for lut_plan (csg360_nested: 309 primitives under 308
 * unions, intersections and differences) is cut in levels: level 1's units are
 * the maximal subtrees of <= HLUT_MAX_BITS primitives, level l + 1's the maximal
 * subtrees of <= HLUT_MAX_BITS level-l units, up to the root, a unit of its own.
 * A unit's value is one bit of its truth table indexed by its lower units'
 * values (a contiguous range of them: they are numbered left to right), so an
 * event updates one unit per level -- its primitive's, then that unit's parent
 * unit, ... -- instead of re-evaluating the tree: per level one LDS read of the
 * lower index's entry (its unit, the unit's range and table offset) and one of
 * the table.  The same event order and values as the flat evaluation, so the
 * hit is the same key bit for bit. */
#define HLUT_MAX_BITS 8u
#define HLUT_MAX_LEVELS 4u
#define HLUT_MAX_WORDS 1024u /* table words: 10-bit offsets in an entry */
typedef struct HPlan {
    uint32_t L;                       /* levels; level L has one unit, the root */
    uint32_t k[HLUT_MAX_LEVELS];      /* units per level */
    uint32_t base[HLUT_MAX_LEVELS];   /* level's first entry in info[] (one per lower index) */
    uint32_t ubase[HLUT_MAX_LEVELS];  /* level's first unit in ulo / un / uoff */
    uint32_t *info, ninfo;            /* unit | lo << 8 | n << 18 | off << 22 */
    uint32_t *ulo, *un, *uoff, nunits;
    uint32_t *table, words;
} HPlan;

static void hplan_free(HPlan* h) {
    free(h->info);
    free(h->ulo);
    free(h->un);
    free(h->uoff);
    free(h->table);
    memset(h, 0, sizeof *h);
}

/* units below x at the current level (unit_of[y] >= 0: y roots lower unit unit_of[y]);
 * *gap is set when the two operands' units are not adjacent ranges (a unit's table
 * is indexed by the contiguous range [first, first + cnt) of the lower level) */
static uint32_t h_count(const TNode* t, int x, const int* unit_of, uint32_t* cnt, uint32_t* first, int* gap) {
    if (unit_of[x] >= 0) {
        cnt[x] = 1u;
        first[x] = (uint32_t)unit_of[x];
        return 1u;
    }
    const int l = t[x].l, r = t[x].r;
    const uint32_t a = h_count(t, l, unit_of, cnt, first, gap), b = h_count(t, r, unit_of, cnt, first, gap);
    cnt[x] = a + b;
    first[x] = first[l] < first[r] ? first[l] : first[r];
    if (first[l] + cnt[l] != first[r] && first[r] + cnt[r] != first[l]) *gap = 1;
    return a + b;
}

static int h_eval(const TNode* t, int x, const int* unit_of, uint32_t lo, uint32_t idx) {
    if (unit_of[x] >= 0) return (int)((idx >> ((uint32_t)unit_of[x] - lo)) & 1u);
    const TNode* n = &t[x];
    const int a = h_eval(t, n->l, unit_of, lo, idx), b = h_eval(t, n->r, unit_of, lo, idx);
    return n->op == WO_OP_UNION ? (a | b) : n->op == WO_OP_INTER ? (a & b) : n->op == WO_OP_DIFF ? (a & !b) : (b & !a);
}

/* the maximal subtrees of <= HLUT_MAX_BITS units, in lower-index order */
static void h_split(const TNode* t, int x, const uint32_t* cnt, const uint32_t* first, int* roots, uint32_t* nr) {
    if (cnt[x] <= HLUT_MAX_BITS) {
        roots[(*nr)++] = x;
        return;
    }
    const int a = t[x].l, b = t[x].r;
    const int lo_first = first[a] <= first[b];
    h_split(t, lo_first ? a : b, cnt, first, roots, nr);
    h_split(t, lo_first ? b : a, cnt, first, roots, nr);
}

static int hlut_plan(const WoRec* prog, uint32_t n_recs, uint32_t n_prims, HPlan* h) {
    memset(h, 0, sizeof *h);
    if (n_prims < 2u || n_prims > 1023u) return 0;
    const uint32_t cap = 2u * n_prims;
    TNode* t = (TNode*)malloc(sizeof(TNode) * cap);
    int* st = (int*)malloc(sizeof(int) * (n_prims + 1u));
    int* unit_of = (int*)malloc(sizeof(int) * cap);
    int* roots = (int*)malloc(sizeof(int) * cap);
    uint32_t* cnt = (uint32_t*)malloc(sizeof(uint32_t) * cap);
    uint32_t* first = (uint32_t*)malloc(sizeof(uint32_t) * cap);
    h->info = (uint32_t*)malloc(sizeof(uint32_t) * (n_prims + HLUT_MAX_LEVELS * 256u));
    /* (at most 255 units per level) */
    h->ulo = (uint32_t*)malloc(sizeof(uint32_t) * HLUT_MAX_LEVELS * 256u);
    h->un = (uint32_t*)malloc(sizeof(uint32_t) * HLUT_MAX_LEVELS * 256u);
    h->uoff = (uint32_t*)malloc(sizeof(uint32_t) * HLUT_MAX_LEVELS * 256u);
    h->table = (uint32_t*)calloc(HLUT_MAX_WORDS, sizeof(uint32_t));
    int ok = t && st && unit_of && roots && cnt && first && h->info && h->ulo && h->un && h->uoff && h->table;
    uint32_t nt = 0, sp = 0;
    for (uint32_t pc = 0; pc < n_recs && ok;) {
        const WoRec* r = &prog[pc];
        if (r->op == WO_OP_PRIM) {
            ok = nt < cap && sp <= n_prims && r->u1 < n_prims;
            if (!ok) break;
            TNode x = {0, -1, -1, r->u1, 1u};
            t[nt] = x;
            st[sp++] = (int)nt++;
            pc += 1u + r->u0;
            continue;
        }
        ++pc;
        if (r->op == WO_OP_BOUND) continue;
        ok = sp >= 2u && nt < cap;
        if (!ok) break;
        const int b = st[--sp], a = st[--sp];
        TNode x = {(int)r->op, a, b, t[a].lo < t[b].lo ? t[a].lo : t[b].lo, t[a].n + t[b].n};
        /* the operands' primitives must be adjacent ranges of ordinals, as lut_plan
         * requires (the scene compiler numbers them in postfix order); another
         * numbering falls back to the decision lists or the lanes */
        ok = t[a].lo + t[a].n == t[b].lo || t[b].lo + t[b].n == t[a].lo;
        t[nt] = x;
        st[sp++] = (int)nt++;
    }
    ok = ok && sp == 1u && t[st[0]].lo == 0u && t[st[0]].n == n_prims;
    const int root = ok ? st[0] : 0;
    /* level 0's units: the primitives (their ordinals) */
    for (uint32_t x = 0; ok && x < nt; ++x) unit_of[x] = t[x].op == 0 ? (int)t[x].lo : -1;
    uint32_t nlow = n_prims;
    while (ok) {
        if (h->L == HLUT_MAX_LEVELS) {
            ok = 0;
            break;
        }
        const uint32_t L = h->L;
        int gap = 0;
        h_count(t, root, unit_of, cnt, first, &gap);
        if (gap) {
            ok = 0;
            break;
        }
        uint32_t k = 0;
        h_split(t, root, cnt, first, roots, &k);
        ok = k >= 1u && k <= 255u;
        h->k[L] = k;
        h->base[L] = h->ninfo;
        h->ubase[L] = h->nunits;
        for (uint32_t j = 0; ok && j < k; ++j) {
            const int x = roots[j];
            const uint32_t lo = first[x], n = cnt[x];
            const uint32_t w = n >= 5u ? 1u << (n - 5u) : 1u;
            ok = lo < 1024u && h->words + w <= HLUT_MAX_WORDS && lo + n <= nlow;
            if (!ok) break;
            const uint32_t off = h->words;
            h->words += w;
            for (uint32_t idx = 0; idx < (1u << n); ++idx)
                if (h_eval(t, x, unit_of, lo, idx)) h->table[off + (idx >> 5)] |= 1u << (idx & 31u);
            for (uint32_t i = lo; i < lo + n; ++i) h->info[h->ninfo + i] = j | (lo << 8) | (n << 18) | (off << 22);
            h->ulo[h->nunits] = lo;
            h->un[h->nunits] = n;
            h->uoff[h->nunits] = off;
            ++h->nunits;
        }
        if (!ok) break;
        h->ninfo += nlow;
        ++h->L;
        if (k == 1u) break; /* the root */
        for (uint32_t x = 0; x < nt; ++x) unit_of[x] = -1;
        for (uint32_t j = 0; j < k; ++j) unit_of[roots[j]] = (int)j;
        nlow = k;
    }
    free(t);
    free(st);
    free(unit_of);
    free(roots);
    free(cnt);
    free(first);
    if (!ok) hplan_free(h);
    return ok;
}

/* index bits [lo, lo + n) of the words vec[0..nwv) into `idx` (static lo) */
static void h_emit_extract_static(Buf* b, const char* vec, uint32_t nwv, uint32_t lo, uint32_t n, int indent) {
    const uint32_t w = lo / 32u, sh = lo % 32u;
    if (sh + n <= 32u || w + 1u >= nwv)
        bput(b, "%*sidx = (%s[%u] >> %u) & 0x%xu;\n", indent, "", vec, w, sh, (1u << n) - 1u);
    else
        bput(b, "%*sidx = (uint32_t)((((uint64_t)%s[%u] << 32) | %s[%u]) >> %u) & 0x%xu;\n", indent, "", vec, w + 1u,
             vec, w, sh, (1u << n) - 1u);
}

/* the full evaluation: every level's unit values from bits[], the root into r */
static void hlut_emit_init(Buf* b, const HPlan* h, uint32_t nw, int indent) {
    bput(b, "%*suint32_t idx;\n", indent, "");
    for (uint32_t L = 0; L < h->L; ++L) {
        char lowv[16];
        snprintf(lowv, sizeof lowv, L ? "hv%u" : "bits", L - 1u);
        const uint32_t nwl = L ? (h->k[L - 1] + 31u) / 32u : 0u;
        const uint32_t last = L + 1u == h->L;
        if (!last)
            for (uint32_t w = 0; w < (h->k[L] + 31u) / 32u; ++w) bput(b, "%*shv%u[%u] = 0u;\n", indent, "", L, w);
        for (uint32_t j = 0; j < h->k[L]; ++j) {
            const uint32_t u = h->ubase[L] + j;
            h_emit_extract_static(b, lowv, L ? nwl : nw, h->ulo[u], h->un[u], indent);
            if (last)
                bput(b, "%*sr = (WO_HTAB[%uu + (idx >> 5)] >> (idx & 31u)) & 1u;\n", indent, "", h->uoff[u]);
            else
                bput(b, "%*shv%u[%u] |= ((WO_HTAB[%uu + (idx >> 5)] >> (idx & 31u)) & 1u) << %u;\n", indent, "", L,
                     j / 32u, h->uoff[u], j % 32u);
        }
    }
}

/* one event's update: primitive `ord`'s unit at each level, the root into r */
static void hlut_emit_update(Buf* b, const HPlan* h, uint32_t nw, int indent) {
    bput(b, "%*suint32_t hi = ord;\n", indent, "");
    for (uint32_t L = 0; L < h->L; ++L) {
        const uint32_t nwl = L ? (h->k[L - 1] + 31u) / 32u : nw;
        char lowv[16];
        snprintf(lowv, sizeof lowv, L ? "hv%u" : "bits", L - 1u);
        bput(b, "%*s{\n", indent, "");
        bput(b,
             "%*s  const uint32_t e = WO_HINFO[%uu + hi];\n"
             "%*s  const uint32_t lo = (e >> 8) & 0x3ffu, n = (e >> 18) & 0xfu;\n",
             indent, "", h->base[L], indent, "");
        if (nwl == 1u) {
            bput(b, "%*s  const uint32_t idx = (%s[0] >> lo) & ((1u << n) - 1u);\n", indent, "", lowv);
        } else {
            bput(b, "%*s  const uint32_t w = lo >> 5;\n", indent, "");
            /* level 0 with the words in LDS: two reads at the word index (the extra word
             * past the last is 0) instead of a select per word */
            /* (at the last word, a1 is any word: a unit's bits never pass the last
             * primitive, so the shift and mask below take none of a1's) */
            if (!L)
                bput(b, "#if WO_HBITS_LDS\n%*s  const uint32_t a0 = bits[w], a1 = bits[w + 1u < %uu ? w + 1u : w];\n#else\n",
                     indent, "", nwl);
            bput(b, "%*s  uint32_t a0 = %s[0], a1 = %s[1];\n", indent, "", lowv, lowv);
            for (uint32_t k = 1; k < nwl; ++k) {
                bput(b, "%*s  a0 = w == %uu ? %s[%u] : a0;\n", indent, "", k, lowv, k);
                if (k + 1u < nwl) bput(b, "%*s  a1 = w == %uu ? %s[%u] : a1;\n", indent, "", k, lowv, k + 1u);
            }
            if (!L) bput(b, "#endif\n");
            bput(b, "%*s  const uint32_t idx = (uint32_t)((((uint64_t)a1 << 32) | a0) >> (lo & 31u)) & ((1u << n) - 1u);\n",
                 indent, "");
        }
        bput(b, "%*s  const uint32_t v = (WO_HTAB[(e >> 22) + (idx >> 5)] >> (idx & 31u)) & 1u;\n", indent, "");
        if (L + 1u == h->L) {
            bput(b, "%*s  r = v;\n", indent, "");
        } else {
            bput(b, "%*s  const uint32_t j = e & 0xffu, jm = 1u << (j & 31u);\n", indent, "");
            for (uint32_t w = 0; w < (h->k[L] + 31u) / 32u; ++w)
                bput(b, "%*s  hv%u[%u] = (j >> 5) == %uu ? ((hv%u[%u] & ~jm) | (v ? jm : 0u)) : hv%u[%u];\n", indent, "", L,
                     w, w, L, w, L, w);
            bput(b, "%*s  hi = j;\n", indent, "");
        }
        bput(b, "%*s}\n", indent, "");
    }
}

/* ---- collect over the CSG tree, culled by relevance boxes ----
 * For a general tree (the levelled tables' scenes) the primitives are collected
 * in a walk of the tree itself, and a subtree of >= WO_RCULL_MIN primitives gets a
 * wave-level test of the sphere around its box: the meet of its bounds (a union's
 * hull, an intersection's meet, a difference's left operand's) with its relevance
 * box (the meet of the bounds of the operands that gate it on its path to the
 * root -- an intersection's other operand, a difference's left one for its right
 * one).  A wave whose rays all miss it skips the subtree: along those rays the
 * subtree is either empty or gated off wherever it is not, so its bits staying 0
 * leaves the root's value, and the hit, unchanged (the lane tracer's relevance
 * argument).  A subtree whose box is empty is never collected. */
typedef struct RBox {
    double lo[3], hi[3];
} RBox;
typedef struct RSph {
    double c[3], r; /* r < 0: none (unbounded) */
} RSph;
typedef struct RTree {
    TNode* t;
    int root;
    RBox *bnd, *rel;
    RSph* sph; /* per node: a sphere around its bounds (tighter than the box's for unions of spheres) */
    uint32_t* pc_of; /* per ordinal: its PRIM record */
    uint32_t cull_min;
} RTree;

static RBox rb_inf(void) {
    RBox b;
    for (int a = 0; a < 3; ++a) b.lo[a] = -INFINITY, b.hi[a] = INFINITY;
    return b;
}
static RBox rb_meet(RBox x, RBox y) {
    for (int a = 0; a < 3; ++a) x.lo[a] = fmax(x.lo[a], y.lo[a]), x.hi[a] = fmin(x.hi[a], y.hi[a]);
    return x;
}
static RBox rb_hull(RBox x, RBox y) {
    for (int a = 0; a < 3; ++a) x.lo[a] = fmin(x.lo[a], y.lo[a]), x.hi[a] = fmax(x.hi[a], y.hi[a]);
    return x;
}
static RBox rb_slack(RBox x, double k) {
    for (int a = 0; a < 3; ++a) {
        if (!isfinite(x.lo[a]) || !isfinite(x.hi[a])) continue;
        const double m = k * (1e-4 * (fabs(x.lo[a]) + fabs(x.hi[a]) + fabs(x.hi[a] - x.lo[a])) + 1e-5);
        x.lo[a] -= m;
        x.hi[a] += m;
    }
    return x;
}
static int rb_empty(const RBox* x) {
    for (int a = 0; a < 3; ++a)
        if (x->lo[a] > x->hi[a]) return 1;
    return 0;
}
static int rb_finite(const RBox* x) {
    for (int a = 0; a < 3; ++a)
        if (!isfinite(x->lo[a]) || !isfinite(x->hi[a])) return 0;
    return 1;
}
/* a convex primitive's box: sphere members and axis-aligned half-spaces (others: none) */
static RBox prim_box(const WoRec* prog, uint32_t pc) {
    RBox b = rb_inf();
    for (uint32_t m = 0; m < prog[pc].u0; ++m) {
        const WoRec* L = &prog[pc + 1u + m];
        if (L->op == WO_LEAF_SPHERE) {
            const double r = sqrt((double)L->f[3]);
            for (int a = 0; a < 3; ++a) {
                b.lo[a] = fmax(b.lo[a], (double)L->f[a] - r);
                b.hi[a] = fmin(b.hi[a], (double)L->f[a] + r);
            }
        } else if (L->op == WO_LEAF_HALFSPACE && L->u1 >= 1u && L->u1 <= 3u) {
            const int a = (int)L->u1 - 1; /* s * x_a <= h */
            if (L->f[a] > 0.0f)
                b.hi[a] = fmin(b.hi[a], (double)L->f[3]);
            else
                b.lo[a] = fmax(b.lo[a], -(double)L->f[3]);
        }
    }
    return b;
}

/* the smallest sphere enclosing two spheres */
static RSph rs_hull(RSph a, RSph b) {
    if (a.r < 0.0 || b.r < 0.0) {
        RSph u = {{0.0, 0.0, 0.0}, -1.0};
        return u;
    }
    double d[3], l = 0.0;
    for (int k = 0; k < 3; ++k) d[k] = b.c[k] - a.c[k], l += d[k] * d[k];
    l = sqrt(l);
    if (l + b.r <= a.r) return a;
    if (l + a.r <= b.r) return b;
    RSph h;
    h.r = 0.5 * (l + a.r + b.r);
    for (int k = 0; k < 3; ++k) h.c[k] = a.c[k] + (l > 0.0 ? d[k] / l * (h.r - a.r) : 0.0);
    return h;
}
/* a convex primitive's sphere: its smallest sphere member (the primitive lies inside each) */
static RSph prim_sph(const WoRec* prog, uint32_t pc) {
    RSph s = {{0.0, 0.0, 0.0}, -1.0};
    for (uint32_t m = 0; m < prog[pc].u0; ++m) {
        const WoRec* L = &prog[pc + 1u + m];
        if (L->op != WO_LEAF_SPHERE) continue;
        const double r = sqrt((double)L->f[3]);
        if (s.r < 0.0 || r < s.r) s.c[0] = L->f[0], s.c[1] = L->f[1], s.c[2] = L->f[2], s.r = r;
    }
    return s;
}

static void rtree_free(RTree* rt) {
    free(rt->sph);
    free(rt->t);
    free(rt->bnd);
    free(rt->rel);
    free(rt->pc_of);
    memset(rt, 0, sizeof *rt);
}

static int rtree_build(const WoRec* prog, uint32_t n_recs, uint32_t n_prims, RTree* rt) {
    memset(rt, 0, sizeof *rt);
    const uint32_t cap = 2u * n_prims;
    rt->t = (TNode*)malloc(sizeof(TNode) * cap);
    rt->bnd = (RBox*)malloc(sizeof(RBox) * cap);
    rt->rel = (RBox*)malloc(sizeof(RBox) * cap);
    rt->pc_of = (uint32_t*)malloc(sizeof(uint32_t) * n_prims);
    rt->sph = (RSph*)malloc(sizeof(RSph) * cap);
    int* st = (int*)malloc(sizeof(int) * (n_prims + 1u));
    int ok = rt->t && rt->bnd && rt->rel && rt->pc_of && rt->sph && st && n_prims > 0u;
    uint32_t nt = 0, sp = 0;
    for (uint32_t pc = 0; pc < n_recs && ok;) {
        const WoRec* r = &prog[pc];
        if (r->op == WO_OP_PRIM) {
            ok = nt < cap && sp <= n_prims && r->u1 < n_prims;
            if (!ok) break;
            TNode x = {0, -1, -1, r->u1, 1u};
            rt->pc_of[r->u1] = pc;
            rt->bnd[nt] = prim_box(prog, pc);
            rt->sph[nt] = prim_sph(prog, pc);
            rt->t[nt] = x;
            st[sp++] = (int)nt++;
            pc += 1u + r->u0;
            continue;
        }
        ++pc;
        if (r->op == WO_OP_BOUND) continue;
        ok = sp >= 2u && nt < cap;
        if (!ok) break;
        const int b = st[--sp], a = st[--sp];
        TNode x = {(int)r->op, a, b, rt->t[a].lo < rt->t[b].lo ? rt->t[a].lo : rt->t[b].lo, rt->t[a].n + rt->t[b].n};
        rt->bnd[nt] = r->op == WO_OP_UNION   ? rb_hull(rt->bnd[a], rt->bnd[b])
                      : r->op == WO_OP_INTER ? rb_meet(rt->bnd[a], rt->bnd[b])
                      : r->op == WO_OP_DIFF  ? rt->bnd[a]
                                             : rt->bnd[b]; /* RDIFF: b AND NOT a */
        {
            const RSph sa = rt->sph[a], sb = rt->sph[b];
            if (r->op == WO_OP_UNION)
                rt->sph[nt] = rs_hull(sa, sb);
            else if (r->op == WO_OP_INTER) /* inside both: the smaller bounded one */
                rt->sph[nt] = sa.r < 0.0 ? sb : (sb.r < 0.0 || sa.r <= sb.r ? sa : sb);
            else
                rt->sph[nt] = r->op == WO_OP_DIFF ? sa : sb;
        }
        rt->t[nt] = x;
        st[sp++] = (int)nt++;
    }
    ok = ok && sp == 1u;
    if (ok) {
        rt->root = st[0];
        rt->rel[rt->root] = rb_inf();
        /* a node before its operands: postfix order reversed */
        for (uint32_t i = nt; i-- > 0;) {
            const TNode* x = &rt->t[i];
            if (x->op == 0) continue;
            const RBox c = rt->rel[i];
            const int a = x->l, b = x->r;
            rt->rel[a] = x->op == WO_OP_INTER || x->op == WO_OP_RDIFF ? rb_meet(c, rt->bnd[b]) : c;
            rt->rel[b] = x->op == WO_OP_INTER || x->op == WO_OP_DIFF ? rb_meet(c, rt->bnd[a]) : c;
        }
    }
    free(st);
    if (!ok) rtree_free(rt);
    return ok;
}

static void gen_rtree_node(Gen* g, int x, int indent) {
    const RTree* rt = g->rtree;
    const TNode* n = &rt->t[x];
    const RBox m = rb_meet(rb_slack(rt->bnd[x], 2.0), rb_slack(rt->rel[x], 2.0));
    if (rb_empty(&m)) return; /* never matters: its bits stay 0 */
    if (n->op == 0) {
        const uint32_t pc = rt->pc_of[n->lo];
        gen_collect(g, pc, pc + 1u + g->prog[pc].u0, indent);
        return;
    }
    int inner = indent;
    const int test = n->n >= rt->cull_min && rb_finite(&m);
    if (test) {
        double c[3], r2 = 0.0;
        for (int a = 0; a < 3; ++a) {
            c[a] = 0.5 * (m.lo[a] + m.hi[a]);
            const double h = 0.5 * (m.hi[a] - m.lo[a]);
            r2 += h * h;
        }
        double R = sqrt(r2) * (1.0 + 1e-6) + 1e-6;
        const RSph ns = rt->sph[x];
        if (ns.r >= 0.0) { /* the node's own sphere (it encloses the bounds, so their meet with the relevance box) when smaller */
            const double nr = ns.r * (1.0 + 2e-4) + 2e-5; /* the BOUND records' slack */
            if (nr < R) {
                R = nr;
                for (int a = 0; a < 3; ++a) c[a] = ns.c[a];
            }
        }
        const uint32_t k = g->nbound++;
        if (g->first_pass) {
            const float fc[3] = {(float)c[0], (float)c[1], (float)c[2]};
            const float fR = (float)(R * (1.0 + 1e-6)), fR2 = (float)(R * R * (1.0 + 4e-6));
            uint32_t vr2 = fbits(fR2);
            static const char* nr[1] = {"bc3"};
            bput(g->b, "%*s{  // relevance group %u (%u primitives)\n%*s  WO_WK(WO_WORK_BOUND_TESTS);\n", indent, "", k,
                 n->n, indent, "");
            emit_consts(g->b, indent + 2, "float", nr, &vr2, 1);
            bput(g->b,
                 "%*s  float ox, oy, oz, tca, d2, tr;\n"
                 "%*s  asm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(ox) : \"v\"(o.x));\n"
                 "%*s  asm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(oy) : \"v\"(o.y));\n"
                 "%*s  asm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(oz) : \"v\"(o.z));\n"
                 "%*s  wodev::bound_tca_d2(ox, oy, oz, d, tca, d2);\n"
                 "%*s  asm(\"v_add_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(tr) : \"v\"(tca));\n"
                 "%*s  const bool miss = (d2 > __builtin_fmaf(4e-6f * tca, tca, bc3)) | (tr < 0.0f);\n"
                 "%*s  if (__ballot(!miss) == 0ull) cull[%u] |= %uu;\n%*s}\n",
                 indent, "", indent, "", fbits(fc[0]), indent, "", fbits(fc[1]), indent, "", fbits(fc[2]), indent, "",
                 indent, "", fbits(fR), indent, "", indent, "", k / 32, 1u << (k % 32), indent, "");
        }
        bput(g->b, "%*sif (!(cull[%u] & %uu)) {\n", indent, "", k / 32, 1u << (k % 32));
        inner = indent + 2;
        {
            /* a lane whose window has already dropped events (n > kWindow) cannot keep an
             * event past its largest key: a group that starts beyond that key's t on every
             * lane of the wave adds nothing the window keeps and nothing to `dropped()` */
            const float fc[3] = {(float)c[0], (float)c[1], (float)c[2]};
            const float fRm = (float)(R * (1.0 + 1e-4) + 1e-4);
            bput(g->b,
                 "#if WO_WINDOW_BEYOND && !WO_JIT_LDS_EVENTS\n"
                 "%*sfloat bx%u, by%u, bz%u;\n"
                 "%*sasm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(bx%u) : \"v\"(o.x));\n"
                 "%*sasm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(by%u) : \"v\"(o.y));\n"
                 "%*sasm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(bz%u) : \"v\"(o.z));\n"
                 "%*sconst float tb%u = __builtin_fmaf(bz%u, d.z, __builtin_fmaf(by%u, d.y, bx%u * d.x));\n"
                 "%*sif (__ballot(!((win.n > (uint32_t)wodev::kWindow) & (tb%u - __builtin_fmaf(1e-4f, fabsf(tb%u), __uint_as_float(0x%08xu)) > __uint_as_float((uint32_t)(win.k[wodev::kWindow - 1] >> 32))))) != 0ull)\n"
                 "#endif\n"
                 "%*s{\n",
                 inner, "", k, k, k, inner, "", fbits(fc[0]), k, inner, "", fbits(fc[1]), k, inner, "", fbits(fc[2]), k,
                 inner, "", k, k, k, k, inner, "", k, k, fbits(fRm), inner, "");
            inner += 2;
        }
        if (!g->first_pass) {
            /* a re-collect wants the events after `after` only: a group whose sphere ends
             * before that key's t on every lane cannot change the root any more.  A ray
             * that has left a sphere never re-enters it (convex), and outside the group's
             * sphere the subtree is empty or gated off -- the first pass's cull argument,
             * which covers half-spaces and a sphere drawn around the meet of the subtree's
             * bounds with its relevance box alike (the primitives' events need not lie
             * inside it).  So the primitives' bits may stay at their values at `after`.
             * The margin covers the fp32 arithmetic; tests/test_jit.py::
             * test_recollect_behind_skip_keeps_the_root restates it in float64. */
            const float fc[3] = {(float)c[0], (float)c[1], (float)c[2]};
            const float fRm = (float)(R * (1.0 + 1e-4) + 1e-4);
            bput(g->b,
                 "#if WO_RECOLLECT_BEHIND\n"
                 "%*sfloat ox%u, oy%u, oz%u;\n"
                 "%*sasm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(ox%u) : \"v\"(o.x));\n"
                 "%*sasm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(oy%u) : \"v\"(o.y));\n"
                 "%*sasm(\"v_sub_f32_e32 %%0, 0x%08x, %%1\" : \"=v\"(oz%u) : \"v\"(o.z));\n"
                 "%*sconst float tca%u = __builtin_fmaf(oz%u, d.z, __builtin_fmaf(oy%u, d.y, ox%u * d.x));\n"
                 "%*sif (__ballot(!(__builtin_fmaf(1e-4f, fabsf(tca%u), tca%u) + __uint_as_float(0x%08xu) < tafter)) != 0ull)\n"
                 "#endif\n"
                 "%*s{\n",
                 inner, "", k, k, k, inner, "", fbits(fc[0]), k, inner, "", fbits(fc[1]), k, inner, "", fbits(fc[2]), k,
                 inner, "", k, k, k, k, inner, "", k, k, fbits(fRm), inner, "");
            inner += 2;
        }
    }
    gen_rtree_node(g, n->l, inner);
    gen_rtree_node(g, n->r, inner);
    if (test && !g->first_pass) bput(g->b, "%*s}\n", indent + 4, "");
    if (test) bput(g->b, "%*s}\n%*s}\n", indent + 2, "", indent, "");
}

static void gen_rtree(Gen* g, int indent) {
    if (g->first_pass)
        /* off: the per-group test costs more than it skips (csg360_nested 178.1 -> 190.2 ms,
         * csg32_nested 8.32 -> 8.60 with it) */
        bput(g->b, "#ifndef WO_WINDOW_BEYOND\n#define WO_WINDOW_BEYOND 0\n#endif\n");
    if (!g->first_pass)
        bput(g->b,
             "#ifndef WO_RECOLLECT_BEHIND\n#define WO_RECOLLECT_BEHIND 1\n#endif\n"
             "%*sconst float tafter = __uint_as_float((uint32_t)(after >> 32));  // the last processed key's t\n"
             "%*s(void)tafter;\n",
             indent, "", indent, "");
    gen_rtree_node(g, g->rtree->root, indent);
}

/* The root's value from bits[] (the truth tables, or the flattened evaluation with
 * WO_JIT_LUT=0) into `out`, as a block of its own (the batch sweep's copies). */
static void gen_eval_block(Gen* g, const LutPlan* lut, int use_lut, uint32_t n_recs, int indent, const char* out) {
    bput(g->b, "%*s{\n%*s  uint32_t r;\n%s", indent, "", indent, "", use_lut ? "#if WO_JIT_LUT\n" : "");
    if (use_lut) {
        bput(g->b, "%*s  {\n", indent, "");
        lut_emit_eval(g->b, lut, indent + 4);
        bput(g->b, "%*s  }\n#else\n", indent, "");
    }
    bput(g->b, "%*s  {\n", indent, "");
    g->nbound = 0;
    Term rt = gen_eval_flat(g, 0, n_recs, indent + 4);
    uint32_t rv = term_name(g, &rt, indent + 4);
    bput(g->b, "%*s    r = v%u ? 1u : 0u;\n%*s  }\n", indent, "", rv, indent, "");
    if (use_lut) bput(g->b, "#endif\n");
    bput(g->b, "%*s  %s = r;\n%*s}\n", indent, "", out, indent, "");
}

char* wo_generate_jit_source(WoRec const* prog, uint32_t n_recs, uint32_t n_prims) {
    Buf b = {0};
    Gen g;
    memset(&g, 0, sizeof g);
    g.prog = prog;
    g.n = n_recs;
    g.b = &b;
    uint32_t nw = n_prims ? (n_prims + 31u) / 32u : 1u;
    /* Wave-level BOUND tests pay only for larger subtrees (csg32 5.17 ms testing
     * subtrees of >= 8 leaves vs 6.94 testing every BOUND; later 4.93 at >= 6, 4.95
     * at 4 / 5; csg256 balanced with the union count 9.80 at 4, 10.02 at 6, 10.46 at 8). */
    g.bound_min_leaves = 4;
    /* Event window: the LDS list wins where rays meet few events per trace and
     * the register window where they meet many (a deep difference chain carves
     * every sphere the ray passes).  Measured, 1920x1080x64: csg32 6.40 vs 6.47 ms,
     * csg256 balanced 20.2 vs 21.4, csg256 chain 35.8 vs 33.9.  Tree depth
     * separates them. */
    g.lds_events = tree_depth(prog, n_recs) <= 32u;
    g.first_event = n_prims <= 64u * 32u;
    uint32_t nbounds = 0;
    /* spatial collect (surface-area splits, leaves of <= 8): for deep trees (no
     * union-cluster hierarchy to cull with: csg256 chain 18.40 -> 13.59 ms) and small
     * scenes (csg32 3.716 -> 3.586 ms, 3840x2160x256 56.08 -> 54.45); csg256
     * balanced's SAH cluster hierarchy over its pairs culls better (10.10 vs 10.58
     * ms).  Leaves: median splits, chain 15.04 / 13.93 / 13.63 ms at 2 / 4 / 8; SAH,
     * csg32 3.687 / 3.612 / 3.628 / 3.589 at 3 / 4 / 6 / 8. */
    g.spatial = !g.lds_events || n_prims <= 64u;
    {
        const char* sp = getenv("WOLOLO_JIT_SPATIAL"); /* (measurement) 1 / 0 forces the spatial collect on / off */
        if (sp && (*sp == '0' || *sp == '1')) g.spatial = *sp == '1';
    }
    g.spatial_leaf = 8;
    /* term mode: where the root allows it, the tree is shallow enough for the
     * event-list path it replaces, and the scene is small enough for the spatial
     * groups over terms to cull as well as the scene compiler's cluster hierarchy
     * (<= 64 primitives: csg32 3.59 -> 3.33 ms; csg256 balanced 9.83 -> 12.40, so off
     * there). */
    uint32_t n_jterms = 0;
    JTerm* jterms = NULL;
    if (n_prims <= 64u && g.lds_events && n_prims) jterms = jit_terms(prog, n_recs, n_prims, &n_jterms);
    SPrim* tunb = NULL;
    if (jterms) {
        uint32_t* pc_of = (uint32_t*)malloc(sizeof(uint32_t) * n_prims);
        SPrim* units = (SPrim*)calloc(n_jterms, sizeof(SPrim));
        tunb = (SPrim*)calloc(n_jterms, sizeof(SPrim));
        if (!pc_of || !units || !tunb) g.err = 1;
        for (uint32_t pc = 0; pc_of && pc < n_recs;) {
            if (prog[pc].op != WO_OP_PRIM) {
                ++pc;
                continue;
            }
            pc_of[prog[pc].u1] = pc;
            pc += 1u + prog[pc].u0;
        }
        uint32_t nb = 0;
        for (uint32_t i = 0; !g.err && i < n_jterms; ++i) {
            SPrim u;
            memset(&u, 0, sizeof u);
            u.term = 1;
            u.npc = jterms[i].n;
            int have = 0;
            for (uint32_t k = 0; k < jterms[i].n; ++k) {
                const uint32_t lit = jterms[i].lit[k];
                u.pcs[k] = pc_of[lit & ~JT_NEG];
                if (lit & JT_NEG) {
                    u.negm |= 1u << k;
                    continue;
                }
                /* the term lies inside each positive literal: the smallest one's sphere bounds it */
                SPrim b;
                if (prim_sphere(prog, u.pcs[k], &b) && (!have || b.r < u.r)) {
                    u.c[0] = b.c[0], u.c[1] = b.c[1], u.c[2] = b.c[2], u.r = b.r;
                    have = 1;
                }
            }
            u.pc = u.pcs[0];
            if (have)
                units[nb++] = u;
            else
                tunb[g.ntunb++] = u;
        }
        /* outsized units (radius > 16x the median: a ground sphere) stay out of the
         * hierarchy, as in the primitive form below */
        if (nb > 2u) {
            double* rs = (double*)malloc(sizeof(double) * nb);
            if (rs) {
                for (uint32_t i = 0; i < nb; ++i) rs[i] = units[i].r;
                for (uint32_t i = 1; i < nb; ++i)
                    for (uint32_t j = i; j > 0 && rs[j - 1] > rs[j]; --j) {
                        const double t = rs[j];
                        rs[j] = rs[j - 1];
                        rs[j - 1] = t;
                    }
                const double med = rs[nb / 2u];
                free(rs);
                uint32_t k = 0;
                for (uint32_t i = 0; i < nb; ++i) {
                    if (units[i].r > 16.0 * med)
                        tunb[g.ntunb++] = units[i];
                    else
                        units[k++] = units[i];
                }
                nb = k;
            } else {
                g.err = 1;
            }
        }
        free(pc_of);
        g.term_mode = 1;
        g.spatial = 1;
        g.sprims = units;
        g.nsprims = nb;
        g.tunb = tunb;
    }
    SPrim* sprims = g.term_mode ? g.sprims : NULL;
    if (g.term_mode) {
        /* the groups it tests: a dry run of the emitter into a scratch buffer */
        Buf scratch = {0};
        Buf* keep = g.b;
        g.b = &scratch;
        g.nbound = 0;
        g.first_pass = 1;
        gen_collect_terms(&g, 0);
        nbounds += g.nbound;
        g.b = keep;
        free(scratch.s);
    }
    if (g.spatial && !g.term_mode) {
        sprims = (SPrim*)malloc(sizeof(SPrim) * (n_prims ? n_prims : 1u));
        if (!sprims) g.err = 1;
        for (uint32_t pc = 0; sprims && pc < n_recs;) {
            if (prog[pc].op != WO_OP_PRIM) {
                ++pc;
                continue;
            }
            if (prim_sphere(prog, pc, &sprims[g.nsprims])) ++g.nsprims;
            pc += 1u + prog[pc].u0;
        }
        /* outsized primitives (radius > 16x the median, e.g. a ground sphere) stay
         * out of the hierarchy, as the scene compiler keeps them out of its BVHs:
         * inside it they would make every group above them a sphere no ray misses */
        if (g.nsprims > 2u) {
            double* rs = (double*)malloc(sizeof(double) * g.nsprims);
            if (!rs) {
                g.err = 1;
            } else {
                for (uint32_t i = 0; i < g.nsprims; ++i) rs[i] = sprims[i].r;
                for (uint32_t i = 1; i < g.nsprims; ++i) /* insertion sort: a few hundred at most */
                    for (uint32_t j = i; j > 0 && rs[j - 1] > rs[j]; --j) {
                        const double t = rs[j];
                        rs[j] = rs[j - 1];
                        rs[j - 1] = t;
                    }
                const double med = rs[g.nsprims / 2u];
                free(rs);
                uint32_t k = 0;
                for (uint32_t i = 0; i < g.nsprims; ++i)
                    if (!(sprims[i].r > 16.0 * med)) sprims[k++] = sprims[i];
                g.nsprims = k;
            }
        }
        g.sprims = sprims;
        {
            /* the groups it tests: a dry run of the emitter into a scratch buffer */
            Buf scratch = {0};
            Buf* keep = g.b;
            g.b = &scratch;
            g.nbound = 0;
            g.first_pass = 1;
            gen_collect_spatial(&g, g.sprims, g.nsprims, 0);
            nbounds += g.nbound;
            g.b = keep;
            free(scratch.s);
        }
    }
    /* the incremental union count's term table, per primitive: its term's mask test */
    uint32_t n_uterms = 0, eval_ops = 0;
    UTerm* uterms = NULL;
    /* when the root is a union of >= 8 literal-set terms (csg32: 9 terms, 3.73 ->
     * 3.68 ms before term mode took it; csg256 balanced's 65) */
    if (n_prims && !g.term_mode) {
        uterms = (UTerm*)malloc(sizeof(UTerm) * n_prims);
        if (!uterms) g.err = 1;
        else n_uterms = union_terms(prog, n_recs, n_prims, uterms, n_prims);
        if (n_uterms < 8u) n_uterms = 0;
    }
    /* truth-table root evaluation for the general form (lut_plan) */
    LutPlan lut;
    memset(&lut, 0, sizeof lut);
    const int use_lut = n_prims && !g.term_mode && !n_uterms && lut_plan(prog, n_recs, n_prims, &lut);
    /* levels of truth tables for a general tree above lut_plan's size (hlut_plan;
     * a chain has too many levels and keeps its decision lists) */
    HPlan hl;
    memset(&hl, 0, sizeof hl);
    const int use_hlut =
        n_prims > 64u && !g.term_mode && !n_uterms && !use_lut && hlut_plan(prog, n_recs, n_prims, &hl);
    /* The truth tables' trees (general trees that are not chains) collect over the
     * tree with relevance-box culls (gen_rtree) instead of the scene compiler's BOUND
     * records or the spatial groups: csg360_nested 201.6 -> 183.5 ms (subtrees of >= 2
     * primitives tested; 184.3 / 184.7 / 201.5 at >= 3 / 4 / 16, and 195.3 with the
     * boxes' spheres alone at 8), csg32_nested 8.83 -> 8.47 ms (>= 4; 8.51 / 8.54 / 8.51 /
     * 8.64 at 3 / 6 / 8 / 12; 8.66 at 2).  The csg256 chain (decision lists, no tables)
     * keeps its BOUND records: 11.3 against 24.8 ms.  WOLOLO_JIT_RCULL=<n> sets the
     * smallest subtree tested (measurements), 0 turns the tree collect off. */
    RTree rtree;
    memset(&rtree, 0, sizeof rtree);
    {
        const char* rc = getenv("WOLOLO_JIT_RCULL");
        const uint32_t cull_min = rc && *rc ? (uint32_t)strtoul(rc, NULL, 10) : use_hlut ? 2u : 4u;
        if ((use_hlut || use_lut) && cull_min && rtree_build(prog, n_recs, n_prims, &rtree)) {
            rtree.cull_min = cull_min;
            g.rtree = &rtree;
            g.spatial = 0;
            Buf scratch = {0};
            Buf* keep = g.b;
            g.b = &scratch;
            g.nbound = 0;
            g.first_pass = 1;
            gen_rtree(&g, 0);
            nbounds = g.nbound; /* (not the spatial groups counted above: unused) */
            g.b = keep;
            free(scratch.s);
        }
    }
    if (!g.rtree)
        for (uint32_t i = 0; i < n_recs && !g.term_mode; ++i) nbounds += prog[i].op == WO_OP_BOUND && bound_tested(&g, i);

    bput(&b, "// generated by scene_jit.c: %u records, %u primitives, %u bounds\n", n_recs, n_prims, nbounds);
    /* Small programs are copied to LDS per workgroup with the materials they use:
     * the hit leaf / material reads then cost an LDS round trip instead of
     * dependent global loads.  Larger ones stay in global memory, where the LDS
     * would cost occupancy. */
    uint32_t n_mats_used = 1;
    for (uint32_t i = 0; i < n_recs; ++i)
        if ((prog[i].op == WO_LEAF_SPHERE || prog[i].op == WO_LEAF_HALFSPACE) && prog[i].u0 + 1u > n_mats_used)
            n_mats_used = prog[i].u0 + 1u;
    const int lds_prog =
        (size_t)n_recs * sizeof(WoRec) + (size_t)n_mats_used * sizeof(WoMaterial) + 4u * n_prims <= 6144u;
    if (use_lut) {
        bput(&b, "#ifndef WO_JIT_LUT\n#define WO_JIT_LUT 1\n#endif\n");
    } else {
        bput(&b, "#define WO_JIT_LUT 0\n");
    }
    bput(&b, "#define WO_JIT_HLUT %d\n", use_hlut);
    /* A full LDS event list keeps its smallest keys (WO_LDS_KEEP_SMALLEST): csg32_nested
     * 20.18 -> 10.97 ms (re-collects per segment 0.86 -> 0.18).  A union of small
     * terms (csg32, csg256 balanced) rarely fills the list, and there the eviction
     * code costs csg32 3.608 -> 3.701 ms: off for the union count. */
    if (g.lds_events && n_uterms) bput(&b, "#ifndef WO_LDS_KEEP_SMALLEST\n#define WO_LDS_KEEP_SMALLEST 0\n#endif\n");
    /* the cull words through an opaque move in re-collects (csg256 chain 13.51 ->
     * 13.21 ms, balanced 9.70 -> 9.47, csg32 3.273 -> 3.238), except for a general
     * root evaluation over the LDS event list (csg32_nested 10.92 -> 11.75: its SGPR
     * spills became 564 spilled VGPRs) */
    /* (off for the LDS event list's general evaluation: csg32_nested's SGPR spills
     * became 564 spilled VGPRs, 10.92 -> 11.75 ms; with the register window and the
     * truth tables it helps: 9.33 -> 9.26) */
    g.cull_barrier = 1;
    bput(&b, "#ifndef WO_JIT_CULL_BARRIER\n#define WO_JIT_CULL_BARRIER %d\n#endif\n", g.cull_barrier);
    /* the register window for deep trees holds 5 events (csg256 chain 29.5 ms at 4,
     * 27.6 at 6, 27.5 at 8; with decision lists 19.36 at 4, 18.47 at 5, 18.65 at 6) */
    /* The register window's events: 5 for deep trees (csg256 chain 29.5 ms at 4, 27.6 at 6,
     * 27.5 at 8; with decision lists 19.36 at 4, 18.47 at 5, 18.65 at 6); the union count
     * (csg256 balanced 9.98 / 9.32 / 10.00 ms at 4 / 5 / 6); 8 for the truth-table form
     * (csg32_nested 9.64 / 9.33 / 9.07 at 4 / 5 / 6, with the cull barrier 9.01 / 8.91 / 8.89
     * at 6 / 7 / 8). */
    /* 14 for the levelled tables' big trees (csg360_nested with the flat evaluation:
     * 250.7 / 243.9 / 235.7 ms at 10 / 12 / 14 events and 5 waves per SIMD, 241.5 at 16
     * and 4 waves; 304.6 at 5 and 8 waves; with the tables and relevance groups, 6 waves:
     * 179.8 ms at 14, 179.2 at 16; 7 waves 179.3; 5 waves 184.5, at 12 events 189.0) */
    bput(&b, "#ifndef WO_WINDOW\n#define WO_WINDOW %d\n#endif\n", use_lut ? 8 : use_hlut ? 14 : 5);
    /* two swept events per trip of the sweep loop (the second without a re-collect):
     * off -- the second copy's registers spill (csg32_nested 6.78 -> 6.91 ms, chain
     * 10.06 -> 10.16; profiles/r06_ab_sweep_unroll.txt) */
    bput(&b, "#ifndef WO_SWEEP_UNROLL\n#define WO_SWEEP_UNROLL 0\n#endif\n");
    bput(&b, "#ifndef WO_SWEEP_BATCH\n#define WO_SWEEP_BATCH 1\n#endif\n#ifndef WO_SWEEP_BATCH_EXIT\n#define WO_SWEEP_BATCH_EXIT 1\n#endif\n");
    /* term mode's lone spheres: the interval on every lane behind the wave-level test,
     * masked, instead of a lane branch on disc >= 0 */
    /* (not for the union count: csg256 balanced then spills 48 B per lane at 7 waves, 1.7 GB
     * of scratch traffic per frame) */
    bput(&b, "#ifndef WO_LONE_SEL\n#define WO_LONE_SEL 1\n#endif\n#ifndef WO_LONE_SEL_EV\n#define WO_LONE_SEL_EV %d\n#endif\n",
         n_uterms ? 0 : 1);
    /* the levelled tables' membership words in LDS (wodev::LdsBits) from 4 words; with
     * them csg360_nested's kernel fits 5 waves per SIMD without scratch (the window of
     * 14 keys; 130.2 ms, against 131.6 at 6 waves with 60 B of scratch per lane and
     * 174-178 ms in round 5; windows 16 / 20 at 5 waves: 125.1 / 120.0 ms but 44 / 72 B
     * of scratch -- the path state spilled around every trace, GBs per frame;
     * profiles/r06_ab_csg360_lds_bits.txt) */
    if (use_hlut)
        bput(&b, "#ifndef WO_HBITS_LDS\n#define WO_HBITS_LDS %d\n#endif\n#define WO_HBITS_WORDS %uu\n",
             (n_prims + 31u) / 32u >= 4u ? 1 : 0, (n_prims + 31u) / 32u);
    if (g.term_mode) bput(&b, "// term mode: %u terms (%u outside the spatial hierarchy)\n", n_jterms, g.ntunb);
    /* small scenes run 8 waves per SIMD: a 7-entry LDS list keeps 8 workgroups'
     * LDS within the CU (csg32 5.24 -> 5.19 ms; csg256 balanced keeps 8 entries:
     * 15.12 vs 15.33 ms at 7) */
    if (g.lds_events && n_prims <= 64u) bput(&b, "#ifndef WO_LDS_EVENTS\n#define WO_LDS_EVENTS 7\n#endif\n");
    /* Camera-ray waves (pathtrace_block): camera rays traced in iterations of their
     * own, so a wave's culling sees coherent rays (csg32 3.125 -> 2.80 ms, chain 12.74
     * -> 11.35; they replace round 4's ring of camera rays, csg32 3.13 -> 3.07).  Mode
     * 1's ring of ready paths (12 KB per workgroup) does not fit beside an LDS event
     * list at 8 workgroups per CU (csg32_nested 10.55 -> 11.76, csg256 balanced 9.30 ->
     * 10.59 at 4 waves per SIMD), so the event window is in registers (below); mode 2
     * rings the camera hits (4 KB). */
    bput(&b, "#ifndef WO_CAM_WAVES\n#define WO_CAM_WAVES 1\n#endif\n");
    /* WO_JIT_LDS_EVENTS=0 (WOLOLO_JIT_FLAGS) puts a small tree's event window in
     * registers (wodev::Window) instead of the LDS list */
    bput(&b, "#include \"wo_device_common.h\"\n#ifndef WO_JIT_LDS_EVENTS\n#define WO_JIT_LDS_EVENTS 0  // tree depth %u\n#endif\n#define WO_JIT_LDS_PROG %d\n\n",
         tree_depth(prog, n_recs), lds_prog);
    if (use_lut) {
        bput(&b, "// root by truth tables: %u subtrees (", lut.k);
        for (uint32_t s2 = 0; s2 < lut.k; ++s2) bput(&b, "%s[%u, %u)", s2 ? ", " : "", lut.lo[s2], lut.lo[s2] + lut.n[s2]);
        bput(&b, ")\n__constant__ uint32_t kLut[%u] = {", lut.words);
        for (uint32_t i = 0; i < lut.words; ++i) bput(&b, "%s0x%08xu", i ? ", " : "", lut.table[i]);
        bput(&b, "};\n");
    }
    if (n_uterms) {
        bput(&b, "struct __attribute__((aligned(16))) WoUTerm { uint64_t m, q; uint32_t w, neg, pad0, pad1; };\n");
        bput(&b, "// root = union of %u literal-set terms: a term is true iff ((window(w) & m) == q) != neg,\n"
                 "// window(w) = bits[w] | bits[w + 1] << 32; per primitive, the term it belongs to\n", n_uterms);
        bput(&b, "__constant__ WoUTerm kUTerm[%u] = {", n_prims);
        for (uint32_t p = 0; p < n_prims; ++p) {
            const UTerm* u = NULL;
            for (uint32_t i = 0; i < n_uterms && !u; ++i)
                if (p >= 32u * uterms[i].w && p < 32u * uterms[i].w + 64u && ((uterms[i].m >> (p - 32u * uterms[i].w)) & 1u))
                    u = &uterms[i];
            if (!u) {
                g.err = 1;
                break;
            }
            bput(&b, "%s{0x%016llxull, 0x%016llxull, %uu, %uu, 0u, 0u}", p ? ", " : "", (unsigned long long)u->m,
                 (unsigned long long)u->q, u->w, u->neg);
        }
        bput(&b, "};\n");
        /* (the table in LDS: no gain for csg32, csg256 balanced 10.01 -> 11.57 ms from
         * the LDS occupancy) */
        bput(&b, "#define WO_UTERM kUTerm\n");
    }
    if (use_hlut) {
        bput(&b, "// root by %u levels of truth tables (units per level:", hl.L);
        for (uint32_t L = 0; L < hl.L; ++L) bput(&b, " %u", hl.k[L]);
        bput(&b, ")\n__constant__ uint32_t kHInfo[%u] = {", hl.ninfo);
        for (uint32_t i = 0; i < hl.ninfo; ++i) bput(&b, "%s0x%08xu", i ? ", " : "", hl.info[i]);
        bput(&b, "};\n__constant__ uint32_t kHTab[%u] = {", hl.words);
        for (uint32_t i = 0; i < hl.words; ++i) bput(&b, "%s0x%08xu", i ? ", " : "", hl.table[i]);
        bput(&b, "};\n");
    }
    bput(&b, "__constant__ uint32_t kOrdPc[%u] = {", n_prims ? n_prims : 1u);
    if (!n_prims) bput(&b, "0u");
    for (uint32_t i = 0, o = 0; i < n_recs; ++i)
        if (prog[i].op == WO_OP_PRIM) bput(&b, "%s%uu", o++ ? ", " : "", i);
    bput(&b, "};\n\n");
    bput(&b,
         "struct JitTracer {\n"
         "  static constexpr bool kCount = WO_COUNT_WORK != 0;  // counting variant: -DWO_COUNT_WORK=1\n"
         "  wodev::WorkCounts wk;\n"
         "  uint64_t tmark;  // end of the first pass (section timing)\n"
         "  const WoRec* __restrict__ prog;\n"
         "  const uint32_t* __restrict__ ordpc;\n"
         "  uint64_t* ev;  // LDS event list column (LdsWindow)\n"
         "#if WO_JIT_LUT\n"
         "  const __attribute__((address_space(3))) uint32_t* lut;  // LDS copy of kLut\n"
         "#define WO_LUT lut\n"
         "#endif\n"
         "#if WO_JIT_HLUT\n"
         "  const __attribute__((address_space(3))) uint32_t* hinfo;  // LDS copies of kHInfo / kHTab\n"
         "  const __attribute__((address_space(3))) uint32_t* htab;\n"
         "#define WO_HINFO hinfo\n"
         "#define WO_HTAB htab\n"
         "#if WO_HBITS_LDS\n"
         "  wodev::LdsBits::P sbits;  // this lane's column of the membership words (LDS)\n"
         "#endif\n"
         "#endif\n"
         "  __device__ __forceinline__ WoRec hit_leaf(const wodev::Hit& h) const {\n"
         "    return prog[ordpc[h.ord()] + 1u + h.member()];\n"
         "  }\n"
         "  __device__ __forceinline__ bool trace(wodev::F3 o, wodev::F3 d, wodev::Hit& hit) {\n");
    if (n_prims == 0) {
        bput(&b, "    return false;\n  }\n};\n");
    } else {
        bput(&b, "    const float tmin = WO_T_MIN;\n");
        /* reciprocal direction components for the axes axis-aligned half-spaces use */
        uint32_t axes = 0;
        for (uint32_t i = 0; i < n_recs; ++i)
            if (prog[i].op == WO_LEAF_HALFSPACE && prog[i].u1 >= 1u && prog[i].u1 <= 3u) axes |= 1u << (prog[i].u1 - 1u);
        for (int a = 0; a < 3; ++a)
            if (axes & (1u << a)) bput(&b, "    const float iv%c = wodev::rcp_dir(d.%c);\n", "xyz"[a], "xyz"[a]);
        uint32_t ncw = nbounds ? (nbounds + 31u) / 32u : 1u;
        g.ncw = ncw;
        if (g.term_mode) {
            bput(&b, "    uint32_t cull[%u];  // bit k: group k culled for this wave\n", ncw);
            for (uint32_t w = 0; w < ncw; ++w) bput(&b, "    cull[%u] = 0u;\n", w);
            bput(&b,
                 "    // the smallest term transition after `after` (its rise flag in the key)\n"
                 "    // and the number of terms true at t_min\n"
                 "    uint64_t best = wodev::kBestNone, after = 0ull;\n"
                 "    uint32_t cnt = 0u;\n"
                 "    (void)after;\n"
                 "    WO_MARK(\"collect_begin\");\n"
                 "    {\n");
            g.first_pass = 1;
            gen_collect_all(&g, 6);
            bput(&b,
                 "    }\n"
                 "    WO_MARK(\"collect_end\");\n"
                 "    WO_TMARK();\n"
                 "    if (best == wodev::kBestNone) return false;\n"
                 "    const bool root = cnt != 0u;\n"
                 "    for (;;) {\n"
                 "      WO_WK(WO_WORK_SWEEP_STEPS);\n"
                 "      WO_WK_WAVE(WO_WORK_SWEEP_TRIPS);\n"
                 "      cnt = wodev::term_rises(best) ? cnt + 1u : cnt - 1u;\n"
                 "      if ((cnt != 0u) != root) {\n"
                 "        wodev::hit_from_key(wodev::term_event(best), cnt != 0u ? 1u : 0u, hit);\n"
                 "        return true;\n"
                 "      }\n"
                 "      // the count moved without flipping the root: the next transition\n"
                 "      after = best;\n"
                 "      best = wodev::kBestNone;\n"
                 "      WO_WK(WO_WORK_RECOLLECTS);\n"
                 "      {\n");
            g.first_pass = 0;
            gen_collect_all(&g, 8);
            bput(&b,
                 "      }\n"
                 "      if (best == wodev::kBestNone) return false;\n"
                 "    }\n"
                 "  }\n"
                 "};\n");
            eval_ops = 4;
            goto kernel_tail;
        }
        if (use_hlut)
            bput(&b, "#if WO_HBITS_LDS\n    wodev::LdsBits bits;\n    bits.p = sbits;\n#else\n    uint32_t bits[%u];\n#endif\n",
                 nw);
        else
            bput(&b, "    uint32_t bits[%u];\n", nw);
        for (uint32_t w = 0; w < nw; ++w) bput(&b, "    bits[%u] = 0u;\n", w);
        bput(&b, "    uint32_t cull[%u];  // bit k: BOUND k culled for this wave\n", ncw);
        for (uint32_t w = 0; w < ncw; ++w) bput(&b, "    cull[%u] = 0u;\n", w);
        /* First pass (culls, membership at t_min, every event), then the sweep;
         * the re-collect copy (events after the last processed one, when the
         * window had dropped some) is separate code so the common pass carries
         * none of its tests. */
        if (g.lds_events)
            bput(&b, "#if WO_JIT_LDS_EVENTS\n    wodev::LdsWindow win; win.ev = ev; win.clear();\n"
                     "#else\n    wodev::Window win; win.clear();\n#endif\n");
        else
            bput(&b, "    wodev::Window win; win.clear();\n");
        bput(&b,
             "    uint64_t after = 0ull, key = 0ull;\n"
             "    WO_MARK(\"collect_begin\");\n"
             "    {\n");
        g.first_pass = 1;
        gen_collect_all(&g, 6);
        bput(&b,
             "    }\n"
             "    WO_MARK(\"collect_end\");\n"
             "    WO_TMARK();\n"
             "    if (win.empty()) return false;\n"
             "    bool have = false;\n"
             "    uint32_t root = 0u;\n");
        if (g.first_event) {
            /* Waves whose lanes all start outside every primitive: the root is 0 at
             * t_min (the operators keep the empty set empty), the first event is an
             * entry, and the root after it is a per-primitive constant (single_root):
             * two evaluations saved when it flips. */
            uint32_t sr[64] = {0};
            for (uint32_t p = 0; p < n_prims && p < 64u * 32u; ++p) {
                int v = single_root(prog, n_recs, p);
                if (v < 0) g.err = 1;
                if (v > 0) sr[p / 32u] |= 1u << (p % 32u);
            }
            bput(&b, "    if (__ballot((bits[0]");
            for (uint32_t w = 1; w < nw; ++w) bput(&b, " | bits[%u]", w);
            bput(&b,
                 ") != 0u) == 0ull) {\n"
                 "      win.next(key);\n"
                 "      WO_WK(WO_WORK_SWEEP_STEPS);\n"
                 "      WO_WK_WAVE(WO_WORK_SWEEP_TRIPS);\n"
                 "      const uint32_t ord = ((uint32_t)key) >> 12;\n"
                 "      const uint32_t w = ord >> 5, m = 1u << (ord & 31u);\n"
                 "      uint32_t single = 0u;\n");
            if (use_hlut) bput(&b, "#if WO_HBITS_LDS\n      bits[w] ^= m;\n#else\n");
            for (uint32_t w = 0; w < nw; ++w) bput(&b, "      bits[%u] ^= w == %uu ? m : 0u;\n", w, w);
            if (use_hlut) bput(&b, "#endif\n");
            for (uint32_t w = 0; w < nw; ++w)
                if (sr[w]) bput(&b, "      single |= w == %uu ? (0x%08xu & m) : 0u;\n", w, sr[w]);
            bput(&b,
                 "      if (single != 0u) { wodev::hit_from_key(key, 1u, hit); return true; }\n"
                 "      have = true;  // root stays 0\n"
                 "    }\n");
        }
        if (n_uterms) {
            gen_union_sweep(&g, uterms, n_uterms, n_recs, nw);
            eval_ops = 12u + 2u * (nw - 1u);
        } else if (use_hlut) {
            bput(&b, "    ");
            for (uint32_t L = 0; L + 1u < hl.L; ++L) bput(&b, "uint32_t hv%u[%u]; ", L, (hl.k[L] + 31u) / 32u);
            bput(&b, "// WO_STATE_DECL\n"
                     "    uint32_t r;\n"
                     "    // WO_EVAL_BEGIN (every level's units from bits[], the root into r; tests/test_jit.py)\n"
                     "    {\n");
            hlut_emit_init(&b, &hl, nw, 6);
            bput(&b,
                 "    }\n"
                 "    // WO_EVAL_END\n"
                 "    for (;;) {\n"
                 "      if (have & (r != root)) { wodev::hit_from_key(key, r, hit); return true; }\n"
                 "      root = r;\n"
                 "      if (!win.next(key)) {  // key keeps the last processed event\n"
                 "        if (!win.dropped()) return false;\n"
                 "        after = key;\n"
                 "        WO_WK(WO_WORK_RECOLLECTS);\n"
                 "        win.clear();\n"
                 "        {\n");
            g.first_pass = 0;
            gen_collect_all(&g, 10);
            bput(&b,
                 "        }\n"
                 "        if (!win.next(key)) return false;\n"
                 "      }\n"
                 "      have = true;\n"
                 "      WO_WK(WO_WORK_SWEEP_STEPS);\n"
                 "      WO_WK_WAVE(WO_WORK_SWEEP_TRIPS);\n"
                 "      // WO_TOGGLE_BEGIN (the event's membership toggle and its units' update; tests/test_jit.py)\n"
                 "      {\n"
                 "        uint32_t ord = ((uint32_t)key) >> 12;\n"
                 "        uint32_t w = ord >> 5, m = 1u << (ord & 31u);\n");
            bput(&b, "#if WO_HBITS_LDS\n        bits[w] ^= m;\n#else\n");
            for (uint32_t w = 0; w < nw; ++w) bput(&b, "        bits[%u] ^= w == %uu ? m : 0u;\n", w, w);
            bput(&b, "#endif\n");
            hlut_emit_update(&b, &hl, nw, 8);
            bput(&b,
                 "      }\n"
                 "      // WO_TOGGLE_END\n"
                 "#if WO_SWEEP_UNROLL\n"
                 "      // a second event per trip while the window holds one (no re-collect here:\n"
                 "      // a lane whose window is empty goes round to the top)\n"
                 "      if (!win.empty()) {\n"
                 "        if (r != root) { wodev::hit_from_key(key, r, hit); return true; }\n"
                 "        root = r;\n"
                 "        win.next(key);\n"
                 "        WO_WK(WO_WORK_SWEEP_STEPS);\n"
                 "        {\n"
                 "          uint32_t ord = ((uint32_t)key) >> 12;\n"
                 "          uint32_t w = ord >> 5, m = 1u << (ord & 31u);\n");
            bput(&b, "#if WO_HBITS_LDS\n          bits[w] ^= m;\n#else\n");
            for (uint32_t w = 0; w < nw; ++w) bput(&b, "          bits[%u] ^= w == %uu ? m : 0u;\n", w, w);
            bput(&b, "#endif\n");
            hlut_emit_update(&b, &hl, nw, 10);
            bput(&b,
                 "        }\n"
                 "      }\n"
                 "#endif\n"
                 "    }\n"
                 "  }\n"
                 "};\n");
            /* per level: the entry's read and fields, the index (a word select per lower
             * word), the table read and bit, the unit's bit set */
            eval_ops = 0;
            for (uint32_t L = 0; L < hl.L; ++L) eval_ops += 12u + 2u * ((L ? (hl.k[L - 1] + 31u) / 32u : nw) - 1u);
        } else {
            /* (one membership word: the form above also compiles for up to four, but the
             * csg256 chain -- four words, a window of 5 -- measured the same 10.06 ms
             * with it as without; profiles/r06_ab_sweep_batch.txt) */
            if (nw == 1u) {
                /* Batch sweep (round 6, WO_SWEEP_BATCH): the root after each of the
                 * window's events in one straight pass -- the prefix states of the
                 * membership word (one XOR each) and their evaluations, which do not
                 * depend on one another -- and the first event whose root differs
                 * from the root at t_min is the hit.  The event loop ran a trip per
                 * event, each waiting on the last one's evaluation, for as many trips
                 * as the wave's slowest lane needed; here every lane does the same
                 * fixed work per window fill.  Same hit key and value as the loop. */
                bput(&b, "#if WO_SWEEP_BATCH && !WO_JIT_LDS_EVENTS\n    {\n      uint32_t r0;\n");
                gen_eval_block(&g, &lut, use_lut, n_recs, 6, "r0");
                bput(&b,
                     "      if (have & (r0 != root)) { wodev::hit_from_key(key, r0, hit); return true; }\n"
                     "      root = r0;\n"
                     "      uint64_t last = key;  // the last processed event (the first-event block's, or none)\n"
                     "      for (;;) {\n"
                     "        uint32_t bb[%u], hr = 0u;\n"
                     "        for (int w = 0; w < %u; ++w) bb[w] = bits[w];\n"
                     "        uint64_t hk = 0ull;\n"
                     "        bool found = false;\n"
                     "#pragma unroll\n"
                     "        for (int j = 0; j < wodev::kWindow; ++j) {\n"
                     "          const uint64_t kj = win.k[j];\n"
                     "          const bool v = kj != wodev::Window::kEmpty;\n"
                     "#if WO_SWEEP_BATCH_EXIT\n"
                     "          // the window is sorted: no lane has a later event to take once none has this one\n"
                     "          if (__ballot(v & !found) == 0ull) break;\n"
                     "#endif\n"
                     "          const uint32_t ord = ((uint32_t)kj) >> 12, m = v ? 1u << (ord & 31u) : 0u;\n",
                     nw, nw);
                if (nw == 1u)
                    bput(&b, "          bb[0] ^= m;\n");
                else
                    for (uint32_t w = 0; w < nw; ++w) bput(&b, "          bb[%u] ^= (ord >> 5) == %uu ? m : 0u;\n", w, w);
                bput(&b,
                     "          uint32_t rj;\n"
                     "          {\n"
                     "            const uint32_t bits[%u] = {bb[0]", nw);
                for (uint32_t w = 1; w < nw; ++w) bput(&b, ", bb[%u]", w);
                bput(&b, "};\n");
                gen_eval_block(&g, &lut, use_lut, n_recs, 12, "rj");
                bput(&b,
                     "          }\n"
                     "          WO_WK_IF(v & !found, WO_WORK_SWEEP_STEPS);\n"
                     "          const bool f = v & !found & (rj != root);\n"
                     "          last = v ? kj : last;\n"
                     "          hk = f ? kj : hk;\n"
                     "          hr = f ? rj : hr;\n"
                     "          found = found | f;\n"
                     "        }\n"
                     "        WO_WK_WAVE(WO_WORK_SWEEP_TRIPS);\n"
                     "        if (found) { wodev::hit_from_key(hk, hr, hit); return true; }\n"
                     "        for (int w = 0; w < %u; ++w) bits[w] = bb[w];\n"
                     "        if (!win.dropped()) return false;\n"
                     "        after = last;\n"
                     "        WO_WK(WO_WORK_RECOLLECTS);\n"
                     "        win.clear();\n"
                     "        {\n", nw);
                g.first_pass = 0;
                gen_collect_all(&g, 10);
                bput(&b,
                     "        }\n"
                     "        if (win.empty()) return false;\n"
                     "      }\n"
                     "    }\n"
                     "#else\n");
            }
            bput(&b,
                 "    for (;;) {\n"
                 "      uint32_t r;\n");
            bput(&b,
                 "      // WO_EVAL_BEGIN (the root's value from bits[] and cull[]; tests/test_jit.py compiles it on the host)\n"
                 "%s      {\n", use_lut ? "#if WO_JIT_LUT\n" : "");
            g.nbound = 0;
            if (use_lut) {
                lut_emit_eval(&b, &lut, 8);
                bput(&b, "      }\n#else\n      {\n");
            }
            {
                Term rt = gen_eval_flat(&g, 0, n_recs, 8);
                const uint32_t m = rt.kind ? (rt.P | rt.N) : 0u;
                eval_ops = rt.dl && dl_cost(&g, rt.dl) < rt.cost + (m ? 3u : 0u) ? dl_cost(&g, rt.dl)
                                                                                 : rt.cost + (m ? 3u : 0u);
                uint32_t rv = term_name(&g, &rt, 8);
                bput(&b, "        r = v%u ? 1u : 0u;\n      }\n", rv);
            }
            if (use_lut) {
                bput(&b, "#endif\n");
                eval_ops = 6u * lut.k + 2u; /* per subtree: index, address, read, bit; the root's shift */
            }
            bput(&b, "      // WO_EVAL_END\n");
            bput(&b,
                 "      if (have & (r != root)) { wodev::hit_from_key(key, r, hit); return true; }\n"
                 "      root = r;\n"
                 "      if (!win.next(key)) {  // key keeps the last processed event\n"
                 "        if (!win.dropped()) return false;\n"
                 "        after = key;\n"
                 "        WO_WK(WO_WORK_RECOLLECTS);\n"
                 "        win.clear();\n"
                 "        {\n");
            g.first_pass = 0;
            gen_collect_all(&g, 10);
            bput(&b,
                 "        }\n"
                 "        if (!win.next(key)) return false;\n"
                 "      }\n"
                 "      have = true;\n"
                 "      WO_WK(WO_WORK_SWEEP_STEPS);\n"
                     "      WO_WK_WAVE(WO_WORK_SWEEP_TRIPS);\n"
                 "      // WO_TOGGLE_BEGIN (the event's membership toggle; tests/test_jit.py)\n"
                 "      {\n"
                 "        uint32_t ord = ((uint32_t)key) >> 12;\n"
                 "        uint32_t w = ord >> 5, m = 1u << (ord & 31u);\n");
            for (uint32_t w = 0; w < nw; ++w) bput(&b, "        bits[%u] ^= w == %uu ? m : 0u;\n", w, w);
            bput(&b,
                 "      }\n"
                 "      // WO_TOGGLE_END\n"
                 "#if WO_SWEEP_UNROLL\n"
                 "      // a second event per trip while the window holds one (no re-collect here:\n"
                 "      // a lane whose window is empty goes round to the top)\n"
                 "      if (!win.empty()) {\n"
                 "        uint32_t r;\n"
                 "%s        {\n", use_lut ? "#if WO_JIT_LUT\n" : "");
            if (use_lut) {
                lut_emit_eval(&b, &lut, 10);
                bput(&b, "        }\n#else\n        {\n");
            }
            {
                g.nbound = 0;
                Term rt = gen_eval_flat(&g, 0, n_recs, 10);
                uint32_t rv = term_name(&g, &rt, 10);
                bput(&b, "          r = v%u ? 1u : 0u;\n        }\n", rv);
            }
            if (use_lut) bput(&b, "#endif\n");
            bput(&b,
                 "        if (r != root) { wodev::hit_from_key(key, r, hit); return true; }\n"
                 "        root = r;\n"
                 "        win.next(key);\n"
                 "        WO_WK(WO_WORK_SWEEP_STEPS);\n"
                 "        {\n"
                 "          uint32_t ord = ((uint32_t)key) >> 12;\n"
                 "          uint32_t w = ord >> 5, m = 1u << (ord & 31u);\n");
            for (uint32_t w = 0; w < nw; ++w) bput(&b, "          bits[%u] ^= w == %uu ? m : 0u;\n", w, w);
            bput(&b,
                 "        }\n"
                 "      }\n"
                 "#endif\n"
                 "    }\n");
            if (nw == 1u) bput(&b, "#endif  // WO_SWEEP_BATCH\n");
            bput(&b,
                 "  }\n"
                 "};\n");
        }
    }
kernel_tail:
    /* Waves per SIMD the register budget is sized for (measured, 1920x1080x64; round
     * 5, with camera-ray waves: the union count 9.39 / 9.24 / 9.55 ms at 8 / 7 / 6 -- at 8
     * it spills 35 VGPRs, 9.6 GB of scratch writes per frame -- csg32_nested 8.83 / 8.92
     * at 8 / 7, chain 11.47 / 11.81):
     * csg256 balanced / chain (128 primitives) 23.7 / 38.0 ms at 6, 21.3 / 33.8 at
     * 8; csg32 (18) 5.24 ms at 7 (8 LDS events), 5.19 at 8 (7 LDS events: 8
     * workgroups' LDS fit the CU only then). */
    bput(&b,
         "\n#ifndef WO_JIT_MIN_WAVES\n"
         "#define WO_JIT_MIN_WAVES %u\n#endif\n",
         n_uterms ? 7u : use_hlut ? ((n_prims + 31u) / 32u >= 4u ? 5u : 6u) : (n_prims > 64u || g.lds_events) ? 8u : 7u);
    bput(&b,
         "extern \"C\" __global__ __launch_bounds__(256, WO_JIT_MIN_WAVES) void wo_jit_pathtrace(\n"
         "    const WoRec* __restrict__ prog, const WoMaterial* __restrict__ mats, WoFrame fr, uint32_t local_rows,\n"
         "    float4* __restrict__ out, unsigned long long* __restrict__ seg_slots, wodev::PathLaunch tg) {\n"
         "  JitTracer tr;\n"
         "#if WO_JIT_LDS_EVENTS\n"
         "  __shared__ uint64_t s_ev[wodev::kLdsEvents * wodev::kBlock];\n"
         "  tr.ev = s_ev + threadIdx.x;\n"
         "#else\n"
         "  tr.ev = nullptr;\n"
         "#endif\n"
         "#if WO_JIT_LUT\n"
         "  __shared__ uint32_t s_lut[sizeof(kLut) / 4];\n"
         "  for (uint32_t i = threadIdx.x; i < sizeof(kLut) / 4; i += wodev::kBlock) s_lut[i] = kLut[i];\n"
         "  tr.lut = (const __attribute__((address_space(3))) uint32_t*)s_lut;\n"
         "#endif\n"
         "#if WO_JIT_HLUT\n"
         "  __shared__ uint32_t s_hinfo[sizeof(kHInfo) / 4], s_htab[sizeof(kHTab) / 4];\n"
         "  for (uint32_t i = threadIdx.x; i < sizeof(kHInfo) / 4; i += wodev::kBlock) s_hinfo[i] = kHInfo[i];\n"
         "  for (uint32_t i = threadIdx.x; i < sizeof(kHTab) / 4; i += wodev::kBlock) s_htab[i] = kHTab[i];\n"
         "  tr.hinfo = (const __attribute__((address_space(3))) uint32_t*)s_hinfo;\n"
         "  tr.htab = (const __attribute__((address_space(3))) uint32_t*)s_htab;\n"
         "#if WO_HBITS_LDS\n"
         "  __shared__ uint32_t s_bits[WO_HBITS_WORDS * wodev::kBlock];  // the membership words\n"
         "  tr.sbits = (wodev::LdsBits::P)(s_bits + threadIdx.x);\n"
         "#endif\n"
         "#endif\n"
         "#if WO_JIT_LDS_PROG  // hit-leaf and material reads from LDS (pathtrace_block's first barrier orders the copy)\n"
         "  __shared__ WoRec s_prog[%u];\n"
         "  __shared__ WoMaterial s_mats[%u];\n"
         "  __shared__ uint32_t s_ordpc[%u];\n"
         "  for (uint32_t i = threadIdx.x; i < %uu; i += wodev::kBlock)\n"
         "    reinterpret_cast<uint32_t*>(s_prog)[i] = reinterpret_cast<const uint32_t*>(prog)[i];\n"
         "  for (uint32_t i = threadIdx.x; i < %uu; i += wodev::kBlock)\n"
         "    reinterpret_cast<uint32_t*>(s_mats)[i] = reinterpret_cast<const uint32_t*>(mats)[i];\n"
         "  for (uint32_t i = threadIdx.x; i < %uu; i += wodev::kBlock) s_ordpc[i] = kOrdPc[i];\n"
         "  tr.prog = s_prog;\n"
         "  tr.ordpc = s_ordpc;\n"
         "  const WoMaterial* m = s_mats;\n"
         "#else\n"
         "  tr.prog = prog;\n"
         "  tr.ordpc = kOrdPc;\n"
         "  const WoMaterial* m = mats;\n"
         "#endif\n"
         "  wodev::pathtrace_block(tr, m, fr, local_rows, out, seg_slots, tg);\n"
         "}\n",
         n_recs ? n_recs : 1u, n_mats_used, n_prims ? n_prims : 1u, n_recs * 8u, n_mats_used * 8u, n_prims);
    /* the root evaluation's operation count per swept event, for bench.py's
     * executed-work roofline (0: not known, e.g. the postfix form) */
    if (eval_ops) bput(&b, "// wo_eval_ops_per_event %u\n", eval_ops);
    /* big tiles per resident workgroup the launch plan wants (trace_kernels.hip plan_tiles):
     * 3 for every tree since bench.py's renders stopped sharing a hardware queue (the
     * chain kept 8 before: 6.88 -> 6.99x at N = 8 with 3 now) */
    bput(&b, "// wo_share_tiles %u\n", 3u);
    free(g.dls);
    free(lut.table);
    hplan_free(&hl);
    rtree_free(&rtree);
    free(uterms);
    free(sprims);
    free(tunb);
    free(jterms);
    if (g.err || b.oom) {
        free(b.s);
        return NULL;
    }
    return b.s;
}
