/*
 * scene_compile.c -- flattens the renderer's node tables into the postfix CSG
 * program the kernels evaluate (layout: include/wololo/wo_scene.h).
 *
 * Input: the reference's node store semantics (renderer.c:180-202, 2220-2313):
 * spheres centred at their local origin, half-spaces {x : n.x <= 0} bounded by a
 * plane through the local origin, and binops whose operands are placed by a
 * Wo_Node_Argument = rotation quaternion then offset (renderer.h:22-27).  The
 * reference never uses these tables, so the semantics below are
 * this build's definition:
 *
 *   1. every root node (wo_renderer_isroot) is expanded into a world-space tree,
 *      composing the operand transforms in double precision; several roots are
 *      combined by a balanced union;
 *   2. maximal intersection-only subtrees of convex leaves become one convex
 *      primitive (WO_OP_PRIM) whose ray interval is [max entry, min exit];
 *   3. operands are emitted larger-stack-need first (Sethi-Ullman), so the
 *      kernel's 32-bit evaluation stack never overflows; DIFF becomes RDIFF
 *      when the subtrahend is emitted first;
 *   4. every maximal union cluster is re-bracketed as a bounding-volume hierarchy
 *      over its operands (regroup; union is associative and commutative);
 *   5. subtrees with >= 2 leaves and a finite extent get a conservative
 *      WO_OP_BOUND sphere so a wave whose rays all miss can skip them.
 */
#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "wo_internal.h"

enum { E_SPHERE, E_HALF, E_UNION, E_INTER, E_DIFF };

typedef struct ENode {
    int kind;
    int l, r;
    double c[3], rad;   /* sphere */
    double n[3], h;     /* half-space {x : n.x <= h} */
    uint32_t material;
    /* analysis */
    int convex;
    int need;
    int leaves;
    int bounded;
    double bc[3], br;
} ENode;

typedef struct Xf {
    double q[4]; /* w x y z, unit */
    double t[3];
} Xf;

typedef struct Ctx {
    Wo_Renderer* r;
    ENode* e;
    size_t n, cap;
    WoRec* prog;
    uint32_t n_recs, cap_recs;
    uint32_t ordinal;
    char* err;
    size_t errlen;
    int failed;
    int bound_min_leaves; /* smallest subtree (in leaves) that gets a BOUND record */
} Ctx;

#define MAX_EXPANDED_NODES (1u << 21)
#define MAX_GROUP_MEMBERS 2047u
/* expand, analyse, regroup and emit recurse once per tree level (a few hundred
 * bytes of native stack each): 8192 levels stay within ~3 MB, so a user-built
 * chain fails with an error instead of overflowing the thread's stack */
#define MAX_TREE_DEPTH 8192

static void fail(Ctx* c, const char* msg) {
    if (!c->failed) snprintf(c->err, c->errlen, "%s", msg);
    c->failed = 1;
}

static int new_enode(Ctx* c) {
    if (c->n >= MAX_EXPANDED_NODES) {
        fail(c, "scene expands to too many nodes (shared sub-graphs are instanced per use)");
        return -1;
    }
    if (c->n == c->cap) {
        size_t nc = c->cap ? c->cap * 2 : 64;
        ENode* ne = (ENode*)realloc(c->e, nc * sizeof(ENode));
        if (!ne) {
            fail(c, "out of host memory");
            return -1;
        }
        c->e = ne;
        c->cap = nc;
    }
    memset(&c->e[c->n], 0, sizeof(ENode));
    c->e[c->n].l = c->e[c->n].r = -1;
    return (int)c->n++;
}

/* ---- double-precision rigid transforms ---- */

static void quat_normalize(const Wo_Quaternion* in, double q[4]) {
    double w = in->real, x = in->imaginary.x, y = in->imaginary.y, z = in->imaginary.z;
    double len = sqrt(w * w + x * x + y * y + z * z);
    if (!(len > 0.0) || !isfinite(len)) {
        q[0] = 1.0;
        q[1] = q[2] = q[3] = 0.0;
        return;
    }
    q[0] = w / len;
    q[1] = x / len;
    q[2] = y / len;
    q[3] = z / len;
}

static void quat_rotate(const double q[4], const double v[3], double out[3]) {
    /* v' = v + 2w (u x v) + 2 u x (u x v), u = (x, y, z) */
    double ux = q[1], uy = q[2], uz = q[3], w = q[0];
    double cx = uy * v[2] - uz * v[1];
    double cy = uz * v[0] - ux * v[2];
    double cz = ux * v[1] - uy * v[0];
    double ccx = uy * cz - uz * cy;
    double ccy = uz * cx - ux * cz;
    double ccz = ux * cy - uy * cx;
    out[0] = v[0] + 2.0 * (w * cx + ccx);
    out[1] = v[1] + 2.0 * (w * cy + ccy);
    out[2] = v[2] + 2.0 * (w * cz + ccz);
}

static void quat_mul(const double a[4], const double b[4], double o[4]) {
    o[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    o[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    o[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
    o[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
}

/* world <- parent <- operand: x_world = P(A(x)) */
static Xf compose(const Xf* p, const Wo_Node_Argument* a) {
    Xf o;
    double qa[4], ta[3] = {a->offset.x, a->offset.y, a->offset.z}, rt[3];
    quat_normalize(&a->orientation, qa);
    quat_mul(p->q, qa, o.q);
    quat_rotate(p->q, ta, rt);
    for (int i = 0; i < 3; ++i) o.t[i] = rt[i] + p->t[i];
    return o;
}

static int expand(Ctx* c, Wo_Node node, const Xf* xf, int depth) {
    Wo_Renderer* r = c->r;
    if (c->failed) return -1;
    if (node >= r->node_count) {
        fail(c, "binop operand refers to a node that does not exist");
        return -1;
    }
    if (depth > MAX_TREE_DEPTH) {
        fail(c, "scene graph too deep (more than 8192 nested binops)");
        return -1;
    }
    const WoNodeInfo* ni = &r->nodes[node];
    int id = new_enode(c);
    if (id < 0) return -1;
    switch (ni->kind) {
    case WO_NODE_SPHERE: {
        ENode* e = &c->e[id];
        e->kind = E_SPHERE;
        for (int i = 0; i < 3; ++i) e->c[i] = xf->t[i];
        e->rad = fabs(ni->radius);
        e->material = ni->material < r->n_mats ? ni->material : 0u;
        return id;
    }
    case WO_NODE_HALFSPACE: {
        ENode* e = &c->e[id];
        double n[3] = {ni->normal.x, ni->normal.y, ni->normal.z};
        double len = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        e->kind = E_HALF;
        if (len > 0.0 && isfinite(len)) {
            for (int i = 0; i < 3; ++i) n[i] /= len;
            quat_rotate(xf->q, n, e->n);
            e->h = e->n[0] * xf->t[0] + e->n[1] * xf->t[1] + e->n[2] * xf->t[2];
        } else {
            /* degenerate normal: 0.x <= 0 holds everywhere (whole space) */
            e->n[0] = e->n[1] = e->n[2] = 0.0;
            e->h = 0.0;
        }
        e->material = ni->material < r->n_mats ? ni->material : 0u;
        return id;
    }
    default: {
        Xf xl = compose(xf, &ni->left);
        Xf xr = compose(xf, &ni->right);
        int l = expand(c, ni->left.node, &xl, depth + 1);
        int rr = expand(c, ni->right.node, &xr, depth + 1);
        if (l < 0 || rr < 0) return -1;
        ENode* e = &c->e[id];
        e->kind = ni->kind == WO_NODE_UNION ? E_UNION : ni->kind == WO_NODE_INTERSECTION ? E_INTER : E_DIFF;
        e->l = l;
        e->r = rr;
        return id;
    }
    }
}

static int make_union(Ctx* c, const int* roots, int n) {
    if (n == 1) return roots[0];
    int h = n / 2;
    int l = make_union(c, roots, h);
    int r = make_union(c, roots + h, n - h);
    if (l < 0 || r < 0) return -1;
    int id = new_enode(c);
    if (id < 0) return -1;
    c->e[id].kind = E_UNION;
    c->e[id].l = l;
    c->e[id].r = r;
    return id;
}

/* ---- bounds ---- */

static void enclose(const double c1[3], double r1, const double c2[3], double r2, double oc[3], double* orad) {
    double dv[3] = {c2[0] - c1[0], c2[1] - c1[1], c2[2] - c1[2]};
    double d = sqrt(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]);
    if (d + r2 <= r1) {
        memcpy(oc, c1, sizeof(double) * 3);
        *orad = r1;
        return;
    }
    if (d + r1 <= r2) {
        memcpy(oc, c2, sizeof(double) * 3);
        *orad = r2;
        return;
    }
    double R = 0.5 * (d + r1 + r2);
    double s = (R - r1) / d;
    for (int i = 0; i < 3; ++i) oc[i] = c1[i] + dv[i] * s;
    *orad = R;
}

static double dot3d(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static void cross3d(const double a[3], const double b[3], double o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

/* Bounding sphere of the polytope {x : n_i.x <= h_i}; returns 0 if unbounded/empty. */
static int polytope_bound(const double (*n)[3], const double* h, int k, double oc[3], double* orad) {
    /* O(k^4): callers pass at most 64 planes; more are treated as unbounded */
    if (k < 4 || k > 64) return 0;
    int any_pair = 0;
    for (int i = 0; i < k; ++i)
        for (int j = i + 1; j < k; ++j) {
            double d[3];
            cross3d(n[i], n[j], d);
            double dl = sqrt(dot3d(d, d));
            if (dl < 1e-12) continue;
            any_pair = 1;
            for (int s = -1; s <= 1; s += 2) {
                int recedes = 1;
                for (int m = 0; m < k && recedes; ++m) recedes = s * dot3d(n[m], d) <= 1e-9 * dl;
                if (recedes) return 0;
            }
        }
    if (!any_pair) return 0;
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    int nv = 0;
    /* vertices: every independent triple of planes, kept if it satisfies all constraints */
    const size_t kk = (size_t)k;
    double* verts = (double*)malloc(sizeof(double) * 3 * (kk * kk * kk / 6 + 8));
    if (!verts) return 0;
    for (int a = 0; a < k; ++a)
        for (int b = a + 1; b < k; ++b)
            for (int cidx = b + 1; cidx < k; ++cidx) {
                double bxc[3], cxa[3], axb[3];
                cross3d(n[b], n[cidx], bxc);
                cross3d(n[cidx], n[a], cxa);
                cross3d(n[a], n[b], axb);
                double det = dot3d(n[a], bxc);
                if (fabs(det) < 1e-12) continue;
                double x[3];
                for (int i = 0; i < 3; ++i) x[i] = (h[a] * bxc[i] + h[b] * cxa[i] + h[cidx] * axb[i]) / det;
                int ok = 1;
                for (int m = 0; m < k && ok; ++m) ok = dot3d(n[m], x) <= h[m] + 1e-7 * (1.0 + fabs(h[m]));
                if (!ok) continue;
                for (int i = 0; i < 3; ++i) {
                    verts[nv * 3 + i] = x[i];
                    if (x[i] < lo[i]) lo[i] = x[i];
                    if (x[i] > hi[i]) hi[i] = x[i];
                }
                ++nv;
            }
    if (nv == 0) {
        free(verts);
        return 0;
    }
    double rad = 0.0;
    for (int i = 0; i < 3; ++i) oc[i] = 0.5 * (lo[i] + hi[i]);
    for (int v = 0; v < nv; ++v) {
        double dx = verts[v * 3] - oc[0], dy = verts[v * 3 + 1] - oc[1], dz = verts[v * 3 + 2] - oc[2];
        double d = sqrt(dx * dx + dy * dy + dz * dz);
        if (d > rad) rad = d;
    }
    free(verts);
    *orad = rad;
    return 1;
}

static void collect_members(Ctx* c, int id, int* out, int* n) {
    ENode* e = &c->e[id];
    if (e->kind == E_SPHERE || e->kind == E_HALF) {
        out[(*n)++] = id;
        return;
    }
    collect_members(c, e->l, out, n);
    collect_members(c, e->r, out, n);
}

/* Operands of the union cluster under `id` (already analysed, bounded). */
static void union_atoms_box(Ctx* c, int id, double lo[3], double hi[3]) {
    const ENode* e = &c->e[id];
    if (e->kind == E_UNION && !e->convex) {
        union_atoms_box(c, e->l, lo, hi);
        union_atoms_box(c, e->r, lo, hi);
        return;
    }
    for (int k = 0; k < 3; ++k) {
        if (e->bc[k] - e->br < lo[k]) lo[k] = e->bc[k] - e->br;
        if (e->bc[k] + e->br > hi[k]) hi[k] = e->bc[k] + e->br;
    }
}
static void union_atoms_radius(Ctx* c, int id, const double oc[3], double* orad) {
    const ENode* e = &c->e[id];
    if (e->kind == E_UNION && !e->convex) {
        union_atoms_radius(c, e->l, oc, orad);
        union_atoms_radius(c, e->r, oc, orad);
        return;
    }
    double d[3] = {e->bc[0] - oc[0], e->bc[1] - oc[1], e->bc[2] - oc[2]};
    double r = sqrt(dot3d(d, d)) + e->br;
    if (r > *orad) *orad = r;
}

/* Post-order analysis: convexity, stack need, leaf count, bounds. */
static void analyse(Ctx* c, int id) {
    ENode* e = &c->e[id];
    if (e->kind == E_SPHERE) {
        e->convex = 1;
        e->need = 1;
        e->leaves = 1;
        e->bounded = 1;
        memcpy(e->bc, e->c, sizeof e->bc);
        e->br = e->rad;
        return;
    }
    if (e->kind == E_HALF) {
        e->convex = 1;
        e->need = 1;
        e->leaves = 1;
        e->bounded = 0;
        return;
    }
    analyse(c, e->l);
    analyse(c, e->r);
    e = &c->e[id];
    ENode* L = &c->e[e->l];
    ENode* R = &c->e[e->r];
    e->leaves = L->leaves + R->leaves;
    e->convex = e->kind == E_INTER && L->convex && R->convex;
    if (e->convex) {
        e->need = 1;
    } else {
        e->need = L->need == R->need ? L->need + 1 : (L->need > R->need ? L->need : R->need);
    }
    e->bounded = 0;
    if (e->convex) {
        /* tightest member sphere, else the polytope of the half-spaces */
        int cnt = 0;
        int* mem = (int*)malloc(sizeof(int) * (size_t)e->leaves);
        if (!mem) return;
        collect_members(c, id, mem, &cnt);
        e = &c->e[id];
        double best = INFINITY;
        int nh = 0;
        for (int i = 0; i < cnt; ++i) {
            ENode* m = &c->e[mem[i]];
            if (m->kind == E_SPHERE) {
                if (m->rad < best) {
                    best = m->rad;
                    memcpy(e->bc, m->c, sizeof e->bc);
                    e->br = m->rad;
                    e->bounded = 1;
                }
            } else {
                ++nh;
            }
        }
        if (!e->bounded && nh >= 4 && nh <= 64) {
            double (*nn)[3] = (double (*)[3])malloc(sizeof(double) * 3 * (size_t)nh);
            double* hh = (double*)malloc(sizeof(double) * (size_t)nh);
            if (nn && hh) {
                int j = 0;
                for (int i = 0; i < cnt; ++i) {
                    ENode* m = &c->e[mem[i]];
                    if (m->kind != E_HALF) continue;
                    memcpy(nn[j], m->n, sizeof(double) * 3);
                    hh[j] = m->h;
                    ++j;
                }
                double oc[3], orad;
                if (polytope_bound((const double (*)[3])nn, hh, nh, oc, &orad)) {
                    memcpy(e->bc, oc, sizeof oc);
                    e->br = orad;
                    e->bounded = 1;
                }
            }
            free(nn);
            free(hh);
        }
        free(mem);
        return;
    }
    if (e->kind == E_UNION) {
        if (L->bounded && R->bounded) {
            enclose(L->bc, L->br, R->bc, R->br, e->bc, &e->br);
            e->bounded = 1;
            /* pairwise enclosing spheres grow loose with depth: also try the sphere
             * around the AABB of the cluster's operand spheres, keep the smaller */
            if (e->leaves <= 4096) {
                double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
                union_atoms_box(c, id, lo, hi);
                double oc[3], orad = 0.0;
                for (int k = 0; k < 3; ++k) oc[k] = 0.5 * (lo[k] + hi[k]);
                union_atoms_radius(c, id, oc, &orad);
                if (orad < e->br) {
                    memcpy(e->bc, oc, sizeof oc);
                    e->br = orad;
                }
            }
        }
    } else if (e->kind == E_INTER) {
        const ENode* pick = NULL;
        if (L->bounded) pick = L;
        if (R->bounded && (!pick || R->br < pick->br)) pick = R;
        if (pick) {
            memcpy(e->bc, pick->bc, sizeof e->bc);
            e->br = pick->br;
            e->bounded = 1;
        }
    } else { /* difference: contained in the minuend */
        if (L->bounded) {
            memcpy(e->bc, L->bc, sizeof e->bc);
            e->br = L->br;
            e->bounded = 1;
        }
    }
}

/* ---- union regrouping ---- */

/* Union is associative and commutative, so every maximal union cluster (a union
 * node and its union descendants) may be re-bracketed freely.  The scene's own
 * bracketing follows the order the caller added nodes in (the RTIOW cover adds
 * its spheres row by row: a balanced union of such a list groups long thin
 * strips whose bounding spheres are huge).  The cluster's operands are rebuilt
 * into a bounding-volume hierarchy instead: median split of the operands'
 * bounding-sphere centres along the longest axis, unbounded operands (half-
 * spaces) unioned on top.  The set the program describes is unchanged. */
typedef struct SortKey {
    double key;
    int id;
} SortKey;

static int cmp_sortkey(const void* a, const void* b) {
    const SortKey* x = (const SortKey*)a;
    const SortKey* y = (const SortKey*)b;
    if (x->key < y->key) return -1;
    if (x->key > y->key) return 1;
    return x->id < y->id ? -1 : x->id > y->id;
}

static int union_of(Ctx* c, int l, int r) {
    int id = new_enode(c);
    if (id < 0) return -1;
    c->e[id].kind = E_UNION;
    c->e[id].l = l;
    c->e[id].r = r;
    return id;
}

/* Running box of operand bounding spheres; its surface area. */
typedef struct Box3 {
    double lo[3], hi[3];
} Box3;
static void box_reset(Box3* b) {
    for (int k = 0; k < 3; ++k) {
        b->lo[k] = INFINITY;
        b->hi[k] = -INFINITY;
    }
}
static void box_add(Box3* b, const ENode* e) {
    for (int k = 0; k < 3; ++k) {
        if (e->bc[k] - e->br < b->lo[k]) b->lo[k] = e->bc[k] - e->br;
        if (e->bc[k] + e->br > b->hi[k]) b->hi[k] = e->bc[k] + e->br;
    }
}
static double box_area(const Box3* b) {
    const double x = b->hi[0] - b->lo[0], y = b->hi[1] - b->lo[1], z = b->hi[2] - b->lo[2];
    return 2.0 * (x * y + y * z + z * x);
}

/* Sort along the longest centre axis, then split where the surface-area cost
 * (box area x operands, both sides) is least; clusters of < 16 operands split
 * at the median.  Measured (1080p64): rtiow_cover 32.4 -> 30.3 ms, csg256 balanced
 * 15.7 -> 15.4 with the area split; csg32's 11-operand cluster is better at
 * the median (5.29 vs 5.35). */
static int bvh_build(Ctx* c, int* ids, int n, SortKey* tmp, int sah) {
    if (n == 1) return ids[0];
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
            double v = c->e[ids[i]].bc[k];
            if (v < lo[k]) lo[k] = v;
            if (v > hi[k]) hi[k] = v;
        }
    int axis = 0;
    for (int k = 1; k < 3; ++k)
        if (hi[k] - lo[k] > hi[axis] - lo[axis]) axis = k;
    for (int i = 0; i < n; ++i) {
        tmp[i].key = c->e[ids[i]].bc[axis];
        tmp[i].id = ids[i];
    }
    qsort(tmp, (size_t)n, sizeof(SortKey), cmp_sortkey);
    for (int i = 0; i < n; ++i) ids[i] = tmp[i].id;
    int h = n / 2;
    if (sah && n > 4) {
        /* prefix areas left to right in tmp[].key, then sweep from the right */
        double* left = (double*)malloc(sizeof(double) * (size_t)n);
        if (left) {
            Box3 bx;
            box_reset(&bx);
            for (int i = 1; i < n; ++i) {
                box_add(&bx, &c->e[ids[i - 1]]);
                left[i] = box_area(&bx) * i;
            }
            box_reset(&bx);
            double best = INFINITY;
            for (int i = n - 1; i >= 1; --i) {
                box_add(&bx, &c->e[ids[i]]);
                double cost = left[i] + box_area(&bx) * (n - i);
                if (cost < best) {
                    best = cost;
                    h = i;
                }
            }
            free(left);
        }
    }
    int l = bvh_build(c, ids, h, tmp, sah);
    int r = bvh_build(c, ids + h, n - h, tmp, sah);
    if (l < 0 || r < 0) return -1;
    return union_of(c, l, r);
}

static int regroup(Ctx* c, int id);

static int gather_union_operands(Ctx* c, int id, int** ops, int* n, int* cap) {
    if (c->e[id].kind == E_UNION) {
        int l = c->e[id].l, r = c->e[id].r;
        if (gather_union_operands(c, l, ops, n, cap)) return -1;
        return gather_union_operands(c, r, ops, n, cap);
    }
    if (*n == *cap) {
        int nc = *cap ? *cap * 2 : 16;
        int* no = (int*)realloc(*ops, sizeof(int) * (size_t)nc);
        if (!no) {
            fail(c, "out of host memory");
            return -1;
        }
        *ops = no;
        *cap = nc;
    }
    (*ops)[(*n)++] = id;
    return 0;
}

static int regroup(Ctx* c, int id) {
    if (c->failed) return -1;
    int kind = c->e[id].kind;
    if (kind == E_SPHERE || kind == E_HALF) return id;
    if (kind != E_UNION) {
        int l = regroup(c, c->e[id].l);
        int r = regroup(c, c->e[id].r);
        if (l < 0 || r < 0) return -1;
        c->e[id].l = l;
        c->e[id].r = r;
        return id;
    }
    int *ops = NULL, n = 0, cap = 0;
    if (gather_union_operands(c, id, &ops, &n, &cap)) {
        free(ops);
        return -1;
    }
    int nb = 0;
    for (int i = 0; i < n; ++i) {
        ops[i] = regroup(c, ops[i]);
        if (ops[i] < 0) {
            free(ops);
            return -1;
        }
        analyse(c, ops[i]);
        if (c->e[ops[i]].bounded) { /* bounded operands first, in their original order */
            int t = ops[i];
            memmove(ops + nb + 1, ops + nb, sizeof(int) * (size_t)(i - nb));
            ops[nb++] = t;
        }
    }
    SortKey* tmp = (SortKey*)malloc(sizeof(SortKey) * (size_t)n);
    if (!tmp) {
        free(ops);
        fail(c, "out of host memory");
        return -1;
    }
    /* Giant operands (bounding radius > 16x the cluster's median, e.g. an RTIOW
     * ground sphere of radius 1000) would give every BOUND above them a giant
     * sphere that no ray misses: they join the unbounded operands on top. */
    if (nb > 2) {
        for (int i = 0; i < nb; ++i) {
            tmp[i].key = c->e[ops[i]].br;
            tmp[i].id = ops[i];
        }
        qsort(tmp, (size_t)nb, sizeof(SortKey), cmp_sortkey);
        const double lim = 16.0 * tmp[nb / 2].key;
        int k = 0;
        for (int i = 0; i < nb; ++i)
            if (!(c->e[ops[i]].br > lim)) tmp[k++].id = ops[i];
        int kept = k;
        for (int i = 0; i < nb; ++i)
            if (c->e[ops[i]].br > lim) tmp[k++].id = ops[i];
        for (int i = 0; i < nb; ++i) ops[i] = tmp[i].id;
        nb = kept;
    }
    int root = nb ? bvh_build(c, ops, nb, tmp, nb >= 16) : -1;
    /* giant and unbounded operands go first in the program (postfix order), so a
     * traversal meets a ground plane or sphere -- the likely nearest hit of a
     * downward ray -- before the hierarchy it may then prune */
    for (int i = nb; i < n && !c->failed; ++i) root = root < 0 ? ops[i] : union_of(c, ops[i], root);
    free(tmp);
    free(ops);
    return c->failed ? -1 : root;
}

/* ---- emission ---- */

static WoRec* push_rec(Ctx* c) {
    if (c->failed) return NULL;
    if (c->n_recs == c->cap_recs) {
        uint32_t nc = c->cap_recs ? c->cap_recs * 2u : 64u;
        WoRec* np = (WoRec*)realloc(c->prog, nc * sizeof(WoRec));
        if (!np) {
            fail(c, "out of host memory");
            return NULL;
        }
        c->prog = np;
        c->cap_recs = nc;
    }
    WoRec* rec = &c->prog[c->n_recs++];
    memset(rec, 0, sizeof *rec);
    return rec;
}

static float round_up_f(double v) {
    float f = (float)v;
    if ((double)f < v) f = nextafterf(f, INFINITY);
    return f;
}

static void emit_leaf(Ctx* c, const ENode* m) {
    WoRec* rec = push_rec(c);
    if (!rec) return;
    rec->u0 = m->material;
    if (m->kind == E_SPHERE) {
        /* every fp32 value of the record finite: the kernels' square root of the
         * discriminant r^2 - ll (sqrt_cr) is exact below +inf only */
        const double r2 = m->rad * m->rad;
        if (!(r2 < (double)FLT_MAX) || !isfinite(m->c[0]) || !isfinite(m->c[1]) || !isfinite(m->c[2]) ||
            !(fabs(m->c[0]) < (double)FLT_MAX && fabs(m->c[1]) < (double)FLT_MAX && fabs(m->c[2]) < (double)FLT_MAX)) {
            fail(c, "sphere leaf out of fp32 range (radius^2 or centre not finite)");
            return;
        }
        rec->op = WO_LEAF_SPHERE;
        rec->f[0] = (float)m->c[0];
        rec->f[1] = (float)m->c[1];
        rec->f[2] = (float)m->c[2];
        rec->f[3] = (float)(m->rad * m->rad);
        rec->f[4] = m->rad > 0.0 ? (float)(1.0 / m->rad) : 0.0f;
    } else {
        rec->op = WO_LEAF_HALFSPACE;
        rec->f[0] = (float)m->n[0];
        rec->f[1] = (float)m->n[1];
        rec->f[2] = (float)m->n[2];
        rec->f[3] = (float)m->h;
        /* axis-aligned normal (exactly, in fp32): flag the axis (wo_scene.h) */
        for (int a = 0; a < 3; ++a) {
            int b = (a + 1) % 3, c = (a + 2) % 3;
            if ((rec->f[a] == 1.0f || rec->f[a] == -1.0f) && rec->f[b] == 0.0f && rec->f[c] == 0.0f) rec->u1 = 1u + a;
        }
    }
}

/* `outer_r`: radius of the innermost BOUND already enclosing this subtree
 * (INFINITY if none).  A nested bound only pays if it is clearly tighter. */
static void emit(Ctx* c, int id, double outer_r) {
    if (c->failed) return;
    ENode* e = &c->e[id];
    int use_bound = e->bounded && e->leaves >= c->bound_min_leaves && e->br < 0.7 * outer_r;
    double inner_r = use_bound ? e->br : outer_r;
    uint32_t bidx = 0;
    if (use_bound) {
        bidx = c->n_recs;
        WoRec* b = push_rec(c);
        if (!b) return;
        double cn = sqrt(dot3d(e->bc, e->bc));
        double R = e->br * (1.0 + 1e-4) + 1e-5 * (cn + e->br) + 1e-6;
        b->op = WO_OP_BOUND;
        b->u1 = (uint32_t)e->leaves;
        b->f[0] = (float)e->bc[0];
        b->f[1] = (float)e->bc[1];
        b->f[2] = (float)e->bc[2];
        b->f[3] = round_up_f(R * R);
        b->f[4] = round_up_f(R);
    }
    if (e->convex) {
        int cnt = 0;
        int* mem = (int*)malloc(sizeof(int) * (size_t)e->leaves);
        if (!mem) {
            fail(c, "out of host memory");
            return;
        }
        collect_members(c, id, mem, &cnt);
        if ((uint32_t)cnt > MAX_GROUP_MEMBERS) {
            free(mem);
            fail(c, "an intersection-only sub-tree has more than 2047 leaves");
            return;
        }
        WoRec* p = push_rec(c);
        if (!p) {
            free(mem);
            return;
        }
        {
            /* the sphere members in ascending radius (stable; half-spaces keep their
             * slots, so slab face pairs stay adjacent): the kernels skip a primitive's
             * later members once its interval is empty on a whole wave, and the
             * smallest sphere empties it most often */
            for (int i = 1; i < cnt; ++i) {
                if (c->e[mem[i]].kind != E_SPHERE) continue;
                for (int j = i; j > 0;) {
                    int k = j - 1;
                    while (k >= 0 && c->e[mem[k]].kind != E_SPHERE) --k;
                    if (k < 0 || !(c->e[mem[j]].rad < c->e[mem[k]].rad)) break;
                    int t = mem[j];
                    mem[j] = mem[k];
                    mem[k] = t;
                    j = k;
                }
            }
        }
        p->op = WO_OP_PRIM;
        p->u0 = (uint32_t)cnt;
        p->u1 = c->ordinal++;
        for (int i = 0; i < cnt; ++i) emit_leaf(c, &c->e[mem[i]]);
        free(mem);
    } else {
        int A = e->l, B = e->r, kind = e->kind;
        uint32_t op;
        if (c->e[B].need > c->e[A].need) {
            emit(c, B, inner_r);
            emit(c, A, inner_r);
            op = kind == E_UNION ? WO_OP_UNION : kind == E_INTER ? WO_OP_INTER : WO_OP_RDIFF;
        } else {
            emit(c, A, inner_r);
            emit(c, B, inner_r);
            op = kind == E_UNION ? WO_OP_UNION : kind == E_INTER ? WO_OP_INTER : WO_OP_DIFF;
        }
        WoRec* rec = push_rec(c);
        if (!rec) return;
        rec->op = op;
    }
    if (use_bound && !c->failed) c->prog[bidx].u0 = c->n_recs;
}

int wo_compile_scene(Wo_Renderer* r, char* err, size_t errlen) {
    Ctx c;
    memset(&c, 0, sizeof c);
    c.r = r;
    c.err = err;
    c.errlen = errlen;
    c.bound_min_leaves = 2;

    int* roots = (int*)malloc(sizeof(int) * (r->node_count ? r->node_count : 1));
    if (!roots) {
        snprintf(err, errlen, "out of host memory");
        return -1;
    }
    int nroots = 0;
    Xf id;
    id.q[0] = 1.0;
    id.q[1] = id.q[2] = id.q[3] = 0.0;
    id.t[0] = id.t[1] = id.t[2] = 0.0;
    for (size_t i = 0; i < r->node_count && !c.failed; ++i) {
        if (r->nonroot[i / 64] & (1ull << (i % 64))) continue;
        int e = expand(&c, (Wo_Node)i, &id, 0);
        if (e >= 0) roots[nroots++] = e;
    }
    if (!c.failed && nroots > 0) {
        int root = make_union(&c, roots, nroots);
        if (root >= 0 && !c.failed) root = regroup(&c, root);
        if (root >= 0 && !c.failed) {
            analyse(&c, root);
            if (c.e[root].need > 31) fail(&c, "CSG tree needs an evaluation stack deeper than 31");
            emit(&c, root, INFINITY);
            if (!c.failed && c.ordinal >= (1u << 20)) fail(&c, "too many primitives (max 2^20-1)");
        }
    }
    free(roots);
    free(c.e);
    if (c.failed) {
        free(c.prog);
        return -1;
    }
    if (!c.prog) { /* empty scene: keep a valid (zero-record) program pointer */
        c.prog = (WoRec*)calloc(1, sizeof(WoRec));
        c.cap_recs = 1;
        if (!c.prog) {
            snprintf(err, errlen, "out of host memory");
            return -1;
        }
    }
    free(r->prog);
    r->prog = c.prog;
    r->n_recs = c.n_recs;
    r->cap_recs = c.cap_recs;
    r->n_prims = c.ordinal;
    r->dirty = 0;
    r->dev_stale = 1;
    return 0;
}

/* RTIOW camera (positionable camera + defocus blur), resolved in double then
 * rounded to the floats the kernel and the oracle both consume. */
void wo_resolve_camera(WoCameraDesc const* d, uint32_t width, uint32_t height, WoCamera* out) {
    double aspect = height ? (double)width / (double)height : 1.0;
    double theta = d->vfov_deg * (3.14159265358979323846 / 180.0);
    double h = tan(theta / 2.0);
    double vh = 2.0 * h, vw = aspect * vh;
    double from[3] = {d->look_from.x, d->look_from.y, d->look_from.z};
    double at[3] = {d->look_at.x, d->look_at.y, d->look_at.z};
    double up[3] = {d->view_up.x, d->view_up.y, d->view_up.z};
    double w[3] = {from[0] - at[0], from[1] - at[1], from[2] - at[2]};
    double wl = sqrt(dot3d(w, w));
    if (!(wl > 0.0)) {
        w[0] = 0.0;
        w[1] = 0.0;
        w[2] = 1.0;
        wl = 1.0;
    }
    for (int i = 0; i < 3; ++i) w[i] /= wl;
    double u[3];
    cross3d(up, w, u);
    double ul = sqrt(dot3d(u, u));
    if (!(ul > 1e-12)) {
        double alt[3] = {fabs(w[0]) < 0.9 ? 1.0 : 0.0, fabs(w[0]) < 0.9 ? 0.0 : 1.0, 0.0};
        cross3d(alt, w, u);
        ul = sqrt(dot3d(u, u));
    }
    for (int i = 0; i < 3; ++i) u[i] /= ul;
    double v[3];
    cross3d(w, u, v);
    double fd = d->focus_dist > 0.0 ? d->focus_dist : 1.0;
    for (int i = 0; i < 3; ++i) {
        double hz = fd * vw * u[i];
        double vt = fd * vh * v[i];
        out->origin[i] = (float)from[i];
        out->horizontal[i] = (float)hz;
        out->vertical[i] = (float)vt;
        out->lower_left[i] = (float)(from[i] - hz / 2.0 - vt / 2.0 - fd * w[i]);
        out->u[i] = (float)u[i];
        out->v[i] = (float)v[i];
    }
    out->lens_radius = (float)(d->aperture > 0.0 ? d->aperture / 2.0 : 0.0);
    out->pad[0] = out->pad[1] = out->pad[2] = 0.0f;
}
