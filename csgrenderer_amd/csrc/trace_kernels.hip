// trace_kernels.hip -- the per-pixel hot path of the wololo renderer for gfx950
// (MI355X, CDNA4, wave64).  Replaces the reference's fragment stage
// (src/wololo/renderer/ubershader1.frag:19-163, one invocation per pixel,
// launched by draw_frame_with_renderer, renderer.c:2085-2219).
//
// Kernels
//   ubershader_kernel  the reference shader restated bit-for-bit in IEEE fp32
//                      (sin hoisted to the host).  HBM-store bound, 16 B/pixel.
//   pathtrace_kernel   CSG path tracer, INTERPRETER form: walks the compiled
//                      postfix program (staged in LDS when it fits), wave-uniform
//                      BOUND culling, sorted event window, bit-stack evaluation.
//   wo_jit_pathtrace   the same path tracer SPECIALISED per scene: source from
//                      scene_jit.c, compiled here with hiprtc at scene upload.
//   assemble_kernel    un-interleaves row-cyclic rank tiles after the gather.
// The shared device code (math, RNG, leaves, event window, shading, path loop)
// is wo_device_common.h; both forms agree bit-for-bit with oracle/oracle.c.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <dlfcn.h>
#include <limits.h>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "wo_dev.h"
// the static kernels raise the wave priority while a hit's leaf and material loads issue
// (RTIOW cover 11.50 -> 11.47 ms in two pairs; the specialised kernel keeps 0: csg32 3.261 vs 3.266)
#ifndef WO_SHADE_PRIO
#define WO_SHADE_PRIO 1
#endif
#include "wo_device_common.h"
#include "wololo/wo_scene.h"

#include "jit_sources.inc"
#include "static_key.inc"  // WO_STATIC_SRC_SHA: the library kernels' source identity

#pragma clang fp contract(off)

namespace {

using namespace wodev;

// 4-bit op codes of the per-wave compacted program (8 per dword).
// (2..5 are WO_OP_UNION, _INTER, _DIFF, _RDIFF unchanged)
constexpr uint32_t kCodePrim = 1, kCodeUnion = 2, kCodeConst0 = 6;

// Per-wave LDS scratch layout (dwords), computed on the host.
struct KLayout {
    uint32_t codes_words;  // packed 4-bit codes of the compacted program
    uint32_t ordpc_off;    // primitive ordinal -> program counter
    uint32_t hib_off;      // membership bits of ordinals >= 64: [word][64 lanes]
    uint32_t wave_words;   // stride between waves
};

struct ProgPtr {
    const WoRec* p;
    __device__ __forceinline__ WoRec operator[](uint32_t i) const { return p[i]; }
};

// `inv`/`have_inv`: the ray's reciprocal direction, computed on the first
// axis-aligned half-space met (wave-uniform condition).
template <bool kCount, class Prog>
__device__ __forceinline__ Ivl prim_interval(Prog prog, uint32_t pc, uint32_t count, F3 o, F3 d, F3& inv,
                                             bool& have_inv, WorkCounts& wk) {
    Ivl iv;
    for (uint32_t m = 0; m < count; ++m) {
        WoRec L = prog[pc + 1u + m];
        uint32_t kind = uni(L.op);
        WO_WK(kind == WO_LEAF_SPHERE ? WO_WORK_SPHERE_TESTS : WO_WORK_HALFSPACE_TESTS);
        if (kind == WO_LEAF_HALFSPACE && !have_inv && uni(L.u1) != 0u) {
            inv = f3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
            have_inv = true;
        }
        float la, lb;
        leaf_interval(L, kind, o, d, inv, la, lb);
        if (m == 0u)
            ivl_first(iv, la, lb);
        else
            ivl_meet(iv, la, lb, m);
    }
    return iv;
}

// Interpreter: walks the program record by record (wave-uniform pc).
template <bool kCountT>
struct InterpTracer {
    static constexpr bool kCount = kCountT;
    WorkCounts wk;
    uint64_t tmark;  // section timing (counting builds)
    ProgPtr prog;
    uint32_t nrec;
    uint32_t* codes;
    uint32_t* ordpc;
    uint32_t* hib;
    uint32_t lane;
    uint32_t ncodes;  // wave-uniform
    uint32_t nprims;  // wave-uniform, primitives surviving the cull
    uint64_t bits;    // membership of ordinals < 64

    __device__ __forceinline__ uint32_t bit(uint32_t ord) const {
        if (ord < 64u) return (uint32_t)(bits >> ord) & 1u;
        uint32_t w = (ord - 64u) >> 5;
        return (hib[w * 64u + lane] >> ((ord - 64u) & 31u)) & 1u;
    }
    __device__ __forceinline__ void toggle(uint32_t ord) {
        if (ord < 64u) {
            bits ^= 1ull << ord;
        } else {
            uint32_t w = (ord - 64u) >> 5;
            hib[w * 64u + lane] ^= 1u << ((ord - 64u) & 31u);
        }
    }
    // Root value over the compacted program, 32-deep bit stack, branch-free per
    // node: value = bit idx of the code's truth table, idx = 2A+B for binops (A
    // second, B top of stack) or the primitive's membership bit; binops pop two.
    //   PRIM 0b0010, UNION 0b1110, INTER 0b1000, DIFF 0b0100, RDIFF 0b0010, CONST0 0.
    static constexpr uint32_t kTruth =
        (0x2u << 4) | (0xEu << 8) | (0x8u << 12) | (0x4u << 16) | (0x2u << 20) | (0x0u << 24);
    __device__ __forceinline__ uint32_t eval_root() const {
        uint32_t st = 0, ord = 0;
        const uint32_t n = ncodes;
        for (uint32_t base = 0; base < n; base += 8u) {
            uint32_t word = uni(codes[base >> 3]);
            uint32_t m = n - base < 8u ? n - base : 8u;
            for (uint32_t j = 0; j < m; ++j) {
                uint32_t c = (word >> (4u * j)) & 15u;
                uint32_t tt = (kTruth >> (4u * c)) & 15u;
                bool isprim = c == kCodePrim;
                uint32_t pop = (c >= kCodeUnion && c < kCodeConst0) ? 2u : 0u;
                uint32_t idx = st & 3u;
                if (isprim) idx = bit(ord);
                uint32_t val = (tt >> idx) & 1u;
                st = ((st >> pop) << 1) | val;
                ord += isprim ? 1u : 0u;
            }
        }
        return st & 1u;
    }

    __device__ __forceinline__ WoRec hit_leaf(const Hit& h) const { return prog[ordpc[h.ord()] + 1u + h.member()]; }

    // Nearest change of the root's membership after WO_T_MIN along o + t d.
    __device__ __forceinline__ bool trace(F3 o, F3 d, Hit& hit) {
        const float tmin = WO_T_MIN;
        Window win;
        win.clear();
        bits = 0;
        ncodes = 0;
        nprims = 0;
        uint32_t code_acc = 0;
        uint32_t hib_acc = 0;
        uint32_t st = 0;  // bit stack: the root value at t_min, evaluated on the way
        F3 inv = f3(0.0f, 0.0f, 0.0f);
        bool have_inv = false;

        // pass 1: walk the program, cull, intersect, collect events
        uint32_t pc = 0;
        while (pc < nrec) {
            WoRec rec = prog[pc];
            uint32_t op = uni(rec.op);
            uint32_t code;
            if (op == WO_OP_BOUND) {
                WO_WK(WO_WORK_BOUND_TESTS);
                bool may = bound_may_hit(rec.f[0], rec.f[1], rec.f[2], rec.f[3], rec.f[4], o, d);
                if (__ballot(may) != 0ull) {
                    ++pc;
                    continue;
                }
                code = kCodeConst0;
                st = st << 1;
                pc = uni(rec.u0);
            } else if (op == WO_OP_PRIM) {
                uint32_t count = uni(rec.u0);
                uint32_t ord = nprims;
                Ivl iv = prim_interval<kCount>(prog, pc, count, o, d, inv, have_inv, wk);
                uint32_t inside = 0;
                if (!(iv.a > iv.b)) {
                    inside = (iv.a <= tmin && iv.b > tmin) ? 1u : 0u;
                    if (iv.a > tmin) {
                        WO_WK(WO_WORK_EVENTS);
                        win.insert(event_key(iv.a, ord, 0u, iv.ma));
                    }
                    if (iv.b > tmin && iv.b < kInf) {
                        WO_WK(WO_WORK_EVENTS);
                        win.insert(event_key(iv.b, ord, 1u, iv.mb));
                    }
                }
                if (ord < 64u) {
                    bits |= (uint64_t)inside << ord;
                } else {
                    uint32_t sh = (ord - 64u) & 31u;
                    hib_acc |= inside << sh;
                    if (sh == 31u) {
                        hib[((ord - 64u) >> 5) * 64u + lane] = hib_acc;
                        hib_acc = 0;
                    }
                }
                ordpc[ord] = pc;
                nprims = ord + 1u;
                code = kCodePrim;
                st = (st << 1) | inside;
                pc += 1u + count;
            } else {
                code = op;  // WO_OP_UNION..RDIFF share values with the codes
                uint32_t tt = (kTruth >> (4u * code)) & 15u;
                st = ((st >> 2) << 1) | ((tt >> (st & 3u)) & 1u);
                ++pc;
            }
            uint32_t slot = ncodes & 7u;
            code_acc |= code << (4u * slot);
            if (slot == 7u) {
                codes[ncodes >> 3] = code_acc;
                code_acc = 0;
            }
            ++ncodes;
        }
        if (ncodes & 7u) codes[ncodes >> 3] = code_acc;
        if (nprims > 64u && ((nprims - 64u) & 31u)) hib[((nprims - 64u) >> 5) * 64u + lane] = hib_acc;

        // pass 2: sweep events in key order; the first root flip is the hit
        if (win.empty()) return false;
        uint32_t root = st & 1u;
        while (!win.empty()) {
            uint64_t key = win.pop();
            WO_WK(WO_WORK_SWEEP_STEPS);
            uint32_t ord = key_ord(key);
            toggle(ord);
            uint32_t r = eval_root();
            if (r != root) {
                hit_from_key(key, r, hit);
                return true;
            }
            root = r;
            if (win.empty() && win.dropped()) {
                // window exhausted but events were dropped: re-collect the events
                // strictly after `key` (the membership state carries on)
                WO_WK(WO_WORK_RECOLLECTS);
                win.clear();
                uint32_t ordc = 0;
                uint32_t nwords = (ncodes + 7u) >> 3;
                for (uint32_t w = 0; w < nwords; ++w) {
                    uint32_t word = uni(codes[w]);
                    uint32_t n = ncodes - w * 8u;
                    n = n < 8u ? n : 8u;
                    for (uint32_t j = 0; j < n; ++j) {
                        if (((word >> (4u * j)) & 15u) != kCodePrim) continue;
                        uint32_t ppc = uni(ordpc[ordc]);
                        uint32_t count = uni(prog[ppc].u0);
                        Ivl iv = prim_interval<kCount>(prog, ppc, count, o, d, inv, have_inv, wk);
                        if (!(iv.a > iv.b)) {
                            if (iv.a > tmin) {
                                uint64_t k2 = event_key(iv.a, ordc, 0u, iv.ma);
                                if (k2 > key) {
                                    WO_WK(WO_WORK_EVENTS);
                                    win.insert(k2);
                                }
                            }
                            if (iv.b > tmin && iv.b < kInf) {
                                uint64_t k2 = event_key(iv.b, ordc, 1u, iv.mb);
                                if (k2 > key) {
                                    WO_WK(WO_WORK_EVENTS);
                                    win.insert(k2);
                                }
                            }
                        }
                        ++ordc;
                    }
                }
            }
        }
        return false;
    }
};

// ---------------------------------------------------------------------------
// Lane traversal, for programs whose every binop is a UNION (scenes like the
// RTIOW cover: hundreds of primitives, no CSG).  Each lane walks the BOUND
// hierarchy on its own (stackless: a missed BOUND jumps to its skip target),
// so a wave costs the LONGEST lane's walk instead of the UNION of its lanes'
// walks -- the difference that matters for incoherent bounce rays.  The trav
// table is the program with the binop records dropped (host: build_trav).
//
// Union semantics need no tree evaluation: the root is inside iff the count
// of primitives containing the point is > 0; an entry event adds one, an exit
// removes one.  A BOUND whose near end (tca - R, with slack) lies beyond the
// nearest event collected so far is pruned; the sweep treats the smallest
// pruned near end as a barrier (`kcut`): reaching it re-collects after the
// last processed event, exactly as an overflowing window does.  Results are
// the general algorithm's, bit for bit.
// ---------------------------------------------------------------------------

// Ordered BVH traversal (the common case).  The host builds a binary AABB
// hierarchy over the bounded primitives (build_lbvh; each node holds its two
// children's boxes, expanded outward), and an `always` list of the unbounded
// and outsized ones.  A lane walks it nearest child first with a short LDS
// stack and prunes every box whose near end lies beyond the nearest entry event
// found so far.  While the ray starts outside every primitive (none contains
// the point at t_min), the first event in key order is an entry -- an exit
// before any entry would need a primitive containing t_min -- and the root
// (a union) flips there: the hit is the smallest entry key, which does not
// depend on the visiting order, so the result is the general algorithm's bit for
// bit.  A ray that starts inside some primitive (counted on the way: boxes that
// contain the ray's start are never pruned) takes the general walk below.
constexpr uint32_t kLeafRef = 0x80000000u, kNoRef = 0xffffffffu;
// 16-bit refs (lane stacks, 4-wide nodes): node index or ordinal in bits 0-14, leaf flag in bit 15
constexpr uint32_t kNoRef16 = 0xffffu;
// term mode (extract_terms): literals per term; a literal is ordinal | kLitNeg (complement)
constexpr uint32_t kTermLits = 2, kLitNeg = 0x80000000u, kNoLit = 0xffffffffu;
// term records (build_lbvh): float4 [0] = literal 0, literal 1, kinds (2 bits per
// literal), 0; [1 + 2x], [2 + 2x] = literal x's sphere members (centre, r^2)
constexpr uint32_t kTermRecF4 = 5, kTermLitSphere = 1, kTermLitSphere2 = 2;  // kind 0: generic (prim_ivl)
// The lane BVH is built with at most kLaneDepthMax internal levels on any path,
// and the per-lane LDS stack holds as many entries as the built tree has levels:
// a walk pushes at most one sibling per ancestor, so the stack never overflows.
constexpr uint32_t kLaneDepthMax = 24;
#ifndef WO_LANES_TERM2
#define WO_LANES_TERM2 1  // term visits of two spheres in all: two sphere tests (visit_leaf)
#endif
#ifndef WO_LANES_PRIO
#define WO_LANES_PRIO 1  // wave priority while a walk trip issues its node load (0: unchanged; RTIOW 11.67 -> 11.58 ms)
#endif
#ifndef WO_LANES_PRIO_LEAF
#define WO_LANES_PRIO_LEAF 1  // the same at a sphere leaf's geometry load (single-sphere walks; RTIOW 11.565 -> 11.505 ms)
#endif
#ifndef WO_LANES_PRIO_TERM
#define WO_LANES_PRIO_TERM 1  // the same at a term record's load (term mode; csg512 43.44 / 43.39 -> 43.37 / 43.28 ms, parity suite green with it)
#endif
#ifndef WO_LANES_FUSED_SPHERE
#define WO_LANES_FUSED_SPHERE 1
#endif
// dynamic LDS of the BVH walk (stacks + top nodes): with the kernel's static LDS,
// 8 workgroups of kBlock fit in a CU's 160 KB
#ifndef WO_LANES_CAM
#define WO_LANES_CAM 0  // the lane kernels' camera-wave mode (pathtrace_block kCam)
#endif
// the camera ring's LDS per workgroup (64 slots of 48 B per wave)
constexpr size_t kCamRingLds = WO_LANES_CAM ? 4u * 64u * 48u : 0u;
// 8 workgroups per CU = 20 KB each, less the kernels' static LDS (2224 B since the
// pixel-row table, round 5; at 18 KB of dynamic LDS the total crossed 20 KB and the
// RTIOW cover ran at 7 workgroups per CU: 11.24 -> 11.69 ms)
constexpr size_t kLanesStaticLdsMax = 2304u;
constexpr size_t kLanesBvhLds = 20u * 1024u - kLanesStaticLdsMax;

// component c (a compile-time constant after unrolling) of a float4
__device__ __forceinline__ float f4c(const float4& v, int c) { return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w)); }

// Slab test of a ray against an expanded AABB: [near, far] of the ray's overlap
// (conservative: the boxes carry the slack; `ri` = reciprocal direction with
// zero components replaced by +-1e30, `oi` = o * ri).
__device__ __forceinline__ float box_near(float4 lo, float4 hi, F3 ri, F3 oi, float& far_t) {
    const float ax = __builtin_fmaf(lo.x, ri.x, -oi.x), bx = __builtin_fmaf(hi.x, ri.x, -oi.x);
    const float ay = __builtin_fmaf(lo.y, ri.y, -oi.y), by = __builtin_fmaf(hi.y, ri.y, -oi.y);
    const float az = __builtin_fmaf(lo.z, ri.z, -oi.z), bz = __builtin_fmaf(hi.z, ri.z, -oi.z);
    const float n = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    far_t = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    return n;
}

// The same over a child box stored as fp16 (lb_half: lo rounded down, hi up, so
// the box only grows): q.x = lo.x | lo.y << 16, q.y = lo.z | hi.x << 16, q.z =
// hi.y | hi.z << 16.  The conversions fold into v_fma_mix_f32.
// kMode (PathKind): 2 ordered BVH over union-only primitives, 3 the same over
// single-sphere primitives only (no generic-primitive code: fewer registers),
// 6 ordered BVH over the terms of a root that is a union of small conjunctions
// (extract_terms: the leaves and the always list hold terms), 7 ordered BVH over
// the primitives of a general tree (the events in key order, kGWin per walk, and
// the tree's value kept per lane and updated along the toggled leaf's path), 14 term mode over a
// 4-wide tree (lb_collapse4: four child boxes per node, half the dependent node
// loads of a walk; 16-bit stacks) with the resumable walk (trace_step, dynamic
// ray fetch).  Measured and removed: the general BOUND walk,
// 16-bit stacks for binary trees, 4-wide trees for primitives, resumable binary
// walks, a uniform grid and fp16 child boxes.
// events a general-tree walk collects (the smallest after `after`, sorted; with
// inserts beyond a full window's last filtered out -- csg360_nested 1029 ms at 4,
// 645 at 8, 503 at 16, 453 at 24, 440 at 32; 48 and 64 spill)
#ifndef WO_LANES_GWIN
#define WO_LANES_GWIN 32
#endif
constexpr int kGWin = WO_LANES_GWIN;
// a walk trip's node steps, then the leaf they reached, in one trip (LaneTracer::trip;
// the same steps per lane in the same order); 0 leaf phases: a trip is a node or a leaf
#ifndef WO_LANES_TRIP_NODES
#define WO_LANES_TRIP_NODES 2
#endif
#ifndef WO_LANES_TRIP_LEAVES
#define WO_LANES_TRIP_LEAVES 1
#endif
// a general tree's node record (build_lbvh): left ref | right ref << 15 | op << 30
constexpr uint32_t kGRefBits = 15u, kGRefMask = (1u << kGRefBits) - 1u;
template <int kModeT, bool kCountT>
struct LaneTracer {
    static_assert(kModeT == 2 || kModeT == 3 || kModeT == 6 || kModeT == 7 || kModeT == 14, "lane tracer forms");
    static constexpr bool kCount = kCountT;
    static constexpr bool kDyn = kModeT == 14;
    static constexpr bool kResumable = kDyn;
    static constexpr int kMode = kModeT;
    static constexpr bool kWide = kMode == 14;
    static constexpr bool kSpheresOnly = kMode == 3;
    static constexpr bool kStack16 = kWide || kMode == 7;
    static constexpr bool kTerms = kMode == 6 || kMode == 14;
    static constexpr bool kGeneral = kMode == 7;
    static constexpr uint32_t kNodeF4 = kWide ? 7u : 4u;  // float4 per node
    // camera-ray waves (pathtrace_block): not for the resumable walk, nor for the general
    // tree (its bits fill the LDS)
    static constexpr int kCamMode = (kDyn || kGeneral) ? 0 : WO_LANES_CAM;
    static constexpr bool kFreshTail = kDyn || kGeneral;  // (TracerFreshTail)
    WorkCounts wk;
    uint64_t tmark;  // section timing (counting builds)
    const WoRec* __restrict__ prog;      // full program (generic primitives, hit leaves)
    const uint32_t* __restrict__ ordpc;  // ordinal -> program pc
    // ordered BVH (build_lbvh)
    const float4* __restrict__ lnodes;   // 4 float4 per node: childA lo|ref, childA hi|ref B, childB lo, childB hi
    const float4* __restrict__ lgeo;     // per ordinal: sphere centre, r^2 (single-sphere primitives)
    const uint32_t* __restrict__ lkind;  // per ordinal: 1 = single sphere, 0 = generic; then the always list
    // term mode: per term 5 float4 -- the two literals (ordinal | kLitNeg, or kNoLit)
    // and their inline kinds, then per literal up to two sphere members (kTermRec*)
    const float4* __restrict__ ltrec;
    uint32_t nalways, lroot, nprims;
    uint32_t* stk;                       // LDS stack column of this lane ([entry][lane])
    uint16_t* stk16;                     // the same with 16-bit entries (kStack16): leaf bit 15
    // LDS copy of nodes [0, ntop) (the top levels, BFS order).  Typed by address
    // space so the two node reads of query() stay an LDS and a global load: one
    // pointer to either would be a flat load, which waits on both counters.
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(3))) float4* LdsNodes;
    typedef const __attribute__((address_space(1))) float4* GlobalNodes;
#else
    typedef const float4* LdsNodes;
    typedef const float4* GlobalNodes;
#endif
    LdsNodes ltop;
    uint32_t ntop;
    // general tree (kGeneral): the tree's refs are its leaves (primitive ordinals,
    // [0, gP)) and internal nodes ([gP, ...)); per lane one bit per ref, the value of
    // that leaf / node at the current key (a column of gwords words in LDS, [w][lane])
    uint32_t* gbits;
    const uint32_t* __restrict__ gpar;   // per ref: its parent's ref, or kNoRef (the root)
    const uint32_t* __restrict__ gnode;  // per internal node: left | right << 15 | op << 30
    uint32_t gP, gwords, groot;
    uint64_t gw[kGWin];  // the walk's smallest event keys after `after`, ascending
    const float4* __restrict__ gclip;  // per primitive: relevance box (LaneBvh::gclip)
    F3 gri, goi;                       // the ray's reciprocal direction and o * ri (trace_general)

    // single-sphere scenes: per ordinal its leaf record, then its material (LaneBvh::leaves)
    const WoRec* __restrict__ lleaf;
    static constexpr bool kHitMaterial = kSpheresOnly;
    __device__ __forceinline__ WoRec hit_leaf(const Hit& h) const {
        if constexpr (kSpheresOnly)
            return lleaf[2u * h.ord()];  // one load (the record of the ordinal's only member)
        else
            return prog[ordpc[h.ord()] + 1u + h.member()];
    }
    // the leaf's material, copied next to its record: loaded beside it, not after it
    __device__ __forceinline__ WoMaterial hit_material(const Hit& h, const WoMaterial* __restrict__) const {
        return reinterpret_cast<const WoMaterial*>(lleaf)[2u * h.ord() + 1u];
    }

    // Interval of primitive `ord` (the interpreter's arithmetic, bit for bit).
    __device__ __forceinline__ Ivl prim_ivl(uint32_t ord, F3 o, F3 d, F3& inv, bool& have_inv) {
        Ivl iv;
        if (kSpheresOnly || lkind[ord] != 0u) {
            WO_WK(WO_WORK_SPHERE_TESTS);
            const float4 g = lgeo[ord];
            float b, ll, la, lb;
            sphere_bl(g.x, g.y, g.z, o, d, b, ll);
            sphere_interval_bl(b, ll, g.w, la, lb);
            ivl_first(iv, la, lb);
        } else {
            const uint32_t ppc = ordpc[ord];
            const uint32_t count = prog[ppc].u0;
            for (uint32_t m = 0; m < count; ++m) {
                WoRec L = prog[ppc + 1u + m];
                float la, lb;
                WO_WK(L.op == WO_LEAF_SPHERE ? WO_WORK_SPHERE_TESTS : WO_WORK_HALFSPACE_TESTS);
                if (L.op == WO_LEAF_SPHERE) {
                    sphere_interval(L.f[0], L.f[1], L.f[2], L.f[3], o, d, la, lb);
                } else if (L.u1 != 0u) {
                    if (!have_inv) {
                        inv = f3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
                        have_inv = true;
                    }
                    uint32_t ax = L.u1 - 1u;
                    halfspace_axis_interval(ax == 0u ? L.f[0] : (ax == 1u ? L.f[1] : L.f[2]), L.f[3], pick3(o, ax),
                                            pick3(d, ax), pick3(inv, ax), la, lb);
                } else {
                    halfspace_interval(L.f[0], L.f[1], L.f[2], L.f[3], o, d, la, lb);
                }
                if (m == 0u)
                    ivl_first(iv, la, lb);
                else
                    ivl_meet(iv, la, lb, m);
            }
        }
        return iv;
    }

    // One query's walk state (query / trace_step): the smallest event key > `after`
    // found so far, whether the count rises there (term mode), the node to visit
    // next and the lane stack's depth, the primitives (terms) holding t_min met so
    // far, and the re-query's lower box bound.
    struct QState {
        uint64_t best, after;
        uint32_t cur, sp, cnt;
        float tlo;
        bool up;
    };

    // A leaf of the walk (or of the always list): a primitive, or in
    // term mode a term.  Term mode: a term (a conjunction of one or two literals,
    // each a primitive or its complement) changes value only at an event of a
    // literal X, and then exactly when the other literal holds at that key; it
    // rises where X's literal becomes true (X's entry for a positive literal, its
    // exit for a complement).  A primitive is in one term, so one key changes one term.
    __device__ __forceinline__ void visit_leaf(uint32_t ref, uint32_t& cnt, QState& s, F3 o, F3 d, F3& inv,
                                               bool& have_inv) {
        const float tmin = WO_T_MIN;
        uint64_t& best = s.best;
        const uint64_t after = s.after;
        if constexpr (kTerms) {
            // the record's header and both literals' inline spheres: independent loads
            const float4* rec = ltrec + kTermRecF4 * ref;
#if WO_LANES_PRIO_TERM
            __builtin_amdgcn_s_setprio(WO_LANES_PRIO_TERM);
#endif
            const float4 hd = rec[0];
#if WO_LANES_PRIO_TERM
            __builtin_amdgcn_s_setprio(0);
#endif
            const uint2 tl = make_uint2(__float_as_uint(hd.x), __float_as_uint(hd.y));
            const uint32_t kinds = __float_as_uint(hd.z);
            uint64_t kin[2], kout[2];
            bool valid[2], pos[2];
            const bool one = tl.y == kNoLit;
            auto lit_keys = [&](int x, const Ivl& iv) {
                const uint32_t lit = x == 0 ? tl.x : tl.y;
                const uint32_t ord = lit & ~kLitNeg;
                pos[x] = !(lit & kLitNeg);
                valid[x] = !(iv.a > iv.b) & (iv.b > tmin) & !(x == 1 && one);
                kin[x] = iv.a > tmin ? event_key(iv.a, ord, 0u, iv.ma) : 0ull;
                kout[x] = iv.b < kInf ? event_key(iv.b, ord, 1u, iv.mb) : kEmptyKey;
            };
            // Two spheres in all (WO_LANES_TERM2): one literal of one or two sphere
            // members, or two literals of one sphere each (csg512's unions, differences
            // and intersections of pairs) -- two sphere tests instead of the four of the
            // record's general form, the same intervals and members (a single sphere's
            // repeated member is a no-op meet), when every lane of the wave has such a term
            const uint32_t k0 = kinds & 3u, k1 = (kinds >> 2) & 3u;
            const bool two = (k0 != 0u) & (one | ((k0 == kTermLitSphere) & (k1 == kTermLitSphere)));
            if (WO_LANES_TERM2 && __ballot(!two) == 0ull) {
                const bool two0 = k0 == kTermLitSphere2;  // literal 0's second member is the second sphere
                WO_WK_N(WO_WORK_SPHERE_TESTS, (two0 | !one) ? 2u : 1u);
                const float4 g0 = rec[1], g1 = rec[two0 ? 2 : 3];
                float la0, lb0, la1 = kInf, lb1 = -kInf;
                sphere_interval(g0.x, g0.y, g0.z, g0.w, o, d, la0, lb0);
                if (__ballot(two0 | !one) != 0ull) {
                    asm volatile("");
                    sphere_interval(g1.x, g1.y, g1.z, g1.w, o, d, la1, lb1);
                }
                Ivl i0, m0, i1;
                ivl_first(i0, la0, lb0);
                m0 = i0;
                ivl_meet(m0, la1, lb1, 1u);
                ivl_first(i1, la1, lb1);
                lit_keys(0, two0 ? m0 : i0);
                lit_keys(1, i1);
            } else {
#pragma unroll
                for (int x = 0; x < 2; ++x) {
                    const uint32_t lit = x == 0 ? tl.x : tl.y;
                    const uint32_t ord = lit & ~kLitNeg;
                    // an inline literal (one or two sphere members; a single sphere repeats
                    // itself as member 1, which leaves the interval and its members as
                    // they are, and a missing second literal is a dummy sphere masked out
                    // below) is branch-free: lanes at different terms stay converged
                    Ivl iv;
                    if ((kinds >> (2 * x)) & 3u) {
                        WO_WK_N(WO_WORK_SPHERE_TESTS, ((kinds >> (2 * x)) & 3u) == kTermLitSphere ? 1u : 2u);
                        const float4 g0 = rec[1 + 2 * x], g1 = rec[2 + 2 * x];
                        float la, lb;
                        sphere_interval(g0.x, g0.y, g0.z, g0.w, o, d, la, lb);
                        ivl_first(iv, la, lb);
                        sphere_interval(g1.x, g1.y, g1.z, g1.w, o, d, la, lb);
                        ivl_meet(iv, la, lb, 1u);
                    } else {
                        iv = prim_ivl(ord, o, d, inv, have_inv);
                    }
                    lit_keys(x, iv);
                }
            }
            // the literal's value just around key e of the other literal (keys are distinct)
            auto lit_at = [&](int x, uint64_t e) {
                const bool in = valid[x] & (kin[x] < e) & (e < kout[x]);
                return pos[x] ? in : !in;
            };
            const bool t0 = (pos[0] ? (valid[0] & (kin[0] == 0ull)) : !(valid[0] & (kin[0] == 0ull))) &
                            (one | (pos[1] ? (valid[1] & (kin[1] == 0ull)) : !(valid[1] & (kin[1] == 0ull))));
            if (t0) ++cnt;
#pragma unroll
            for (int x = 0; x < 2; ++x) {
                const int y = 1 - x;
                const bool has = valid[x] & !(x == 1 && one);
                const uint64_t ei = kin[x], eo = kout[x];
                // selects, not branches (lanes at different terms stay converged)
                const bool ti = has & (ei != 0ull) & (ei > after) & (ei < best) & (one | lit_at(y, ei));
                WO_WK_N(WO_WORK_EVENTS, ti ? 1u : 0u);
                best = ti ? ei : best;
                s.up = ti ? pos[x] : s.up;
                const bool to = has & (eo != kEmptyKey) & (eo > after) & (eo < best) & (one | lit_at(y, eo));
                WO_WK_N(WO_WORK_EVENTS, to ? 1u : 0u);
                best = to ? eo : best;
                s.up = to ? !pos[x] : s.up;
            }
            return;
        }
        const uint32_t ord = ref;
#if WO_LANES_FUSED_SPHERE
        if constexpr (kSpheresOnly && !kGeneral) {
            // a sphere's interval [-b - s, -b + s] exists exactly when disc >= 0: the
            // count and the events inside the sqrt branch, no empty interval formed
            // (the specialised kernel's lone spheres; same bits as prim_ivl's form)
            WO_WK(WO_WORK_SPHERE_TESTS);
#if WO_LANES_PRIO_LEAF
            __builtin_amdgcn_s_setprio(WO_LANES_PRIO_LEAF);
#endif
            const float4 g = lgeo[ord];
#if WO_LANES_PRIO_LEAF
            __builtin_amdgcn_s_setprio(0);
#endif
            float b, ll;
            sphere_bl(g.x, g.y, g.z, o, d, b, ll);
            const float disc = g.w - ll;
            if (__ballot(sphere_need(b, disc)) != 0ull) {
                asm volatile("");
                if (!(disc < 0.0f)) {
                    const float s = sqrt_pt(disc), nb = -b, la = nb - s, lb = nb + s;
                    if ((la <= tmin) & (lb > tmin)) ++cnt;
                    const uint64_t k0 = event_key(la, ord, 0u, 0u), k1 = event_key(lb, ord, 1u, 0u);
                    if ((la > tmin) & (k0 > after)) {
                        WO_WK(WO_WORK_EVENTS);
                        best = k0 < best ? k0 : best;
                    }
                    if ((lb > tmin) & (lb < kInf) & (k1 > after)) {
                        WO_WK(WO_WORK_EVENTS);
                        best = k1 < best ? k1 : best;
                    }
                }
            }
            return;
        }
#endif
        Ivl iv = prim_ivl(ord, o, d, inv, have_inv);
        if constexpr (kGeneral) {
            // The primitive restricted to its relevance box (build_lbvh): outside it the
            // primitive cannot change the root (an intersection's other operand, or a
            // difference's left one, is empty there), so its interval is clipped to the
            // box's span, widened by a margin past the slab test's rounding.  An end
            // the clip moves is an event of the clipped primitive that never flips the
            // root, so the hit -- the first key where the root flips -- is unchanged.
            if (gclip != nullptr) {
                const float4 cl = gclip[2u * ord];
                if (__float_as_uint(cl.w) != 0u) {
                    float c1;
                    const float c0 = box_near(cl, gclip[2u * ord + 1u], gri, goi, c1);
                    const float m0 = __builtin_fmaf(-2e-5f, fabsf(c0), c0) - 1e-5f;
                    const float m1 = __builtin_fmaf(2e-5f, fabsf(c1), c1) + 1e-5f;
                    iv.a = fmaxf(iv.a, m0);
                    iv.b = fminf(iv.b, m1);
                }
            }
            if (!(iv.a > iv.b)) {
                // the first query sets the leaves that hold t_min (the tree's value at
                // t_min); every query keeps its kGWin smallest keys after `after`, and
                // prunes with the largest once it has them all
                if ((after == 0ull) & (iv.a <= tmin) & (iv.b > tmin)) gtoggle(ord);
                const uint64_t k0 = event_key(iv.a, ord, 0u, iv.ma), k1 = event_key(iv.b, ord, 1u, iv.mb);
                // a key at or beyond a full window's last cannot enter it
                if ((iv.a > tmin) & (k0 > after) & (k0 < gw[kGWin - 1])) {
                    WO_WK(WO_WORK_EVENTS);
                    ginsert(k0);
                }
                if ((iv.b > tmin) & (iv.b < kInf) & (k1 > after) & (k1 < gw[kGWin - 1])) {
                    WO_WK(WO_WORK_EVENTS);
                    ginsert(k1);
                }
                best = gw[kGWin - 1];
            }
            return;
        }
        if (!(iv.a > iv.b)) {
            if ((iv.a <= tmin) & (iv.b > tmin)) ++cnt;
            const uint64_t k0 = event_key(iv.a, ord, 0u, iv.ma), k1 = event_key(iv.b, ord, 1u, iv.mb);
            if ((iv.a > tmin) & (k0 > after)) {
                WO_WK(WO_WORK_EVENTS);
                best = k0 < best ? k0 : best;
            }
            if ((iv.b > tmin) & (iv.b < kInf) & (k1 > after)) {
                WO_WK(WO_WORK_EVENTS);
                best = k1 < best ? k1 : best;
            }
        }
    }

    // A query's start: the always list, then the walk from the root.  A re-query
    // (after != 0) prunes boxes that end before the last key: their events all lie
    // at or before it (the boxes' slack covers the slab test's rounding; the
    // margin below covers the key's own t).  The first query keeps every box that
    // holds the ray's start (the count at t_min).
    __device__ __forceinline__ void qbegin(QState& s, uint64_t after, F3 o, F3 d, F3& inv, bool& have_inv) {
        s.best = kEmptyKey;
        s.after = after;
        s.up = false;
        s.cnt = 0;
        for (uint32_t i = 0; i < nalways; ++i) visit_leaf(lkind[nprims + i], s.cnt, s, o, d, inv, have_inv);
        const float tafter = after == 0ull ? 0.0f : __uint_as_float((uint32_t)(after >> 32));
        s.tlo = fmaxf(__builtin_fmaf(-2e-5f, tafter, tafter) - 1e-6f, 0.0f);
        s.cur = lroot;
        s.sp = 0;
    }

    // One trip of the walk: a leaf, or a node (its children's boxes, nearest hit
    // child next, the other(s) pushed); then a pop when the walk has no next node.
    // WO_LANES_TRIP_NODES node steps and then WO_LANES_TRIP_LEAVES leaves in one trip:
    // a lane walks node -> node -> leaf in one trip instead of three, so the wave's
    // lanes, at different depths, still share most trips' node and leaf code.
    __device__ __forceinline__ void trip(QState& s, F3 o, F3 d, F3 ri, F3 oi, F3& inv, bool& have_inv) {
        WO_WK_WAVE(WO_WORK_SWEEP_TRIPS);  // lane tracer: walk trips per wave
        uint32_t cur = s.cur, sp = s.sp;
        const float tlo = s.tlo;
        auto pop = [&]() {
            if ((cur == kNoRef) & (sp != 0u)) {
                --sp;
                if constexpr (kStack16) {
                    const uint32_t e = stk16[sp * kBlock];
                    cur = (e & 0x7fffu) | ((e & 0x8000u) << 16);
                } else {
                    cur = stk[sp * kBlock];
                }
            }
        };
        // a leaf (not the walk's end) visited, then the next entry popped
        auto leaf_phase = [&]() {
            if (((cur & kLeafRef) != 0u) & (cur != kNoRef)) {
                visit_leaf(cur & ~kLeafRef, s.cnt, s, o, d, inv, have_inv);
                cur = kNoRef;
                pop();
            }
        };
        // the node step (the non-fused walk: or the leaf), then a pop when it ends a path
        auto node_phase = [&]() {
            const bool at_leaf = (cur & kLeafRef) != 0u;  // (the walk's end, kNoRef, included)
            if (!WO_LANES_TRIP_LEAVES && at_leaf) {
                visit_leaf(cur & ~kLeafRef, s.cnt, s, o, d, inv, have_inv);
                cur = kNoRef;
            } else if (kWide && !at_leaf) {
                // four children: lo.x, hi.x, lo.y, hi.y, lo.z, hi.z of each, then the refs
                WO_WK_N(WO_WORK_BOUND_TESTS, 4u);
                float4 q[7];
#if WO_LANES_PRIO
                __builtin_amdgcn_s_setprio(WO_LANES_PRIO);
#endif
                if (cur < ntop) {
                    const LdsNodes nd = ltop + 7u * cur;
#pragma unroll
                    for (int k = 0; k < 7; ++k) q[k] = nd[k];
                    asm volatile("");
                } else {
                    const GlobalNodes nd = (GlobalNodes)lnodes + 7u * cur;
#pragma unroll
                    for (int k = 0; k < 7; ++k) q[k] = nd[k];
                }
#if WO_LANES_PRIO
                __builtin_amdgcn_s_setprio(0);
#endif
                const float tb = s.best == kEmptyKey ? kInf : __uint_as_float((uint32_t)(s.best >> 32));
                // per child a sort key: the top 16 bits of max(near, 0) (monotone as an
                // unsigned integer; the order only steers the walk) | the child's 16-bit
                // ref; ~0 for a miss or an empty slot
                uint32_t kk[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float ax = __builtin_fmaf(f4c(q[0], c), ri.x, -oi.x), bx = __builtin_fmaf(f4c(q[1], c), ri.x, -oi.x);
                    const float ay = __builtin_fmaf(f4c(q[2], c), ri.y, -oi.y), by = __builtin_fmaf(f4c(q[3], c), ri.y, -oi.y);
                    const float az = __builtin_fmaf(f4c(q[4], c), ri.z, -oi.z), bz = __builtin_fmaf(f4c(q[5], c), ri.z, -oi.z);
                    const float n = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
                    const float f = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
                    const uint32_t r16 = __float_as_uint(f4c(q[6], c));
                    const float n0 = fmaxf(n, 0.0f);
                    const bool h = (f >= fmaxf(n0, tlo)) & (n <= tb) & (r16 != kNoRef16);
                    kk[c] = h ? ((__float_as_uint(n0) & 0xffff0000u) | r16) : 0xffffffffu;
                }
                // nearest first: a 4-key sorting network (misses sort last)
                auto ce = [&](int i, int j) {
                    const uint32_t lo = kk[i] < kk[j] ? kk[i] : kk[j], hi = kk[i] < kk[j] ? kk[j] : kk[i];
                    kk[i] = lo;
                    kk[j] = hi;
                };
                ce(0, 1);
                ce(2, 3);
                ce(0, 2);
                ce(1, 3);
                ce(1, 2);
                cur = kk[0] == 0xffffffffu ? kNoRef : (kk[0] & 0x7fffu) | ((kk[0] & 0x8000u) << 16);
                // the farther ones on the stack, farthest deepest (sp < 3 x the tree's levels)
#pragma unroll
                for (int c = 3; c >= 1; --c) {
                    if (kk[c] != 0xffffffffu) {
                        stk16[sp * kBlock] = (uint16_t)kk[c];
                        ++sp;
                    }
                }
            } else if (!kWide && !at_leaf) {
                WO_WK_N(WO_WORK_BOUND_TESTS, 2u);
                float na, nb, fa, fb;
                uint32_t ra, rb;
                {
                    float4 a0, a1, b0, b1;
#if WO_LANES_PRIO
                    __builtin_amdgcn_s_setprio(WO_LANES_PRIO);  // a wave about to issue its node load goes first
#endif
                    if (cur < ntop) {  // the top levels: LDS latency instead of a cache round trip
                        const LdsNodes nd = ltop + 4u * cur;
                        a0 = nd[0], a1 = nd[1], b0 = nd[2], b1 = nd[3];
                        asm volatile("");  // the branches' tails differ: the loads are not merged into flat loads
                    } else {
                        const GlobalNodes nd = (GlobalNodes)lnodes + 4u * cur;
                        a0 = nd[0], a1 = nd[1], b0 = nd[2], b1 = nd[3];
                    }
#if WO_LANES_PRIO
                    __builtin_amdgcn_s_setprio(0);
#endif
                    na = box_near(a0, a1, ri, oi, fa);
                    nb = box_near(b0, b1, ri, oi, fb);
                    ra = __float_as_uint(a0.w);
                    rb = __float_as_uint(a1.w);
                }
                // useful range: up to the best event so far
                const float tb = s.best == kEmptyKey ? kInf : __uint_as_float((uint32_t)(s.best >> 32));
                const bool ha = (fa >= fmaxf(na, tlo)) & (na <= tb);
                const bool hb = (fb >= fmaxf(nb, tlo)) & (nb <= tb);
                if (ha & hb) {
                    const bool a_first = na <= nb;
                    cur = a_first ? ra : rb;
                    const uint32_t other = a_first ? rb : ra;
                    if constexpr (kStack16)  // refs < 2^15 (build_lbvh): the leaf flag moves to bit 15
                        stk16[sp * kBlock] = (uint16_t)((other & 0x7fffu) | ((other >> 16) & 0x8000u));
                    else
                        stk[sp * kBlock] = other;  // sp < the tree's depth (build_lbvh)
                    ++sp;
                } else {
                    cur = ha ? ra : (hb ? rb : kNoRef);
                }
            }
            pop();
        };
        // (a lane at a leaf or at the walk's end skips a node step)
#pragma unroll
        for (int k = 0; k < WO_LANES_TRIP_NODES; ++k) node_phase();
#pragma unroll
        for (int k = 0; k < WO_LANES_TRIP_LEAVES; ++k) leaf_phase();
        s.cur = cur;
        s.sp = sp;
    }

    // The smallest event key > `after` (entries and exits after t_min), or
    // kEmptyKey; `inside` (first query only) counts the primitives whose
    // interval holds t_min.  Boxes are pruned beyond the best event so far; the
    // boxes holding the ray's start never are, so the count is complete.
    // `up`: the count of true members (primitives; terms in term mode) rises at
    // the returned key.
    __device__ __forceinline__ uint64_t query(F3 o, F3 d, F3 ri, F3 oi, uint64_t after, uint32_t& inside, bool& up,
                                              F3& inv, bool& have_inv) {
        QState s;
        qbegin(s, after, o, d, inv, have_inv);
        while (s.cur != kNoRef) trip(s, o, d, ri, oi, inv, have_inv);
        inside = s.cnt;
        if constexpr (kTerms)
            up = s.up;
        else  // a primitive's count rises at its entry
            up = !(s.best & kKeyTypeBit);
        return s.best;
    }

    // Events in key order, one query each, from the count of primitives holding
    // t_min; the root (count > 0) flips at the hit.  A ray that starts outside
    // every primitive needs one query: its first event is an entry.
    __device__ __forceinline__ bool trace_ordered(F3 o, F3 d, Hit& hit) {
        // culling arithmetic only: approximate reciprocals are fine (the boxes carry the slack)
        const float dx = fabsf(d.x) < 1e-30f ? copysignf(1e-30f, d.x) : d.x;
        const float dy = fabsf(d.y) < 1e-30f ? copysignf(1e-30f, d.y) : d.y;
        const float dz = fabsf(d.z) < 1e-30f ? copysignf(1e-30f, d.z) : d.z;
        const F3 ri = f3(__builtin_amdgcn_rcpf(dx), __builtin_amdgcn_rcpf(dy), __builtin_amdgcn_rcpf(dz));
        const F3 oi = f3(o.x * ri.x, o.y * ri.y, o.z * ri.z);
        F3 inv = f3(0.0f, 0.0f, 0.0f);
        bool have_inv = false;
        uint32_t cnt = 0, unused = 0;
        bool up = false;
        uint64_t key = query(o, d, ri, oi, 0ull, cnt, up, inv, have_inv);
        const uint32_t root = cnt > 0u ? 1u : 0u;
        while (key != kEmptyKey) {
            WO_WK(WO_WORK_SWEEP_STEPS);
            cnt = up ? cnt + 1u : cnt - 1u;
            const uint32_t rv = cnt > 0u ? 1u : 0u;
            if (rv != root) {
                hit_from_key(key, rv, hit);
                return true;
            }
            WO_WK(WO_WORK_RECOLLECTS);
            key = query(o, d, ri, oi, key, unused, up, inv, have_inv);
        }
        return false;
    }

    // Resumable trace (kDyn, pathtrace_block's dynamic ray fetch): the walk of a
    // query carries over between calls in `dq`, so a wave whose lanes' walks end
    // at different trips need not run its slowest lane's walk to the end before
    // the finished lanes shade and take their next rays.  Once at most
    // WO_LANES_DYN_WALKERS lanes are still walking (and `may_bail`: the tile's
    // queue still has jobs, so the finished lanes have work to fetch), the walking
    // lanes return kTracePending after a trip and resume from the same state at
    // the next call.  Each call makes at least one trip, so every walk finishes.
    // Same queries, same keys: the hit is trace_ordered's bit for bit.
    QState dq;
    uint32_t dyn_walkers;  // bail-out threshold (LaneBvh::dyn_walkers, wave-uniform)
    uint32_t dcnt;   // the count of true members at the last key processed
    bool droot;      // the root's value at t_min
    bool dfirst;     // the walk in dq is the ray's first query
    bool dpending;   // a walk is in dq (set up by an earlier call)
    __device__ __forceinline__ int trace_step(F3 o, F3 d, Hit& hit, bool may_bail) {
        const float dx = fabsf(d.x) < 1e-30f ? copysignf(1e-30f, d.x) : d.x;
        const float dy = fabsf(d.y) < 1e-30f ? copysignf(1e-30f, d.y) : d.y;
        const float dz = fabsf(d.z) < 1e-30f ? copysignf(1e-30f, d.z) : d.z;
        const F3 ri = f3(__builtin_amdgcn_rcpf(dx), __builtin_amdgcn_rcpf(dy), __builtin_amdgcn_rcpf(dz));
        const F3 oi = f3(o.x * ri.x, o.y * ri.y, o.z * ri.z);
        // the exact reciprocal (generic primitives' axis half-spaces) on first need
        // in this call: the same values whenever it is recomputed
        F3 inv = f3(0.0f, 0.0f, 0.0f);
        bool have_inv = false;
        if (!dpending) {
            qbegin(dq, 0ull, o, d, inv, have_inv);
            dfirst = true;
        }
        for (;;) {
            bool walked = false;
            while (dq.cur != kNoRef) {
                if (walked && may_bail && (uint32_t)__popcll(__ballot(true)) <= dyn_walkers) {
                    dpending = true;
                    return kTracePending;
                }
                trip(dq, o, d, ri, oi, inv, have_inv);
                walked = true;
            }
            const uint64_t key = dq.best;
            const bool up = kTerms ? dq.up : !(key & kKeyTypeBit);
            if (dfirst) {
                dcnt = dq.cnt;
                droot = dcnt > 0u;
                dfirst = false;
            }
            if (key == kEmptyKey) {
                dpending = false;
                return kTraceMiss;
            }
            WO_WK(WO_WORK_SWEEP_STEPS);
            dcnt = up ? dcnt + 1u : dcnt - 1u;
            const bool rv = dcnt > 0u;
            if (rv != droot) {
                hit_from_key(key, rv ? 1u : 0u, hit);
                dpending = false;
                return kTraceHit;
            }
            WO_WK(WO_WORK_RECOLLECTS);
            qbegin(dq, key, o, d, inv, have_inv);
        }
    }

    // ---- general tree (kGeneral) ----
    __device__ __forceinline__ uint32_t gbit(uint32_t ref) const { return (gbits[(ref >> 5) * kBlock] >> (ref & 31u)) & 1u; }
    __device__ __forceinline__ void gflip(uint32_t ref) { gbits[(ref >> 5) * kBlock] ^= 1u << (ref & 31u); }
    // toggle leaf `ord` and re-evaluate its ancestors while their values change
    __device__ __forceinline__ void gtoggle(uint32_t ord) {
        WO_WK(WO_WORK_SWEEP_STEPS);
        uint32_t ref = ord;
        gflip(ref);
        for (;;) {
            const uint32_t par = gpar[ref];
            if (par == kNoRef) break;  // ref is the root
            const uint32_t nd = gnode[par - gP];
            const uint32_t a = gbit(nd & kGRefMask), b = gbit((nd >> kGRefBits) & kGRefMask), op = nd >> 30;
            const uint32_t v = op == 0u ? (a | b) : op == 1u ? (a & b) : op == 2u ? (a & (b ^ 1u)) : (b & (a ^ 1u));
            if (v == gbit(par)) break;
            gflip(par);
            ref = par;
        }
    }
    // the sorted window's insert (branch-free: an early exit once no lane shifts
    // measured slower, 488 against 440 ms on csg360_nested)
    __device__ __forceinline__ void ginsert(uint64_t key) {
#pragma unroll
        for (int i = kGWin - 1; i > 0; --i) gw[i] = key < gw[i - 1] ? gw[i - 1] : (key < gw[i] ? key : gw[i]);
        gw[0] = key < gw[0] ? key : gw[0];
    }
    // Events in key order, kGWin per walk (the walk prunes boxes beyond the largest
    // once it holds kGWin), each toggling its primitive's leaf; the hit is the first
    // key at which the root's value differs from its value at t_min -- the general
    // sweep's hit bit for bit (the tree's value after a key is the program's value of
    // the leaves' membership there).
    __device__ __forceinline__ bool trace_general(F3 o, F3 d, Hit& hit) {
        const float dx = fabsf(d.x) < 1e-30f ? copysignf(1e-30f, d.x) : d.x;
        const float dy = fabsf(d.y) < 1e-30f ? copysignf(1e-30f, d.y) : d.y;
        const float dz = fabsf(d.z) < 1e-30f ? copysignf(1e-30f, d.z) : d.z;
        const F3 ri = f3(__builtin_amdgcn_rcpf(dx), __builtin_amdgcn_rcpf(dy), __builtin_amdgcn_rcpf(dz));
        const F3 oi = f3(o.x * ri.x, o.y * ri.y, o.z * ri.z);
        gri = ri;
        goi = oi;
        F3 inv = f3(0.0f, 0.0f, 0.0f);
        bool have_inv = false;
        for (uint32_t w = 0; w < gwords; ++w) gbits[w * kBlock] = 0u;  // every leaf and node 0
        uint64_t after = 0ull;
        uint32_t root0 = 0u;
        for (;;) {
#pragma unroll
            for (int i = 0; i < kGWin; ++i) gw[i] = kEmptyKey;
            QState s;
            qbegin(s, after, o, d, inv, have_inv);
            while (s.cur != kNoRef) trip(s, o, d, ri, oi, inv, have_inv);
            if (after == 0ull) root0 = gbit(groot);
#pragma unroll
            for (int i = 0; i < kGWin; ++i) {
                const uint64_t key = gw[i];
                if (key == kEmptyKey) return false;  // every event after `after` processed
                gtoggle(key_ord(key));
                const uint32_t rv = gbit(groot);
                if (rv != root0) {
                    hit_from_key(key, rv, hit);
                    return true;
                }
            }
            WO_WK(WO_WORK_RECOLLECTS);
            after = gw[kGWin - 1];
        }
    }

    __device__ __forceinline__ bool trace(F3 o, F3 d, Hit& hit) {
        if constexpr (kGeneral)
            return trace_general(o, d, hit);
        else
            return trace_ordered(o, d, hit);
    }
};

#ifndef WO_LANES_MIN_WAVES
#define WO_LANES_MIN_WAVES 8  // rtiow_cover: 40.0 ms at 6, 37.4 at 7, 36.5 at 8 (64 VGPRs)
#endif
// The ordered-BVH tables of a union-only program (build_lbvh).
struct LaneBvh {
    const float4* nodes;
    const float4* geo;
    const uint32_t* kind;  // per ordinal, then the always list
    const float4* trec;    // term mode: kTermRecF4 float4 per term
    const WoRec* leaves;   // single-sphere scenes: per ordinal its leaf record
    uint32_t nalways, root, nprims;
    uint32_t depth;        // internal levels of the tree: the lane stack's entries
    uint32_t ntop;         // nodes [0, ntop) staged in LDS after the lane stacks
    uint32_t dyn_walkers;  // resumable walk: walking lanes at which a wave bails out
    // general tree (kind 7): parent per ref, node records, leaves, words per lane, root ref
    const uint32_t* gpar;
    const uint32_t* gnode;
    const float4* gclip;  // per primitive: relevance box lo (w: 1 = clip) and hi; nullptr: none
    uint32_t gP, gwords, groot;
};

// Dynamic LDS: the BVH walk's lane stacks ([depth][kBlock] u32 or u16) and top nodes.
#ifndef WO_LANES_BVH_MIN_WAVES
#define WO_LANES_BVH_MIN_WAVES 7  // rtiow_cover: 16.86 ms at 8, 16.63 at 7, 17.26 at 6
#endif
template <int kMode, bool kCount>
#ifndef WO_LANES_TERMS_MIN_WAVES
#define WO_LANES_TERMS_MIN_WAVES 7  // csg512_balanced: 80.8 ms at 7 (13 VGPRs spilled), 82.0 at 6 (none)
#endif
#ifndef WO_LANES_DYN_MIN_WAVES
#define WO_LANES_DYN_MIN_WAVES 7
#endif
#ifndef WO_LANES_DYN_TERMS_MIN_WAVES
#define WO_LANES_DYN_TERMS_MIN_WAVES 6  // csg512_balanced: 56.4 ms at 6 (no spill), 57.2 at 7 (31 VGPRs spilled)
#endif
#ifndef WO_LANES_GENERAL_MIN_WAVES
#define WO_LANES_GENERAL_MIN_WAVES 4  // the tree's bits take ~20 KB of LDS per workgroup (csg360_nested)
#endif
__global__ __launch_bounds__(kBlock, kMode == 14  ? WO_LANES_DYN_TERMS_MIN_WAVES
                                    : kMode == 7 ? WO_LANES_GENERAL_MIN_WAVES
                                    : kMode == 6 ? WO_LANES_TERMS_MIN_WAVES
                                    : kMode == 2 ? WO_LANES_BVH_MIN_WAVES
                                                 : WO_LANES_MIN_WAVES) void pathtrace_lanes_kernel(
    const WoRec* __restrict__ prog, const uint32_t* __restrict__ ordpc, const WoMaterial* __restrict__ mats, WoFrame fr,
    uint32_t local_rows, float4* __restrict__ out, unsigned long long* __restrict__ seg_slots, PathLaunch tg,
    LaneBvh bvh) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    LaneTracer<kMode, kCount> tr;
    tr.prog = prog;
    tr.ordpc = ordpc;
    tr.lnodes = bvh.nodes;
    tr.lgeo = bvh.geo;
    tr.lkind = bvh.kind;
    tr.ltrec = bvh.trec;
    tr.lleaf = bvh.leaves;
    tr.nalways = bvh.nalways;
    tr.lroot = bvh.root;
    tr.nprims = bvh.nprims;
    tr.stk = smem + threadIdx.x;
    tr.stk16 = reinterpret_cast<uint16_t*>(smem) + threadIdx.x;
    tr.ntop = 0;
    tr.ltop = (typename LaneTracer<kMode, kCount>::LdsNodes)nullptr;
    if constexpr (LaneTracer<kMode, kCount>::kDyn) {
        tr.dpending = false;
        tr.dyn_walkers = bvh.dyn_walkers;
    }
    {
        // the top levels of the BVH next to the stacks; pathtrace_block's first
        // barrier orders the copy before any walk
        constexpr bool kStack16 = LaneTracer<kMode, kCount>::kStack16;
        const uint32_t stack_words = kStack16 ? (bvh.depth * kBlock + 1u) / 2u : bvh.depth * kBlock;
        float4* top = reinterpret_cast<float4*>(smem + ((stack_words + 3u) & ~3u));
        constexpr uint32_t kNodeF4 = LaneTracer<kMode, kCount>::kNodeF4;
        for (uint32_t i = threadIdx.x; i < kNodeF4 * bvh.ntop; i += kBlock) top[i] = bvh.nodes[i];
        tr.ltop = (typename LaneTracer<kMode, kCount>::LdsNodes)top;
        tr.ntop = bvh.ntop;
        if constexpr (LaneTracer<kMode, kCount>::kGeneral) {
            // the tree's bits after the top nodes, [word][lane]
            tr.gbits = reinterpret_cast<uint32_t*>(top + kNodeF4 * bvh.ntop) + threadIdx.x;
            tr.gpar = bvh.gpar;
            tr.gnode = bvh.gnode;
            tr.gclip = bvh.gclip;
            tr.gP = bvh.gP;
            tr.gwords = bvh.gwords;
            tr.groot = bvh.groot;
        }
    }
    pathtrace_block(tr, mats, fr, local_rows, out, seg_slots, tg);
}

// ---------------------------------------------------------------------------
// ubershader1.frag restated (ref ubershader1.frag:19-163).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void ubershader_kernel(WoFrame fr, uint32_t local_rows, float4* __restrict__ out) {
    uint32_t lx = blockIdx.x * kBlock + threadIdx.x;
    uint32_t lrow = blockIdx.y;
    if (lx >= fr.width || lrow >= local_rows) return;
    uint32_t y = local_to_global_row(fr, lrow);
    if (y >= fr.height) return;

    float resx = (float)fr.width, resy = (float)fr.height;
    float aspect = resx / resy;   // frag:20
    float fx = (float)lx + 0.5f;  // gl_FragCoord at the pixel centre,
    float fy = (float)y + 0.5f;   // OriginUpperLeft (row 0 = top)
    float stx = fx / resx;        // frag:26-29
    float sty = 1.0f - fy / resy;
    float4 res;
    if (fr.mode == WO_MODE_DEBUG_ST) {  // frag:133-138
        res = make_float4(stx, sty, 0.0f, 1.0f);
    } else {
        // camera (frag:50-60): llc = (-aspect/2, -0.5, -1); ray dir (frag:74-82), not normalised
        float dx = (0.0f - aspect * 0.5f) + stx * aspect;
        float dy = -0.5f + sty;
        float dz = -1.0f;
        // hit_sphere (frag:84-95), centre (0, 2 sin(w t), -11), r = 0.5 (frag:100-105)
        float sy = fr.sphere_y;
        float ocy = 0.0f - sy;
        float ocz = 11.0f;
        float a = (dx * dx + dy * dy) + dz * dz;
        float b = 2.0f * ((0.0f * dx + ocy * dy) + ocz * dz);
        float c = ((0.0f * 0.0f + ocy * ocy) + ocz * ocz) - 0.5f * 0.5f;
        float disc = b * b - (4.0f * a) * c;
        float t = -1.0f;
        if (!(disc < 0.0f)) t = (-b - sqrtf(disc)) / (2.0f * a);
        if (t > 0.0f) {  // frag:107-111
            float nx = dx * t - 0.0f, ny = dy * t - sy, nz = dz * t - (-11.0f);
            float len = sqrtf((nx * nx + ny * ny) + nz * nz);
            nx = nx / len;
            ny = ny / len;
            nz = nz / len;
            res = make_float4(0.5f * (nx + 1.0f), 0.5f * (ny + 1.0f), 0.5f * (nz + 1.0f), 1.0f);
        } else {  // frag:116-122
            float len = sqrtf((dx * dx + dy * dy) + dz * dz);
            float uy = dy / len;
            float s = 1.0f - uy;
            res = make_float4(s + uy * 0.5f, s + uy * 0.7f, s + uy * 1.0f, 1.0f);
        }
    }
    out[(size_t)lrow * fr.width + lx] = res;
}

template <bool kProgInLds, bool kCount>
__global__ __launch_bounds__(kBlock) void pathtrace_kernel(const WoRec* __restrict__ gprog,
                                                           const WoMaterial* __restrict__ mats, WoFrame fr,
                                                           KLayout lay, uint32_t local_rows,
                                                           float4* __restrict__ out,
                                                           unsigned long long* __restrict__ seg_slots,
                                                           PathLaunch tg) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t nrec = fr.n_recs;

    uint32_t* scratch = smem;
    InterpTracer<kCount> tr;
    if constexpr (kProgInLds) {
        const uint4* src = reinterpret_cast<const uint4*>(gprog);
        uint4* dst = reinterpret_cast<uint4*>(smem);
        for (uint32_t i = tid; i < nrec * 2u; i += kBlock) dst[i] = src[i];
        __syncthreads();
        tr.prog.p = reinterpret_cast<const WoRec*>(smem);
        scratch = smem + nrec * 8u;
    } else {
        tr.prog.p = gprog;
    }
    uint32_t* ws = scratch + wave * lay.wave_words;
    tr.nrec = nrec;
    tr.codes = ws;
    tr.ordpc = ws + lay.ordpc_off;
    tr.hib = ws + lay.hib_off;
    tr.lane = lane;
    pathtrace_block(tr, mats, fr, local_rows, out, seg_slots, tg);
}

// Sums (and clears) the segment slots into the caller's counter.
__global__ __launch_bounds__(kBlock) void seg_collect_kernel(unsigned long long* __restrict__ slots,
                                                             unsigned long long* __restrict__ counter) {
    __shared__ unsigned long long part[kBlock / 64];
    unsigned long long v = 0;
    for (uint32_t i = threadIdx.x; i < kSegSlots; i += kBlock) {
        // read and clear in one atomic: a kernel of another stream may be adding
        v += atomicExch(&slots[i * kSegStride], 0ull);
    }
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63u) == 0u) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0u) {
        unsigned long long t = 0;
        for (uint32_t w = 0; w < kBlock / 64u; ++w) t += part[w];
        if (t) atomicAdd(counter, t);
    }
}

// Sums (and clears) the work counters of the segment slots (kinds 1..) into
// out[kind] (counting launches).
__global__ __launch_bounds__(kBlock) void work_collect_kernel(unsigned long long* __restrict__ slots,
                                                              unsigned long long* __restrict__ out) {
    __shared__ unsigned long long part[WO_WORK_KINDS][kBlock / 64];
    static_assert(kSegSlots == kBlock, "one slot per thread");
    const uint32_t i = threadIdx.x;
#pragma unroll
    for (uint32_t k = 1; k < WO_WORK_KINDS; ++k) {
        unsigned long long v = slots[i * kSegStride + k];
        slots[i * kSegStride + k] = 0ull;
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if ((i & 63u) == 0u) part[k][i >> 6] = v;
    }
    __syncthreads();
    if (i > 0u && i < WO_WORK_KINDS) {
        unsigned long long t = 0;
        for (uint32_t w = 0; w < kBlock / 64u; ++w) t += part[i][w];
        out[i] = t;
    }
}

__global__ __launch_bounds__(kBlock) void assemble_kernel(const float4* __restrict__ gathered, float4* __restrict__ frame,
                                                          uint32_t W, uint32_t H, uint32_t T, uint32_t N,
                                                          uint32_t cycle, uint32_t skip, uint32_t local_rows) {
    size_t total = (size_t)W * H;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < total; i += (size_t)gridDim.x * kBlock) {
        uint32_t y = (uint32_t)(i / W), x = (uint32_t)(i - (size_t)y * W);
        uint32_t g = y / T;
        uint32_t r, lb;
        band_local(g, N, cycle, skip, r, lb);
        uint32_t lrow = lb * T + (y - g * T);
        frame[i] = gathered[((size_t)r * local_rows + lrow) * W + x];
    }
}

// Present encode (present.c): float RGBA -> B8G8R8A8 sRGB, the reference's
// preferred swapchain format (renderer.c:813-832).  A channel's code is the
// count of the 255 thresholds <= its value (binary search in LDS), which is
// round-half-up(255 * srgb(clamp(v))) exactly; NaN -> 0.  HBM-bound: 16 B read
// + 4 B written per pixel.
__device__ __forceinline__ uint32_t srgb8_code(const float* t, float v) {
    uint32_t k = 0;
#pragma unroll
    for (uint32_t s = 128u; s > 0u; s >>= 1)
        if (t[k + s - 1u] <= v) k += s;  // t[255] = +inf keeps k <= 255
    return k;
}
__device__ __forceinline__ uint32_t unorm8(float a) {
    if (!(a > 0.0f)) return 0u;
    if (a >= 1.0f) return 255u;
    return (uint32_t)((double)a * 255.0 + 0.5);  // exact in double: round-half-up
}
__global__ __launch_bounds__(kBlock) void srgb8_kernel(const float4* __restrict__ in, uint32_t* __restrict__ out,
                                                       size_t n, const float* __restrict__ tab) {
    __shared__ float t[256];
    t[threadIdx.x] = threadIdx.x < 255u ? tab[threadIdx.x] : kInf;
    __syncthreads();
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        const float4 p = in[i];
        out[i] = srgb8_code(t, p.z) | (srgb8_code(t, p.y) << 8) | (srgb8_code(t, p.x) << 16) | (unorm8(p.w) << 24);
    }
}

// Exhaustive check of sqrt_cr / rcp_cr over float bit patterns [lo, lo + count)
// against the definition of correct rounding, evaluated exactly in double
// (independent of any library expansion): s = RN(sqrt x) iff (s - u/2)^2 <= x
// <= (s + u/2)^2, u = ulp(s) (the squares of 25-bit numbers are exact in double,
// and no float x sits on a midpoint); r = RN(1/x) iff |1 - r x| <= (u/2) |x|,
// u = ulp(r) (r x is exact in double).  Counts the patterns that fail.
__global__ __launch_bounds__(kBlock) void fastmath_check_kernel(uint32_t lo, uint32_t count, int which,
                                                                unsigned long long* __restrict__ bad,
                                                                uint32_t* __restrict__ first_bad) {
    unsigned long long nbad = 0;
    uint32_t first = 0xffffffffu;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < count; i += gridDim.x * kBlock) {
        const uint32_t u = lo + i;
        const float x = __uint_as_float(u);
        bool ok;
        if (which == 0) {
            const float s = sqrt_cr(x);
            const double sd = s, h = 0.5 * ((double)__uint_as_float(__float_as_uint(s) + 1u) - sd);
            ok = (sd - h) * (sd - h) <= (double)x && (double)x <= (sd + h) * (sd + h);
        } else {
            const float r = rcp_cr(x);
            const double rd = r, h = 0.5 * fabs((double)__uint_as_float(__float_as_uint(r) + 1u) - rd);
            ok = fabs(1.0 - rd * (double)x) <= h * fabs((double)x);
        }
        if (!ok) {
            ++nbad;
            first = u < first ? u : first;
        }
    }
    for (int off = 32; off > 0; off >>= 1) nbad += __shfl_xor(nbad, off, 64);
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)first, off, 64);
        first = o < first ? o : first;
    }
    if ((threadIdx.x & 63u) == 0u) {
        if (nbad) atomicAdd(bad, nbad);
        if (first != 0xffffffffu) atomicMin(first_bad, first);
    }
}

}  // namespace

extern "C" int wo_fastmath_check(int which, uint32_t lo_bits, uint32_t hi_bits, unsigned long long* mismatches,
                                 uint32_t* first_mismatch) {
    unsigned long long* d_bad = nullptr;
    uint32_t* d_first = nullptr;
    if (hi_bits < lo_bits) return -1;
    if (hipMalloc((void**)&d_bad, sizeof *d_bad) != hipSuccess) return -1;
    if (hipMalloc((void**)&d_first, sizeof *d_first) != hipSuccess) {
        (void)hipFree(d_bad);
        return -1;
    }
    const uint32_t init = 0xffffffffu;
    hipError_t e = hipMemset(d_bad, 0, sizeof *d_bad);
    if (e == hipSuccess) e = hipMemcpy(d_first, &init, sizeof init, hipMemcpyHostToDevice);
    const uint64_t total = (uint64_t)hi_bits - lo_bits + 1u;
    for (uint64_t done = 0; e == hipSuccess && done < total;) {
        const uint32_t n = (uint32_t)(total - done < (1ull << 30) ? total - done : (1ull << 30));
        hipLaunchKernelGGL(fastmath_check_kernel, dim3(8192), dim3(kBlock), 0, nullptr, (uint32_t)(lo_bits + done), n,
                           which, d_bad, d_first);
        e = hipGetLastError();
        done += n;
    }
    if (e == hipSuccess) e = hipMemcpy(mismatches, d_bad, sizeof *d_bad, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(first_mismatch, d_first, sizeof *d_first, hipMemcpyDeviceToHost);
    (void)hipFree(d_bad);
    (void)hipFree(d_first);
    return e == hipSuccess ? 0 : -1;
}

// ===========================================================================
// Host glue (C ABI declared in wo_dev.h)
// ===========================================================================
// big tiles per resident workgroup of a rank's share (plan_tiles), every kernel;
// a generated source may name its own (`// wo_share_tiles N`, scene_jit.c)
constexpr uint32_t kShareTiles = 3u;

struct WoDev {
    int device;
    int cus;           // compute units (multiProcessorCount)
    std::string arch;  // gcnArchName, e.g. gfx950:sramecc+:xnack-
    WoRec* d_prog;
    size_t prog_cap;
    WoMaterial* d_mats;
    size_t mats_cap;
    uint32_t n_recs, n_prims, n_mats;
    float4* d_frame;
    size_t frame_cap;
    hipStream_t stream;
    // lane tracer: ordinal -> program pc (generic primitives, hit leaves)
    uint32_t* d_ordpc;
    size_t ordpc_cap;
    // the lane tracer's ordered BVH (build_lbvh): [4 float4 per node][float4 per
    // ordinal] then u32 [kind per ordinal][always list]
    float4* d_lbvh;
    size_t lbvh_cap;
    uint32_t lb_nodes, lb_always, lb_root, lb_nprims;
    bool lb_spheres_only;  // every primitive is a single sphere (kind 3)
    bool lb_stack16;       // 16-bit stack entries (the 4-wide tree)
    bool lb_wide;          // 4-wide nodes of 7 float4 (lb_collapse4; kind 14)
    uint32_t lb_terms;     // term mode (kinds 6 / 14): terms the BVH's leaves and always list refer to
    bool lb_general;       // a general tree (kind 7): the BVH over primitives, the tree's tables below
    uint32_t lb_gpar_off, lb_gnode_off;  // u32 offsets in d_lbvh of the parent per ref / node records
    uint32_t lb_gclip_off;               // u32 offset of the primitives' relevance boxes (0: none)
    uint32_t lb_gP, lb_gwords, lb_groot;  // leaves (= primitives), bit words per lane, the root's ref
    uint32_t last_kind;    // the PathKind of the last path launch (wo_dev_lanes_info)
    uint32_t lb_term_off;  // their records (kTermRecF4 float4 each) at this u32 offset of d_lbvh
    uint32_t lb_leaf_off;  // single-sphere scenes: per ordinal its leaf record (WoRec) at this u32 offset, else 0
    uint32_t lb_top;       // nodes staged in LDS per workgroup
    uint32_t lb_depth;     // internal levels of the lane BVH (<= kLaneDepthMax)
    unsigned long long* d_segslots;  // kSegSlots segment counters, kSegStride apart
    unsigned long long* d_work;      // WO_WORK_KINDS totals of a counting launch
    // progressive accumulation (3 int64 per pixel) and the frame slots (wo_dev.h
    // WO_SLOT_*): the draw_frame pipeline's two, the synchronous render's scratch
    // slot and the two device-frame slots; a present slot holds a device frame, a
    // pinned host copy and an event
    long long* d_accum;
    size_t accum_cap;
    float4* d_slot[WO_SLOTS];
    size_t dslot_cap[WO_SLOTS];
    float* h_slot[WO_SLOTS];
    size_t hslot_cap[WO_SLOTS];
    uint32_t* d_bgra[WO_SLOTS];  // the slot's frame encoded for present (B8G8R8A8 sRGB)
    size_t dbgra_cap[WO_SLOTS];
    uint32_t* h_bgra[WO_SLOTS];
    size_t hbgra_cap[WO_SLOTS];
    hipEvent_t slot_ev[WO_SLOTS];  // the slot's map-back is done (on copy_stream)
    // Map-back of presented frames: the present encode and
    // the D2H copies run on their own stream, gated by rend_ev (the slot's frame is
    // rendered), so the next frame's kernel starts as soon as this one ends.
    hipStream_t copy_stream;
    // On-demand float map-back of a presented frame (wo_dev_frame_map_float): its own
    // stream, created on first use, so it never queues behind the next frame's
    // map-back on copy_stream (which waits for that frame's render).
    hipStream_t map_stream;
    hipEvent_t rend_ev[WO_SLOTS];
    bool slot_float[WO_SLOTS];  // the float frame was copied with the last map-back
    size_t slot_pixels[WO_SLOTS];  // pixels of the slot's last frame
    bool slot_recorded[WO_SLOTS];  // slot_ev has been recorded (never wait on an unrecorded event)
    // pipeline timestamps (wo_dev_set_stamps): render begin / render end / map-back end
    bool stamps;
    hipEvent_t st_base;
    hipEvent_t st_ev[WO_SLOTS][3];
    bool st_valid[WO_SLOTS];
    // several devices per renderer (wo_dev_frame_submit_ranks): on the root,
    // the rank-major buffer the ranks' shares are copied into and the event that
    // opens a slot to the ranks; on every rank, its share of the frame and the
    // event that marks the share delivered (copied, or staged in host memory)
    float4* d_gather[WO_SLOTS];
    size_t dgather_cap[WO_SLOTS];
    hipEvent_t gate_ev[WO_SLOTS];
    float4* d_part[WO_SLOTS];
    size_t dpart_cap[WO_SLOTS];
    float4* h_part[WO_SLOTS];  // WO_PEER_STAGED: the share's pinned host copy
    size_t hpart_cap[WO_SLOTS];
    hipEvent_t part_ev[WO_SLOTS];
    // the split present (present_rows): this rank's rows encoded for present, and the
    // events that order its encode after its render (psrc), the gather's reuse of
    // the share after the encode (penc) and the root's slot after the D2H (pmap)
    uint32_t* d_pbgra[WO_SLOTS];
    size_t dpbgra_cap[WO_SLOTS];
    hipEvent_t psrc_ev[WO_SLOTS], penc_ev[WO_SLOTS], pmap_ev[WO_SLOTS];
    int peer_mode;  // how this rank's share reaches the root (WO_PEER_*; wo_dev_enable_peer)
    unsigned long long* d_segacc;  // segments of this rank's device frames (wo_dev_take_segments)
    bool union_only;
    bool lanes_on;
    // scene-specialised kernel (hiprtc)
    hipModule_t jit_module;
    hipFunction_t jit_fn;
    uint32_t jit_share_tiles;  // big tiles per resident workgroup for the specialised kernel (plan_tiles)
    std::string jit_key;  // SHA-256 (hex) of the loaded code object's inputs
    std::string jit_src;  // its source (the counting variant is built from it on demand)
    hipModule_t count_module;
    hipFunction_t count_fn;
    int jit_attr[3];  // the loaded specialised kernel's scratch bytes per lane, VGPRs, static LDS (kernel_info)
    int jit_origin;       // 0 process cache, 1 disk cache, 2 compiled
    double jit_compile_sec;
};

static void set_err(char* err, size_t len, const char* what, hipError_t e) {
    if (err && len) snprintf(err, len, "%s: %s", what, hipGetErrorString(e));
}

// Zero device memory and wait for it: hipMemset may still be running on the null
// stream when a kernel on one of the non-blocking streams starts, and a late
// memset would wipe what that kernel counted.  (One-time set-ups only.)
static hipError_t zero_now(void* p, size_t bytes) {
    hipError_t e = hipMemset(p, 0, bytes);
    return e == hipSuccess ? hipDeviceSynchronize() : e;
}

extern "C" int wo_hip_runtime_version(void) {
    int v = 0;
    return hipRuntimeGetVersion(&v) == hipSuccess ? v : -1;
}

extern "C" int wo_dev_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" int wo_dev_device(WoDev* dev) { return dev ? dev->device : -1; }

extern "C" int wo_dev_select(int device) { return hipSetDevice(device) == hipSuccess ? 0 : -1; }

extern "C" int wo_dev_current(void) {
    int d = -1;
    if (hipGetDevice(&d) != hipSuccess) return -1;
    return d;
}

extern "C" int wo_dev_create(int device, WoDev** out, char* err, size_t errlen) {
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipSetDevice", e);
        return -1;
    }
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipGetDeviceProperties", e);
        return -1;
    }
    WoDev* dev = new (std::nothrow) WoDev();
    if (!dev) {
        snprintf(err, errlen, "out of host memory");
        return -1;
    }
    dev->device = device;
    dev->cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 1;
    dev->arch = prop.gcnArchName;
    e = hipStreamCreateWithFlags(&dev->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipStreamCreate", e);
        delete dev;
        return -1;
    }
    e = hipStreamCreateWithFlags(&dev->copy_stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipStreamCreate(copy)", e);
        (void)hipStreamDestroy(dev->stream);
        delete dev;
        return -1;
    }
    *out = dev;
    return 0;
}

extern "C" void wo_dev_destroy(WoDev* dev) {
    if (!dev) return;
    (void)hipSetDevice(dev->device);
    // device frames assemble on the caller's stream from this rank's buffers
    (void)hipDeviceSynchronize();
    if (dev->d_prog) (void)hipFree(dev->d_prog);
    if (dev->d_mats) (void)hipFree(dev->d_mats);
    if (dev->d_frame) (void)hipFree(dev->d_frame);
    if (dev->d_lbvh) (void)hipFree(dev->d_lbvh);
    if (dev->d_ordpc) (void)hipFree(dev->d_ordpc);
    if (dev->d_segslots) (void)hipFree(dev->d_segslots);
    if (dev->d_work) (void)hipFree(dev->d_work);
    if (dev->d_accum) (void)hipFree(dev->d_accum);
    if (dev->d_segacc) (void)hipFree(dev->d_segacc);
    for (int i = 0; i < WO_SLOTS; ++i) {
        if (dev->h_part[i]) (void)hipHostFree(dev->h_part[i]);
        if (dev->d_slot[i]) (void)hipFree(dev->d_slot[i]);
        if (dev->h_slot[i]) (void)hipHostFree(dev->h_slot[i]);
        if (dev->slot_ev[i]) (void)hipEventDestroy(dev->slot_ev[i]);
        if (dev->d_bgra[i]) (void)hipFree(dev->d_bgra[i]);
        if (dev->h_bgra[i]) (void)hipHostFree(dev->h_bgra[i]);
        if (dev->d_gather[i]) (void)hipFree(dev->d_gather[i]);
        if (dev->gate_ev[i]) (void)hipEventDestroy(dev->gate_ev[i]);
        if (dev->d_part[i]) (void)hipFree(dev->d_part[i]);
        if (dev->part_ev[i]) (void)hipEventDestroy(dev->part_ev[i]);
        if (dev->d_pbgra[i]) (void)hipFree(dev->d_pbgra[i]);
        for (hipEvent_t ev : {dev->psrc_ev[i], dev->penc_ev[i], dev->pmap_ev[i]})
            if (ev) (void)hipEventDestroy(ev);
        if (dev->rend_ev[i]) (void)hipEventDestroy(dev->rend_ev[i]);
        for (int k = 0; k < 3; ++k)
            if (dev->st_ev[i][k]) (void)hipEventDestroy(dev->st_ev[i][k]);
    }
    if (dev->st_base) (void)hipEventDestroy(dev->st_base);
    if (dev->jit_module) (void)hipModuleUnload(dev->jit_module);
    if (dev->count_module) (void)hipModuleUnload(dev->count_module);
    if (dev->map_stream) (void)hipStreamDestroy(dev->map_stream);
    (void)hipStreamDestroy(dev->copy_stream);
    (void)hipStreamDestroy(dev->stream);
    delete dev;
}

template <class T>
static int ensure_buffer(T** p, size_t* cap, size_t bytes, char* err, size_t errlen) {
    if (bytes <= *cap && *p) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    size_t alloc = bytes ? bytes : 64;
    hipError_t e = hipMalloc((void**)p, alloc);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipMalloc", e);
        return -1;
    }
    *cap = alloc;
    return 0;
}

// Whether the program is union-only (the lane tracer's union count), and the
// ordinal -> program pc map the lane tracer reads generic primitives and hit
// leaves through.
static int scene_maps(WoDev* dev, WoRec const* prog, uint32_t n_recs, uint32_t n_prims, char* err, size_t errlen) {
    bool union_only = n_prims > 0;
    std::vector<uint32_t> ordpc(n_prims ? n_prims : 1u, 0u);
    for (uint32_t pc = 0; pc < n_recs;) {
        const uint32_t op = prog[pc].op;
        if (op == WO_OP_PRIM) {
            if (prog[pc].u1 < n_prims) ordpc[prog[pc].u1] = pc;
            pc += 1u + prog[pc].u0;
        } else {
            if (op != WO_OP_UNION && op != WO_OP_BOUND) union_only = false;
            ++pc;
        }
    }
    dev->union_only = union_only;
    if (ensure_buffer(&dev->d_ordpc, &dev->ordpc_cap, ordpc.size() * sizeof(uint32_t), err, errlen)) return -1;
    hipError_t e = hipMemcpy(dev->d_ordpc, ordpc.data(), ordpc.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipMemcpy(ordinal map)", e);
        return -1;
    }
    return 0;
}

// ---- the lane tracer's ordered BVH ----
// Axis-aligned box of a convex primitive from its members (spheres, axis-aligned
// half-spaces; general planes bound nothing), in double; false if unbounded or
// empty.
static bool prim_aabb(WoRec const* prog, uint32_t pc, double lo[3], double hi[3]) {
    for (int a = 0; a < 3; ++a) {
        lo[a] = -INFINITY;
        hi[a] = INFINITY;
    }
    for (uint32_t m = 0; m < prog[pc].u0; ++m) {
        const WoRec& L = prog[pc + 1u + m];
        if (L.op == WO_LEAF_SPHERE) {
            const double r = sqrt((double)L.f[3]);
            for (int a = 0; a < 3; ++a) {
                lo[a] = fmax(lo[a], (double)L.f[a] - r);
                hi[a] = fmin(hi[a], (double)L.f[a] + r);
            }
        } else if (L.op == WO_LEAF_HALFSPACE && L.u1 >= 1u && L.u1 <= 3u) {
            const int a = (int)L.u1 - 1;  // s * x_a <= h
            if (L.f[a] > 0.0f)
                hi[a] = fmin(hi[a], (double)L.f[3]);
            else
                lo[a] = fmax(lo[a], -(double)L.f[3]);
        }
    }
    for (int a = 0; a < 3; ++a)
        if (!std::isfinite(lo[a]) || !std::isfinite(hi[a]) || lo[a] > hi[a]) return false;
    return true;
}

struct LbPrim {
    double lo[3], hi[3], c[3];
    uint32_t ord;
};

struct LbBox {
    double lo[3], hi[3];
    void empty() {
        for (int a = 0; a < 3; ++a) {
            lo[a] = INFINITY;
            hi[a] = -INFINITY;
        }
    }
    void grow(const double* l, const double* h) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = fmin(lo[a], l[a]);
            hi[a] = fmax(hi[a], h[a]);
        }
    }
    double area() const {
        const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
        return x < 0.0 ? 0.0 : 2.0 * (x * y + y * z + z * x);
    }
};

static uint32_t ceil_log2(uint32_t c) {
    uint32_t k = 0;
    while ((1ull << k) < c) ++k;
    return k;
}

// Binned-SAH build over prims[b, e) with at most `levels` internal levels below
// (ceil_log2(e - b) <= levels on entry); returns the subtree's ref and its
// depth.  A SAH split that would leave a child more primitives than its levels
// can hold becomes the median split, which always fits.  Node n is written to
// nodes[4n..4n+3] as the two children's boxes (rounded outward to float) with
// their refs in the .w of the first two.
static uint32_t lb_build(std::vector<LbPrim>& prims, uint32_t b, uint32_t e, uint32_t levels,
                         std::vector<float4>& nodes, LbBox& box_out, uint32_t& depth_out) {
    box_out.empty();
    for (uint32_t i = b; i < e; ++i) box_out.grow(prims[i].lo, prims[i].hi);
    depth_out = 0;
    if (e - b == 1u) return kLeafRef | prims[b].ord;
    LbBox cb;
    cb.empty();
    for (uint32_t i = b; i < e; ++i) cb.grow(prims[i].c, prims[i].c);
    int axis = 0;
    for (int a = 1; a < 3; ++a)
        if (cb.hi[a] - cb.lo[a] > cb.hi[axis] - cb.lo[axis]) axis = a;
    uint32_t mid = b + (e - b) / 2u;
    const double ext = cb.hi[axis] - cb.lo[axis];
    if (ext > 0.0) {
        constexpr int kBins = 16;
        LbBox bb[kBins];
        uint32_t bn[kBins] = {};
        for (int k = 0; k < kBins; ++k) bb[k].empty();
        auto bin_of = [&](const LbPrim& p) {
            int k = (int)((p.c[axis] - cb.lo[axis]) / ext * kBins);
            return k < 0 ? 0 : (k >= kBins ? kBins - 1 : k);
        };
        for (uint32_t i = b; i < e; ++i) {
            const int k = bin_of(prims[i]);
            bb[k].grow(prims[i].lo, prims[i].hi);
            ++bn[k];
        }
        double best = INFINITY;
        int split = -1;
        for (int s = 1; s < kBins; ++s) {
            LbBox l, r;
            l.empty();
            r.empty();
            uint32_t nl = 0, nr = 0;
            for (int k = 0; k < s; ++k) l.grow(bb[k].lo, bb[k].hi), nl += bn[k];
            for (int k = s; k < kBins; ++k) r.grow(bb[k].lo, bb[k].hi), nr += bn[k];
            if (!nl || !nr) continue;
            const double cost = l.area() * nl + r.area() * nr;
            if (cost < best) best = cost, split = s;
        }
        if (split > 0) {
            auto it = std::partition(prims.begin() + b, prims.begin() + e,
                                     [&](const LbPrim& p) { return bin_of(p) < split; });
            mid = (uint32_t)(it - prims.begin());
        }
    }
    if (mid == b || mid == e || ceil_log2(mid - b) >= levels || ceil_log2(e - mid) >= levels) {
        // no useful split, or one too deep for the lane stack: the median along the axis
        mid = b + (e - b) / 2u;
        std::nth_element(prims.begin() + b, prims.begin() + mid, prims.begin() + e,
                         [&](const LbPrim& x, const LbPrim& y) { return x.c[axis] < y.c[axis]; });
    }
    const uint32_t n = (uint32_t)(nodes.size() / 4u);
    nodes.resize(nodes.size() + 4u);
    LbBox lb, rb;
    uint32_t ld, rd;
    const uint32_t lref = lb_build(prims, b, mid, levels - 1u, nodes, lb, ld);
    const uint32_t rref = lb_build(prims, mid, e, levels - 1u, nodes, rb, rd);
    depth_out = 1u + (ld > rd ? ld : rd);
    auto bits_f = [](uint32_t u) {
        float f;
        memcpy(&f, &u, sizeof f);
        return f;
    };
    auto down = [](double v) { return nextafterf((float)v, -INFINITY); };
    auto up = [](double v) { return nextafterf((float)v, INFINITY); };
    float4* q = &nodes[4u * n];
    q[0] = make_float4(down(lb.lo[0]), down(lb.lo[1]), down(lb.lo[2]), bits_f(lref));
    q[1] = make_float4(up(lb.hi[0]), up(lb.hi[1]), up(lb.hi[2]), bits_f(rref));
    q[2] = make_float4(down(rb.lo[0]), down(rb.lo[1]), down(rb.lo[2]), 0.0f);
    q[3] = make_float4(up(rb.hi[0]), up(rb.hi[1]), up(rb.hi[2]), 0.0f);
    return n;
}

// 4-wide tree from lb_build's binary one (refs before the breadth-first order):
// a node takes its two children and, while it has fewer than four, replaces the
// internal child of largest surface area by that child's two children.  Node n
// is written to n4[7n..7n+6]: lo.x, hi.x, lo.y, hi.y, lo.z, hi.z of the four
// children (the binary nodes' expanded, outward-rounded boxes), then their refs
// (kNoRef for an empty slot; lb_bfs4 turns them into 16-bit refs, kNoRef16).
// `levels` = internal levels on the longest path.
struct Lb4Child {
    float lo[3], hi[3];
    uint32_t ref;
    double area() const {
        const double x = (double)hi[0] - lo[0], y = (double)hi[1] - lo[1], z = (double)hi[2] - lo[2];
        return 2.0 * (x * y + y * z + z * x);
    }
};
static void lb_children2(const std::vector<float4>& n2, uint32_t n, Lb4Child out[2]) {
    const float4* q = &n2[4u * n];
    const float4 lo[2] = {q[0], q[2]}, hi[2] = {q[1], q[3]};
    for (int c = 0; c < 2; ++c) {
        out[c].lo[0] = lo[c].x, out[c].lo[1] = lo[c].y, out[c].lo[2] = lo[c].z;
        out[c].hi[0] = hi[c].x, out[c].hi[1] = hi[c].y, out[c].hi[2] = hi[c].z;
        memcpy(&out[c].ref, c == 0 ? &q[0].w : &q[1].w, sizeof(uint32_t));
    }
}
static uint32_t lb_collapse4(const std::vector<float4>& n2, uint32_t n, std::vector<float4>& n4, uint32_t& levels) {
    std::vector<Lb4Child> ch(2);
    lb_children2(n2, n, ch.data());
    while (ch.size() < 4u) {
        int pick = -1;
        double best = -1.0;
        for (int i = 0; i < (int)ch.size(); ++i)
            if (!(ch[i].ref & kLeafRef) && ch[i].area() > best) best = ch[i].area(), pick = i;
        if (pick < 0) break;
        Lb4Child sub[2];
        lb_children2(n2, ch[pick].ref, sub);
        ch[pick] = sub[0];
        ch.push_back(sub[1]);
    }
    const uint32_t me = (uint32_t)(n4.size() / 7u);
    n4.resize(n4.size() + 7u);
    levels = 1u;
    uint32_t refs[4];
    for (uint32_t i = 0; i < 4u; ++i) {
        if (i >= ch.size()) {
            refs[i] = kNoRef;
        } else if (ch[i].ref & kLeafRef) {
            refs[i] = ch[i].ref;
        } else {
            uint32_t lv = 0;
            refs[i] = lb_collapse4(n2, ch[i].ref, n4, lv);
            levels = std::max(levels, 1u + lv);
        }
    }
    float v[7][4];
    for (uint32_t i = 0; i < 4u; ++i) {
        const bool has = i < ch.size();
        for (int a = 0; a < 3; ++a) {
            v[2 * a][i] = has ? ch[i].lo[a] : 0.0f;
            v[2 * a + 1][i] = has ? ch[i].hi[a] : 0.0f;
        }
        memcpy(&v[6][i], &refs[i], sizeof(float));  // full refs here; 16-bit after lb_bfs4
    }
    for (int k = 0; k < 7; ++k) n4[7u * me + (uint32_t)k] = make_float4(v[k][0], v[k][1], v[k][2], v[k][3]);
    return me;
}
// breadth-first order of a 4-wide tree rooted at node `root` (the root becomes 0)
static void lb_bfs4(std::vector<float4>& n4, uint32_t root) {
    const uint32_t nn = (uint32_t)(n4.size() / 7u);
    auto ref_at = [&](uint32_t n, int c) {
        uint32_t u;
        memcpy(&u, reinterpret_cast<const float*>(&n4[7u * n + 6u]) + c, sizeof u);
        return u;
    };
    std::vector<uint32_t> order, newidx(nn, 0u);
    order.push_back(root);
    for (size_t h = 0; h < order.size(); ++h)
        for (int c = 0; c < 4; ++c) {
            const uint32_t r = ref_at(order[h], c);
            if (r != kNoRef && !(r & kLeafRef)) order.push_back(r);
        }
    for (uint32_t i = 0; i < nn; ++i) newidx[order[i]] = i;
    std::vector<float4> bfs(n4.size());
    for (uint32_t i = 0; i < nn; ++i) {
        for (int k = 0; k < 7; ++k) bfs[7u * i + (uint32_t)k] = n4[7u * order[i] + (uint32_t)k];
        for (int c = 0; c < 4; ++c) {
            uint32_t r = ref_at(order[i], c);
            if (r != kNoRef && !(r & kLeafRef)) r = newidx[r];
            // 16-bit form (the kernel's sort keys and stack entries; refs < 2^15 checked by the caller)
            r = r == kNoRef ? kNoRef16 : ((r & 0x7fffu) | ((r >> 16) & 0x8000u));
            memcpy(reinterpret_cast<float*>(&bfs[7u * i + 6u]) + c, &r, sizeof r);
        }
    }
    n4.swap(bfs);
}

// ---- union of conjunctions (the lane tracer's term mode) ----
// A program whose root is a union of TERMS, each a conjunction of at most
// kTermLits literals (a primitive or its complement: a DIFF of one primitive by
// another is a AND NOT b) and each primitive in one term: csg256 / csg512
// balanced's pairs, csg32's box minus sphere.  Along a ray, a term's value can
// only change at an event of its own literals, so the root (a union) changes
// exactly when the count of true terms crosses 0 -- the union-only sweep with
// term transitions in place of primitive events (LaneTracer::visit_term).
// Literal encoding: ordinal | kLitNeg for a complement.

struct TermSub {
    int kind;  // 0 conjunction (lits), 1 union of conjunctions (terms), 2 not expressible
    std::vector<uint32_t> lits;
    std::vector<std::vector<uint32_t>> terms;
};

// The root's terms, or false when the program is not such a union.
static bool extract_terms(WoRec const* prog, uint32_t n_recs, uint32_t n_prims,
                          std::vector<std::vector<uint32_t>>& terms) {
    std::vector<TermSub> st;
    auto bad = []() { TermSub t; t.kind = 2; return t; };
    auto as_terms = [](const TermSub& x) {
        return x.kind == 0 ? std::vector<std::vector<uint32_t>>{x.lits} : x.terms;
    };
    // NOT of a union of single positive literals (a difference's right operand)
    auto negated = [](const TermSub& x, std::vector<uint32_t>& out) {
        if (x.kind == 0) {
            if (x.lits.size() != 1u || (x.lits[0] & kLitNeg)) return false;
            out.push_back(x.lits[0] | kLitNeg);
            return true;
        }
        if (x.kind != 1) return false;
        for (const auto& t : x.terms) {
            if (t.size() != 1u || (t[0] & kLitNeg)) return false;
            out.push_back(t[0] | kLitNeg);
        }
        return true;
    };
    for (uint32_t pc = 0; pc < n_recs;) {
        const WoRec& r = prog[pc];
        if (r.op == WO_OP_PRIM) {
            TermSub t;
            t.kind = 0;
            t.lits.push_back(r.u1);
            st.push_back(t);
            pc += 1u + r.u0;
            continue;
        }
        ++pc;
        if (r.op == WO_OP_BOUND) continue;  // a culling hint: evaluators may ignore it
        if (st.size() < 2u) return false;
        TermSub b = st.back();
        st.pop_back();
        TermSub a = st.back();
        st.pop_back();
        TermSub out = bad();
        if (a.kind != 2 && b.kind != 2) {
            if (r.op == WO_OP_UNION) {
                out.kind = 1;
                out.terms = as_terms(a);
                const auto tb = as_terms(b);
                out.terms.insert(out.terms.end(), tb.begin(), tb.end());
            } else if (r.op == WO_OP_INTER && a.kind == 0 && b.kind == 0) {
                out.kind = 0;
                out.lits = a.lits;
                out.lits.insert(out.lits.end(), b.lits.begin(), b.lits.end());
            } else if ((r.op == WO_OP_DIFF || r.op == WO_OP_RDIFF)) {
                const TermSub& keep = r.op == WO_OP_DIFF ? a : b;  // DIFF: a AND NOT b; RDIFF: b AND NOT a
                const TermSub& sub = r.op == WO_OP_DIFF ? b : a;
                std::vector<uint32_t> neg;
                if (keep.kind == 0 && negated(sub, neg)) {
                    out.kind = 0;
                    out.lits = keep.lits;
                    out.lits.insert(out.lits.end(), neg.begin(), neg.end());
                }
            }
        }
        st.push_back(out);
    }
    if (st.size() != 1u || st[0].kind == 2) return false;
    terms = as_terms(st[0]);
    std::vector<uint8_t> seen(n_prims, 0);
    for (const auto& t : terms) {
        if (t.empty() || t.size() > kTermLits) return false;
        for (uint32_t l : t) {
            const uint32_t o = l & ~kLitNeg;
            if (o >= n_prims || seen[o]) return false;  // one term per primitive
            seen[o] = 1;
        }
    }
    return true;
}

static uint32_t lb_node_f4(const WoDev* dev) { return dev->lb_wide ? 7u : 4u; }

static int build_lbvh(WoDev* dev, WoRec const* prog, uint32_t n_recs, uint32_t n_prims, WoMaterial const* mats,
                      uint32_t n_mats, char* err, size_t errlen) {
    dev->lb_nodes = dev->lb_always = dev->lb_top = dev->lb_depth = 0;
    dev->lb_root = kNoRef;
    dev->lb_nprims = n_prims;
    dev->lb_spheres_only = false;
    dev->lb_stack16 = false;
    dev->lb_wide = false;
    dev->lb_terms = 0;
    dev->lb_general = false;
    // not union-only: the BVH over the root's terms, when the root is a union of
    // small conjunctions (extract_terms); else over the primitives of the general tree,
    // whose value the lanes keep (gpar / gnode: the tree over the primitives, BOUND
    // records dropped; refs [0, P) the primitives' leaves, [P, P + nodes) the binops)
    std::vector<std::vector<uint32_t>> terms;
    std::vector<uint32_t> gpar, gnode;
    uint32_t groot = kNoRef;
    if (!dev->union_only && !extract_terms(prog, n_recs, n_prims, terms)) {
        if (!n_prims) return 0;
        gpar.assign(n_prims, kNoRef);
        std::vector<uint32_t> st;
        for (uint32_t pc = 0; pc < n_recs;) {
            const WoRec& r = prog[pc];
            if (r.op == WO_OP_PRIM) {
                st.push_back(r.u1);
                pc += 1u + r.u0;
                continue;
            }
            ++pc;
            if (r.op == WO_OP_BOUND) continue;
            if (st.size() < 2u) {
                snprintf(err, errlen, "malformed program (binop without operands)");
                return -1;
            }
            const uint32_t b = st.back();
            st.pop_back();
            const uint32_t a = st.back();
            st.pop_back();
            const uint32_t op = r.op == WO_OP_UNION ? 0u : r.op == WO_OP_INTER ? 1u : r.op == WO_OP_DIFF ? 2u : 3u;
            const uint32_t n = n_prims + (uint32_t)gnode.size();
            gnode.push_back(a | (b << kGRefBits) | (op << 30));
            gpar.push_back(kNoRef);
            gpar[a] = n;
            gpar[b] = n;
            st.push_back(n);
        }
        if (st.size() != 1u || gpar.size() > kGRefMask) return 0;  // (refs beyond 15 bits: no lane form)
        groot = st[0];
        dev->lb_general = true;
    }
    std::vector<LbPrim> prims;
    std::vector<uint32_t> always;
    std::vector<float4> geo(n_prims, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    std::vector<uint32_t> kind(n_prims, 0u);
    std::vector<uint32_t> pc_of(n_prims, 0u);
    for (uint32_t pc = 0; pc < n_recs;) {
        const WoRec& r = prog[pc];
        if (r.op != WO_OP_PRIM) {
            ++pc;
            continue;
        }
        const uint32_t ord = r.u1;
        if (ord >= n_prims) {
            snprintf(err, errlen, "primitive ordinal out of range");
            return -1;
        }
        const WoRec& L = prog[pc + 1u];
        if (r.u0 == 1u && L.op == WO_LEAF_SPHERE) {
            geo[ord] = make_float4(L.f[0], L.f[1], L.f[2], L.f[3]);
            kind[ord] = 1u;
        }
        pc_of[ord] = pc;
        if (!terms.empty()) {  // boxes per term below
            pc += 1u + r.u0;
            continue;
        }
        LbPrim p;
        p.ord = ord;
        if (prim_aabb(prog, pc, p.lo, p.hi)) {
            for (int a = 0; a < 3; ++a) {
                const double m = 1e-4 * (fabs(p.lo[a]) + fabs(p.hi[a]) + (p.hi[a] - p.lo[a])) + 1e-5;
                p.lo[a] -= m;
                p.hi[a] += m;
                p.c[a] = 0.5 * (p.lo[a] + p.hi[a]);
            }
            prims.push_back(p);
        } else {
            always.push_back(ord);
        }
        pc += 1u + r.u0;
    }
    // term mode: a term's box is the meet of its positive literals' boxes (its
    // value, and every change of it, lies inside each of them); a term with no
    // bounded positive literal goes to the always list
    std::vector<float4> term_recs;
    auto bits_f = [](uint32_t u) {
        float f;
        memcpy(&f, &u, sizeof f);
        return f;
    };
    for (uint32_t ti = 0; ti < (uint32_t)terms.size(); ++ti) {
        const auto& t = terms[ti];
        // inline geometry: a literal that is one sphere, or two sphere members
        float4 rec[kTermRecF4];
        for (uint32_t k = 0; k < kTermRecF4; ++k) rec[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        uint32_t kinds = 0;
        for (uint32_t x = 0; x < (uint32_t)t.size(); ++x) {
            const uint32_t pc = pc_of[t[x] & ~kLitNeg];
            const uint32_t nm = prog[pc].u0;
            bool spheres = nm >= 1u && nm <= 2u;
            for (uint32_t m = 0; m < nm && spheres; ++m) spheres = prog[pc + 1u + m].op == WO_LEAF_SPHERE;
            if (!spheres) continue;
            kinds |= (nm == 1u ? kTermLitSphere : kTermLitSphere2) << (2u * x);
            for (uint32_t m = 0; m < 2u; ++m) {  // a single sphere repeats as member 1 (a no-op meet)
                const WoRec& L = prog[pc + 1u + (m < nm ? m : 0u)];
                rec[1u + 2u * x + m] = make_float4(L.f[0], L.f[1], L.f[2], L.f[3]);
            }
        }
        if (t.size() == 1u) kinds |= kTermLitSphere << 2u;  // no second literal: a dummy sphere, masked out
        rec[0] = make_float4(bits_f(t[0]), bits_f(t.size() > 1u ? t[1] : kNoLit), bits_f(kinds), 0.0f);
        term_recs.insert(term_recs.end(), rec, rec + kTermRecF4);
        LbPrim p;
        p.ord = ti;
        bool bounded = false;
        for (int a = 0; a < 3; ++a) {
            p.lo[a] = -INFINITY;
            p.hi[a] = INFINITY;
        }
        for (uint32_t l : t) {
            if (l & kLitNeg) continue;
            double lo[3], hi[3];
            if (!prim_aabb(prog, pc_of[l], lo, hi)) continue;
            bounded = true;
            for (int a = 0; a < 3; ++a) {
                p.lo[a] = fmax(p.lo[a], lo[a]);
                p.hi[a] = fmin(p.hi[a], hi[a]);
            }
        }
        for (int a = 0; a < 3 && bounded; ++a)
            if (p.lo[a] > p.hi[a]) p.hi[a] = p.lo[a];  // an empty meet: a point box (never empty arithmetic)
        if (!bounded) {
            always.push_back(ti);
            continue;
        }
        for (int a = 0; a < 3; ++a) {
            const double m = 1e-4 * (fabs(p.lo[a]) + fabs(p.hi[a]) + (p.hi[a] - p.lo[a])) + 1e-5;
            p.lo[a] -= m;
            p.hi[a] += m;
            p.c[a] = 0.5 * (p.lo[a] + p.hi[a]);
        }
        prims.push_back(p);
    }
    // General tree: each primitive's relevance box, the meet of the bounds of the
    // operands that gate it -- an intersection's other operand, a difference's
    // left one for its right one -- along its path to the root (outside it the
    // primitive cannot change the root).  The walk's leaf box becomes the meet of
    // the primitive's box with it (twice the slack, so the clip's ends lie inside
    // with room), a primitive whose meet is empty even with the slack never matters
    // and leaves the walk, and an unbounded primitive with a bounded relevance box
    // joins the BVH.  visit_leaf clips the primitive's interval to the box's span.
    std::vector<float4> gclip;
    if (dev->lb_general) {
        typedef std::array<double, 6> Box;  // lo xyz, hi xyz
        const Box inf_box = {-INFINITY, -INFINITY, -INFINITY, INFINITY, INFINITY, INFINITY};
        auto meet = [](const Box& x, const Box& y) {
            Box m;
            for (int a = 0; a < 3; ++a) {
                m[a] = fmax(x[a], y[a]);
                m[3 + a] = fmin(x[3 + a], y[3 + a]);
            }
            return m;
        };
        auto hull = [](const Box& x, const Box& y) {
            Box h;
            for (int a = 0; a < 3; ++a) {
                h[a] = fmin(x[a], y[a]);
                h[3 + a] = fmax(x[3 + a], y[3 + a]);
            }
            return h;
        };
        auto slacked = [](Box x, double k) {
            for (int a = 0; a < 3; ++a) {
                if (!std::isfinite(x[a]) || !std::isfinite(x[3 + a])) continue;
                const double m = k * (1e-4 * (fabs(x[a]) + fabs(x[3 + a]) + fabs(x[3 + a] - x[a])) + 1e-5);
                x[a] -= m;
                x[3 + a] += m;
            }
            return x;
        };
        const uint32_t nref = (uint32_t)gpar.size();
        std::vector<Box> bnd(nref, inf_box), con(nref, inf_box);
        for (uint32_t ord = 0; ord < n_prims; ++ord) {
            double lo[3], hi[3];
            if (prim_aabb(prog, pc_of[ord], lo, hi)) bnd[ord] = {lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]};
        }
        for (uint32_t i = 0; i < (uint32_t)gnode.size(); ++i) {  // operands before their node
            const uint32_t nd = gnode[i], a = nd & kGRefMask, b = (nd >> kGRefBits) & kGRefMask, op = nd >> 30;
            bnd[n_prims + i] = op == 0u ? hull(bnd[a], bnd[b]) : op == 1u ? meet(bnd[a], bnd[b]) : op == 2u ? bnd[a] : bnd[b];
        }
        for (uint32_t i = (uint32_t)gnode.size(); i-- > 0;) {  // a node before its operands
            const uint32_t nd = gnode[i], a = nd & kGRefMask, b = (nd >> kGRefBits) & kGRefMask, op = nd >> 30;
            const Box& c = con[n_prims + i];
            con[a] = op == 1u ? meet(c, bnd[b]) : op == 3u ? meet(c, bnd[b]) : c;  // b AND NOT a: a gated by b
            con[b] = op == 1u || op == 2u ? meet(c, bnd[a]) : c;                    // a AND NOT b: b gated by a
        }
        gclip.assign(2u * n_prims, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
        std::vector<LbPrim> kept;
        std::vector<uint32_t> alw;
        size_t clipped = 0, dropped = 0;
        for (uint32_t ord = 0; ord < n_prims; ++ord) {
            const Box& c = con[ord];
            bool bounded = false;
            for (int a = 0; a < 6; ++a) bounded = bounded || std::isfinite(c[a]);
            if (bounded) {
                const Box cs = slacked(c, 1.0);
                auto fl = [](double v) { return (float)fmax(-1e30, fmin(1e30, v)); };
                gclip[2u * ord] = make_float4(fl(cs[0]), fl(cs[1]), fl(cs[2]), 1.0f);  // w != 0: clip
                gclip[2u * ord + 1u] = make_float4(fl(cs[3]), fl(cs[4]), fl(cs[5]), 0.0f);
                ++clipped;
            }
            const Box m = meet(slacked(bnd[ord], 2.0), slacked(c, 2.0));
            bool empty = false, finite = true;
            for (int a = 0; a < 3; ++a) {
                empty = empty || m[a] > m[3 + a];
                finite = finite && std::isfinite(m[a]) && std::isfinite(m[3 + a]);
            }
            if (empty) {
                ++dropped;
                continue;  // never matters: its bit stays 0
            }
            if (!finite) {
                alw.push_back(ord);
                continue;
            }
            LbPrim p;
            p.ord = ord;
            for (int a = 0; a < 3; ++a) {
                p.lo[a] = m[a];
                p.hi[a] = m[3 + a];
                p.c[a] = 0.5 * (p.lo[a] + p.hi[a]);
            }
            kept.push_back(p);
        }
        prims.swap(kept);
        always.swap(alw);
        if (!clipped) gclip.clear();
        (void)dropped;
    }
    if (!prims.empty()) {
        std::vector<double> diag(prims.size());
        for (size_t i = 0; i < prims.size(); ++i) {
            double s = 0.0;
            for (int a = 0; a < 3; ++a) s += (prims[i].hi[a] - prims[i].lo[a]) * (prims[i].hi[a] - prims[i].lo[a]);
            diag[i] = sqrt(s);
        }
        std::vector<double> sorted = diag;
        std::nth_element(sorted.begin(), sorted.begin() + sorted.size() / 2, sorted.end());
        const double med = sorted[sorted.size() / 2];
        std::vector<LbPrim> kept;
        for (size_t i = 0; i < prims.size(); ++i) {
            if (prims.size() > 4u && diag[i] > 16.0 * med)
                always.push_back(prims[i].ord);
            else
                kept.push_back(prims[i]);
        }
        prims.swap(kept);
    }
    std::vector<float4> nodes;
    if (ceil_log2((uint32_t)prims.size()) > kLaneDepthMax) {  // > 2^24 primitives (launches allow 2^20)
        snprintf(err, errlen, "too many primitives for the lane BVH");
        return -1;
    }
    if (!prims.empty()) {
        // levels: SAH's freedom over the balanced tree's log2(n), within the stack's limit
        // (the balanced tree, levels = log2(n): RTIOW cover 12.20 ms against 11.60)
        uint32_t levels = ceil_log2((uint32_t)prims.size()) + 6u;
        if (levels > kLaneDepthMax) levels = kLaneDepthMax;
        LbBox root_box;
        dev->lb_root = lb_build(prims, 0u, (uint32_t)prims.size(), levels, nodes, root_box, dev->lb_depth);
        // 4-wide nodes: refs must fit the 16-bit stack entries.  For term mode over 256
        // terms (csg512_balanced, resumable walks: 50.1 -> 44.7 ms over the binary tree;
        // non-resumable 82.0 -> 70.5); neutral on csg256 balanced's 65 terms, 16.4 / 16.5
        // ms; slower on csg32's 14, 8.9 -> 9.6, and on the RTIOW cover's spheres, 11.7 ->
        // 13.7
        const bool want_wide = terms.size() > 256u;
        const uint32_t nrefs = terms.empty() ? n_prims : (uint32_t)terms.size();
        if (want_wide && !(dev->lb_root & kLeafRef) && nrefs < 0x8000u) {
            std::vector<float4> n4;
            uint32_t lv4 = 0;
            const uint32_t r4 = lb_collapse4(nodes, dev->lb_root, n4, lv4);
            if (n4.size() / 7u < 0x8000u) {
                lb_bfs4(n4, r4);
                nodes.swap(n4);
                dev->lb_root = 0u;
                dev->lb_wide = true;
                dev->lb_depth = 3u * lv4;  // stack entries: at most three siblings per level
            }
        }
        // breadth-first node order: the top levels are then nodes [0, k), the ones
        // every walk visits first, and they are staged in LDS (lb_top)
        if (!dev->lb_wide && !(dev->lb_root & kLeafRef)) {
            const uint32_t nn = (uint32_t)(nodes.size() / 4u);
            auto ref_at = [&](uint32_t n, int c) {
                uint32_t u;
                memcpy(&u, &nodes[4u * n + (uint32_t)c].w, sizeof u);
                return u;
            };
            std::vector<uint32_t> order, newidx(nn, 0u);
            order.reserve(nn);
            order.push_back(dev->lb_root);
            for (size_t h = 0; h < order.size(); ++h)
                for (int c = 0; c < 2; ++c) {
                    const uint32_t r = ref_at(order[h], c);
                    if (!(r & kLeafRef)) order.push_back(r);
                }
            for (uint32_t i = 0; i < nn; ++i) newidx[order[i]] = i;
            std::vector<float4> bfs(nodes.size());
            for (uint32_t i = 0; i < nn; ++i) {
                for (int k = 0; k < 4; ++k) bfs[4u * i + (uint32_t)k] = nodes[4u * order[i] + (uint32_t)k];
                for (int c = 0; c < 2; ++c) {
                    uint32_t r = ref_at(order[i], c);
                    if (!(r & kLeafRef)) r = newidx[r];
                    memcpy(&bfs[4u * i + (uint32_t)c].w, &r, sizeof r);
                }
            }
            nodes.swap(bfs);
            dev->lb_root = 0u;
        }
    }
    const uint32_t node_f4 = lb_node_f4(dev);
    dev->lb_nodes = (uint32_t)(nodes.size() / node_f4);
    dev->lb_always = (uint32_t)always.size();
    {
        // 16-bit stack entries for 4-wide nodes and the general tree (its bits need the
        // LDS; binary trees otherwise: 32-bit, RTIOW cover 11.60 ms against 11.76 with
        // 16-bit entries and more top nodes)
        dev->lb_stack16 = dev->lb_wide || dev->lb_general;
        if (dev->lb_general && (dev->lb_nodes >= 0x8000u || n_prims >= 0x8000u)) {
            dev->lb_general = false;  // refs beyond the 16-bit stack entries: no lane form
            return 0;
        }
        // the top nodes fill what the stacks leave of kLanesBvhLds (8 workgroups per CU)
        const size_t stacks =
            ((((size_t)dev->lb_depth * kBlock * (dev->lb_stack16 ? 2u : 4u)) + 15u) & ~(size_t)15u);
        const size_t used = stacks + (dev->lb_general ? (size_t)((gpar.size() + 31u) / 32u) * kBlock * 4u : 0u);
        // (the kernels with camera-ray waves give the ring's LDS: LaneTracer::kCamMode)
        const size_t budget = kLanesBvhLds - (dev->lb_wide || dev->lb_general ? 0u : kCamRingLds);
        const uint32_t top = used < budget ? (uint32_t)((budget - used) / (node_f4 * sizeof(float4))) : 0u;
        dev->lb_top = top < dev->lb_nodes ? top : dev->lb_nodes;
    }
    dev->lb_spheres_only = terms.empty() && !dev->lb_general &&
                           std::all_of(kind.begin(), kind.end(), [](uint32_t k) { return k != 0u; });
    dev->lb_terms = (uint32_t)terms.size();
    const size_t f4 = nodes.size() + n_prims;
    // ... | kind per ordinal | always list | (term mode) kTermRecF4 float4 per term, 16-byte aligned
    size_t words = (size_t)n_prims + always.size();
    words = (words + 3u) & ~(size_t)3u;
    const size_t term_off = f4 * sizeof(float4) + words * sizeof(uint32_t);
    dev->lb_term_off = (uint32_t)(term_off / sizeof(uint32_t));
    // single-sphere scenes: each ordinal's leaf record and its material (2 x 32 B), so
    // a hit's shading reads them in two independent loads instead of the ordinal ->
    // pc -> record -> material chain (hit_leaf, hit_material)
    static_assert(sizeof(WoRec) == 32 && sizeof(WoMaterial) == 32, "leaf table entries are 2 x 32 bytes");
    const size_t leaf_off = term_off + term_recs.size() * sizeof(float4);
    dev->lb_leaf_off = dev->lb_spheres_only ? (uint32_t)(leaf_off / sizeof(uint32_t)) : 0u;
    const size_t gpar_off = leaf_off + (dev->lb_spheres_only ? (size_t)n_prims * 2u * sizeof(WoRec) : 0u);
    const size_t gnode_off = gpar_off + gpar.size() * sizeof(uint32_t);
    const size_t gclip_off = (gnode_off + gnode.size() * sizeof(uint32_t) + 15u) & ~(size_t)15u;
    const size_t bytes = gclip_off + gclip.size() * sizeof(float4);
    dev->lb_gpar_off = (uint32_t)(gpar_off / sizeof(uint32_t));
    dev->lb_gnode_off = (uint32_t)(gnode_off / sizeof(uint32_t));
    dev->lb_gclip_off = gclip.empty() ? 0u : (uint32_t)(gclip_off / sizeof(uint32_t));
    dev->lb_gP = n_prims;
    dev->lb_gwords = (uint32_t)((gpar.size() + 31u) / 32u);
    dev->lb_groot = groot;
    if (ensure_buffer(&dev->d_lbvh, &dev->lbvh_cap, bytes, err, errlen)) return -1;
    std::vector<char> blob(bytes);
    if (!gpar.empty()) memcpy(blob.data() + gpar_off, gpar.data(), gpar.size() * sizeof(uint32_t));
    if (!gnode.empty()) memcpy(blob.data() + gnode_off, gnode.data(), gnode.size() * sizeof(uint32_t));
    if (!gclip.empty()) memcpy(blob.data() + gclip_off, gclip.data(), gclip.size() * sizeof(float4));
    if (dev->lb_spheres_only)
        for (uint32_t ord = 0; ord < n_prims; ++ord) {
            const WoRec& L = prog[pc_of[ord] + 1u];
            char* e = blob.data() + leaf_off + (size_t)ord * 2u * sizeof(WoRec);
            memcpy(e, &L, sizeof(WoRec));
            if (L.u0 < n_mats) memcpy(e + sizeof(WoRec), &mats[L.u0], sizeof(WoMaterial));
        }
    memcpy(blob.data(), nodes.data(), nodes.size() * sizeof(float4));
    memcpy(blob.data() + nodes.size() * sizeof(float4), geo.data(), n_prims * sizeof(float4));
    memcpy(blob.data() + f4 * sizeof(float4), kind.data(), n_prims * sizeof(uint32_t));
    memcpy(blob.data() + f4 * sizeof(float4) + n_prims * sizeof(uint32_t), always.data(),
           always.size() * sizeof(uint32_t));
    if (!term_recs.empty()) memcpy(blob.data() + term_off, term_recs.data(), term_recs.size() * sizeof(float4));
    hipError_t e = hipMemcpy(dev->d_lbvh, blob.data(), bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipMemcpy(lane BVH)", e);
        return -1;
    }
    return 0;
}

static LaneBvh lane_bvh(const WoDev* dev) {
    LaneBvh b;
    const uint32_t node_f4 = lb_node_f4(dev);
    b.nodes = dev->d_lbvh;
    b.geo = dev->d_lbvh + node_f4 * dev->lb_nodes;
    b.kind = reinterpret_cast<const uint32_t*>(dev->d_lbvh + node_f4 * dev->lb_nodes + dev->lb_nprims);
    b.nalways = dev->lb_always;
    b.root = dev->lb_root;
    b.nprims = dev->lb_nprims;
    b.ntop = dev->lb_top;
    b.depth = dev->lb_depth;
    // csg512_balanced: 60.4 / 57.6 / 57.2 / 58.1 / 59.2 ms at 8 / 16 / 24 / 32 / 40;
    // WOLOLO_DYN_WALKERS (measurement) overrides
    static const uint32_t walkers = [] {
        const char* w = getenv("WOLOLO_DYN_WALKERS");
        return w && *w ? (uint32_t)atoi(w) : 24u;
    }();
    b.dyn_walkers = walkers;
    b.trec = dev->lb_terms ? reinterpret_cast<const float4*>(reinterpret_cast<const uint32_t*>(dev->d_lbvh) +
                                                            dev->lb_term_off)
                           : nullptr;
    b.leaves = dev->lb_leaf_off ? reinterpret_cast<const WoRec*>(reinterpret_cast<const uint32_t*>(dev->d_lbvh) +
                                                                dev->lb_leaf_off)
                                : nullptr;
    b.gpar = reinterpret_cast<const uint32_t*>(dev->d_lbvh) + dev->lb_gpar_off;
    b.gnode = reinterpret_cast<const uint32_t*>(dev->d_lbvh) + dev->lb_gnode_off;
    b.gclip = dev->lb_gclip_off ? reinterpret_cast<const float4*>(reinterpret_cast<const uint32_t*>(dev->d_lbvh) +
                                                                 dev->lb_gclip_off)
                                : nullptr;
    b.gP = dev->lb_gP;
    b.gwords = dev->lb_gwords;
    b.groot = dev->lb_groot;
    return b;
}

extern "C" int wo_dev_upload_scene(WoDev* dev, WoRec const* prog, uint32_t n_recs, uint32_t n_prims,
                                   WoMaterial const* mats, uint32_t n_mats, char* err, size_t errlen) {
    hipError_t e = hipSetDevice(dev->device);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipSetDevice", e);
        return -1;
    }
    // Kernels of the previous scene may still run on any stream of the device
    // (the frame pipeline's, or a caller's stream for render_rows_device): the
    // buffers below are overwritten (or reallocated) in place and the JIT module
    // replaced next, so the whole device drains first.  Scene changes are rare.
    e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        set_err(err, errlen, "hipDeviceSynchronize (before scene upload)", e);
        return -1;
    }
    if (ensure_buffer(&dev->d_prog, &dev->prog_cap, (size_t)n_recs * sizeof(WoRec), err, errlen)) return -1;
    if (ensure_buffer(&dev->d_mats, &dev->mats_cap, (size_t)n_mats * sizeof(WoMaterial), err, errlen)) return -1;
    if (n_recs) {
        e = hipMemcpy(dev->d_prog, prog, (size_t)n_recs * sizeof(WoRec), hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            set_err(err, errlen, "hipMemcpy(program)", e);
            return -1;
        }
    }
    if (n_mats) {
        e = hipMemcpy(dev->d_mats, mats, (size_t)n_mats * sizeof(WoMaterial), hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            set_err(err, errlen, "hipMemcpy(materials)", e);
            return -1;
        }
    }
    dev->n_recs = n_recs;
    dev->n_prims = n_prims;
    dev->n_mats = n_mats;
    if (scene_maps(dev, prog, n_recs, n_prims, err, errlen)) return -1;
    return build_lbvh(dev, prog, n_recs, n_prims, mats, n_mats, err, errlen);
}

// ---- scene-specialised kernels (hiprtc) ----

// Process-wide cache of compiled code objects (the same scene compiled once per
// process, loaded on every rank), in front of the on-disk cache (jit_cache.c)
// shared by processes.  Bounded: the least recently used entries go beyond
// kJitCacheEntries (an interactive session that edits the scene would otherwise
// keep every version's object, megabytes each; the disk cache still has them).
struct JitEntry {
    std::vector<char> code;
    uint64_t used;
};
static const size_t kJitCacheEntries = 8;
// The process cache and its lock live on the heap and are never destroyed: a
// background compile still running when the process exits (a renderer never
// closed) then touches no destroyed static.
static std::mutex& g_jit_mu = *new std::mutex;
static uint64_t g_jit_tick;
static std::unordered_map<std::string, JitEntry>& jit_cache() {
    static auto* m = new std::unordered_map<std::string, JitEntry>;
    return *m;
}
static void jit_cache_put(const std::string& key, const std::vector<char>& code) {  // g_jit_mu held
    auto& m = jit_cache();
    m[key] = JitEntry{code, ++g_jit_tick};
    while (m.size() > kJitCacheEntries) {
        auto old = m.begin();
        for (auto it = m.begin(); it != m.end(); ++it)
            if (it->second.used < old->second.used) old = it;
        m.erase(old);
    }
}

// Extra hiprtc options from WOLOLO_JIT_FLAGS (space separated), e.g.
// "-DWO_WINDOW=2 -DWO_JIT_MIN_WAVES=4" -- a tuning knob; part of the cache key.
static std::vector<std::string> jit_extra_flags() {
    std::vector<std::string> out;
    const char* e = getenv("WOLOLO_JIT_FLAGS");
    if (!e) return out;
    std::string s(e), cur;
    for (char c : s) {
        if (c == ' ') {
            if (!cur.empty()) out.push_back(cur);
            cur.clear();
        } else {
            cur.push_back(c);
        }
    }
    if (!cur.empty()) out.push_back(cur);
    return out;
}

// `count`: the counting variant (executed-work counters, wo_dev_count_work)
static std::vector<std::string> jit_options(const std::string& arch, bool count) {
    // no SLP vectorisation: its packed fp32 pairs need register moves to form and
    // shorten no dependent chain (csg32 4.14 -> 4.05 ms, csg256 balanced 12.50 -> 12.08);
    // WOLOLO_JIT_FLAGS=-fslp-vectorize turns it back on
    std::vector<std::string> opts = {"--offload-arch=" + arch, "-O3", "-ffp-contract=off", "-std=c++17",
                                     "-fno-slp-vectorize"};
    for (const std::string& f : jit_extra_flags()) opts.push_back(f);
    if (count) opts.push_back("-DWO_COUNT_WORK=1");
    return opts;
}

// The compiler process (wo_jitc, next to this library): used when the hiprtc that
// serves this process is not the system ROCm's -- a process that imported torch first
// runs the library on torch's bundled HIP runtime, hiprtc and comgr (the sonames are
// shared), and that older compiler spilled csg32_nested's kernel (12 B per lane, 3 %
// slower).  wo_jitc links only the system hiprtc, in a
// process of its own.  "" = compile in this process (the system hiprtc serves it, the
// helper is missing, or WOLOLO_JITC=0).
extern "C" char** environ;
static const std::string& jitc_path() {
    static const std::string path = []() -> std::string {
        const char* env = getenv("WOLOLO_JITC");
        if (env && *env == '0') return std::string();
        Dl_info di;
        char rp[PATH_MAX], rr[PATH_MAX];
        const char* root = getenv("ROCM_PATH");
        if (dladdr((void*)&hiprtcCompileProgram, &di) && di.dli_fname && realpath(di.dli_fname, rp) &&
            realpath(root && *root ? root : "/opt/rocm", rr) && strncmp(rp, rr, strlen(rr)) == 0)
            return std::string();  // the system hiprtc already
        if (!dladdr((void*)&jitc_path, &di) || !di.dli_fname) return std::string();
        std::string lib(di.dli_fname);
        const size_t slash = lib.rfind('/');
        std::string p = (slash == std::string::npos ? std::string(".") : lib.substr(0, slash)) + "/wo_jitc";
        return access(p.c_str(), X_OK) == 0 ? p : std::string();
    }();
    return path;
}

// One compile through wo_jitc: the source and the code object through a private
// temporary directory.  False: no object (the caller compiles in this process).
static bool jitc_compile(const char* src, const std::vector<std::string>& opts, std::vector<char>& code) {
    const char* td = getenv("TMPDIR");
    std::string dir = std::string(td && *td ? td : "/tmp") + "/wojitc.XXXXXX";
    if (!mkdtemp(&dir[0])) return false;
    const std::string in = dir + "/k.hip", out = dir + "/k.co";
    bool ok = false;
    if (FILE* f = fopen(in.c_str(), "wb")) {
        const size_t n = strlen(src);
        ok = fwrite(src, 1, n, f) == n;
        ok = (fclose(f) == 0) && ok;
    }
    if (ok) {
        std::vector<char*> argv;
        argv.push_back(const_cast<char*>(jitc_path().c_str()));
        argv.push_back(const_cast<char*>(in.c_str()));
        argv.push_back(const_cast<char*>(out.c_str()));
        for (const std::string& o : opts) argv.push_back(const_cast<char*>(o.c_str()));
        argv.push_back(nullptr);
        pid_t pid;
        int st = 0;
        ok = posix_spawn(&pid, jitc_path().c_str(), nullptr, nullptr, argv.data(), environ) == 0 &&
             waitpid(pid, &st, 0) == pid && WIFEXITED(st) && WEXITSTATUS(st) == 0;
    }
    if (ok) {
        ok = false;
        if (FILE* f = fopen(out.c_str(), "rb")) {
            std::vector<char> buf;
            char tmp[65536];
            size_t n;
            while ((n = fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + n);
            fclose(f);
            ok = buf.size() >= 4 && memcmp(buf.data(), "\x7f" "ELF", 4) == 0;
            if (ok) code.swap(buf);
        }
    }
    (void)unlink(in.c_str());
    (void)unlink(out.c_str());
    (void)rmdir(dir.c_str());
    return ok;
}

static int jit_compile(const char* src, const std::string& arch, bool count, std::vector<char>& code, char* err,
                       size_t errlen) {
    if (!jitc_path().empty() && jitc_compile(src, jit_options(arch, count), code)) return 0;
    hiprtcProgram p;
    const char* hdr_src[] = {kEmbed_wo_device_common_h, kEmbed_wo_scene_h};
    const char* hdr_names[] = {"wo_device_common.h", "wololo/wo_scene.h"};
    if (hiprtcCreateProgram(&p, src, "wo_scene_jit.hip", 2, hdr_src, hdr_names) != HIPRTC_SUCCESS) {
        snprintf(err, errlen, "hiprtcCreateProgram failed");
        return -1;
    }
    std::vector<std::string> opt_s = jit_options(arch, count);
    std::vector<const char*> opts;
    for (const std::string& o : opt_s) opts.push_back(o.c_str());
    hiprtcResult rc = hiprtcCompileProgram(p, (int)opts.size(), opts.data());
    if (rc != HIPRTC_SUCCESS) {
        size_t ls = 0;
        hiprtcGetProgramLogSize(p, &ls);
        std::string log(ls + 1, '\0');
        hiprtcGetProgramLog(p, &log[0]);
        snprintf(err, errlen, "hiprtc: %s: %.400s", hiprtcGetErrorString(rc), log.c_str());
        hiprtcDestroyProgram(&p);
        return -1;
    }
    size_t cs = 0;
    hiprtcGetCodeSize(p, &cs);
    code.resize(cs);
    hiprtcGetCode(p, code.data());
    hiprtcDestroyProgram(&p);
    return 0;
}

// SHA-256 over everything the code object depends on: a format tag, the hiprtc
// and HIP runtime versions, the target, the options (WOLOLO_JIT_FLAGS included), the embedded
// headers and the generated source; each part length-prefixed.
static std::string jit_key(const char* src, const std::string& arch, bool count = false) {
    WoSha256 s;
    wo_sha256_init(&s);
    auto part = [&](const char* p, size_t n) {
        const uint64_t len = n;
        wo_sha256_update(&s, &len, sizeof len);
        wo_sha256_update(&s, p, n);
    };
    part("wololo-jit-2", 12);
    // the toolchain: hiprtc's major.minor and the HIP runtime's full version
    // (patch level included: a ROCm update that changes the compiler or the
    // device libraries misses instead of loading a stale object)
    // (queried once: hiprtcVersion waits while another thread's compile holds
    // hiprtc's lock, which stalled draw_frame behind a background compile)
    static const std::array<int, 3> ver = []() {
        int vmaj = 0, vmin = 0, vrt = 0;
        (void)hiprtcVersion(&vmaj, &vmin);
        (void)hipRuntimeGetVersion(&vrt);
        return std::array<int, 3>{vmaj, vmin, vrt};
    }();
    part((const char*)ver.data(), sizeof(int) * ver.size());
    // compiled by wo_jitc (the system hiprtc) rather than the hiprtc serving this process
    if (!jitc_path().empty()) part("wo_jitc", 7);
    part(arch.data(), arch.size());
    for (const std::string& o : jit_options(arch, count)) part(o.data(), o.size());
    part(kEmbed_wo_device_common_h, strlen(kEmbed_wo_device_common_h));
    part(kEmbed_wo_scene_h, strlen(kEmbed_wo_scene_h));
    part(src, strlen(src));
    uint8_t dg[32];
    wo_sha256_final(&s, dg);
    char hex[65];
    wo_sha256_hex(dg, hex);
    return std::string(hex);
}

static int jit_code(const char* src, const std::string& arch, bool count, std::vector<char>& code, std::string& key,
                    int& origin, double& seconds, char* err, size_t errlen) {
    auto t0 = std::chrono::steady_clock::now();
    key = jit_key(src, arch, count);
    {
        std::lock_guard<std::mutex> lock(g_jit_mu);
        auto it = jit_cache().find(key);
        if (it != jit_cache().end()) {
            it->second.used = ++g_jit_tick;
            code = it->second.code;
            origin = 0;
        }
    }
    if (code.empty()) {
        void* buf = nullptr;
        size_t n = 0;
        if (wo_jit_disk_load(key.c_str(), &buf, &n) == 0) {
            code.assign((char*)buf, (char*)buf + n);
            free(buf);
            origin = 1;
        } else {
            if (jit_compile(src, arch, count, code, err, errlen)) return -1;
            origin = 2;
            (void)wo_jit_disk_store(key.c_str(), code.data(), code.size());  // best effort
        }
        std::lock_guard<std::mutex> lock(g_jit_mu);
        jit_cache_put(key, code);
    }
    seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return 0;
}

extern "C" long long wo_jit_code_object(const char* src, const char* arch, int* origin, double* seconds,
                                        char* key_hex, char* err, size_t errlen) {
    std::vector<char> code;
    std::string key;
    int org = -1;
    double sec = 0.0;
    if (jit_code(src, arch ? std::string(arch) : std::string("gfx950"), false, code, key, org, sec, err, errlen))
        return -1;
    if (origin) *origin = org;
    if (seconds) *seconds = sec;
    if (key_hex) snprintf(key_hex, 65, "%s", key.c_str());
    return (long long)code.size();
}

// The group (LDS) and private (scratch per lane) segment sizes of kernel `name` as its
// code object states them: the first two words of its AMDHSA kernel descriptor, the
// symbol `<name>.kd` of the ELF's symbol table.  (hipFuncGetAttribute can answer for
// another loaded module's kernel of the same name -- a second renderer's counting
// variant -- so kernel_info reads the code object itself.)  False if `code` is not
// such an ELF.
static bool kd_segment_sizes(const std::vector<char>& code, const char* name, uint32_t* group, uint32_t* priv) {
    const unsigned char* b = reinterpret_cast<const unsigned char*>(code.data());
    const size_t n = code.size();
    auto rd = [&](size_t off, size_t len, uint64_t* v) {
        if (off > n || len > n - off) return false;
        uint64_t x = 0;
        for (size_t i = 0; i < len; ++i) x |= (uint64_t)b[off + i] << (8u * i);
        *v = x;
        return true;
    };
    if (n < 64 || memcmp(b, "\x7f" "ELF", 4) != 0 || b[4] != 2 || b[5] != 1) return false;  // ELF64, little-endian
    uint64_t shoff, shentsize, shnum;
    if (!rd(0x28, 8, &shoff) || !rd(0x3a, 2, &shentsize) || !rd(0x3c, 2, &shnum) || shentsize < 64) return false;
    auto sh = [&](uint64_t i, size_t field, size_t len, uint64_t* v) { return rd(shoff + i * shentsize + field, len, v); };
    const std::string want = std::string(name) + ".kd";
    for (uint64_t i = 0; i < shnum; ++i) {
        uint64_t type, off, size, link, entsize;
        if (!sh(i, 4, 4, &type) || type != 2u) continue;  // SHT_SYMTAB
        if (!sh(i, 24, 8, &off) || !sh(i, 32, 8, &size) || !sh(i, 40, 4, &link) || !sh(i, 56, 8, &entsize) ||
            entsize < 24)
            return false;
        uint64_t stroff, strsize;
        if (!sh(link, 24, 8, &stroff) || !sh(link, 32, 8, &strsize)) return false;
        for (uint64_t k = 0; k + entsize <= size; k += entsize) {
            uint64_t nm, shndx, value;
            if (!rd(off + k, 4, &nm) || !rd(off + k + 6, 2, &shndx) || !rd(off + k + 8, 8, &value)) return false;
            if (nm >= strsize || stroff + nm + want.size() + 1 > n) continue;
            if (memcmp(b + stroff + nm, want.c_str(), want.size() + 1) != 0) continue;
            uint64_t saddr, soff, g, p;
            if (!sh(shndx, 16, 8, &saddr) || !sh(shndx, 24, 8, &soff) || value < saddr) return false;
            if (!rd(soff + (value - saddr), 4, &g) || !rd(soff + (value - saddr) + 4, 4, &p)) return false;
            *group = (uint32_t)g;
            *priv = (uint32_t)p;
            return true;
        }
    }
    return false;
}

extern "C" int wo_jit_code_resources(const char* src, const char* arch, uint32_t* out, char* err, size_t errlen) {
    std::vector<char> code;
    std::string key;
    int org = -1;
    double sec = 0.0;
    if (!src || !out) {
        snprintf(err, errlen, "no source");
        return -1;
    }
    if (jit_code(src, arch ? std::string(arch) : std::string("gfx950"), false, code, key, org, sec, err, errlen))
        return -1;
    uint32_t group = 0, priv = 0;
    if (!kd_segment_sizes(code, "wo_jit_pathtrace", &group, &priv)) {
        snprintf(err, errlen, "no kernel descriptor for wo_jit_pathtrace in the code object (%zu bytes)", code.size());
        return -1;
    }
    out[0] = priv;
    out[1] = group;
    return 0;
}

static int load_jit_module(const std::vector<char>& code, hipModule_t* mod, hipFunction_t* fn, char* err,
                           size_t errlen) {
    hipError_t e = hipModuleLoadData(mod, code.data());
    if (e != hipSuccess) {
        set_err(err, errlen, "hipModuleLoadData", e);
        return -1;
    }
    e = hipModuleGetFunction(fn, *mod, "wo_jit_pathtrace");
    if (e != hipSuccess) {
        (void)hipModuleUnload(*mod);
        *mod = nullptr;
        set_err(err, errlen, "hipModuleGetFunction", e);
        return -1;
    }
    return 0;
}

extern "C" int wo_dev_set_jit(WoDev* dev, const char* src, char* err, size_t errlen) {
    hipError_t e = hipSetDevice(dev->device);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipSetDevice", e);
        return -1;
    }
    if (dev->count_module) (void)hipModuleUnload(dev->count_module);  // built again on demand
    dev->count_module = nullptr;
    dev->count_fn = nullptr;
    if (!src) {  // disable
        if (dev->jit_module) (void)hipModuleUnload(dev->jit_module);
        dev->jit_module = nullptr;
        dev->jit_fn = nullptr;
        dev->jit_key.clear();
        dev->jit_src.clear();
        dev->jit_origin = -1;
        return 0;
    }
    std::vector<char> code;
    std::string key;
    int origin = -1;
    double sec = 0.0;
    if (dev->jit_fn && dev->jit_key == jit_key(src, dev->arch)) return 0;
    if (jit_code(src, dev->arch, false, code, key, origin, sec, err, errlen)) return -1;
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    if (load_jit_module(code, &mod, &fn, err, errlen)) return -1;
    if (dev->jit_module) (void)hipModuleUnload(dev->jit_module);
    dev->jit_module = mod;
    dev->jit_fn = fn;
    dev->jit_key = key;
    // its resources, read now: once the counting variant (the same kernel name in another
    // module) is loaded, an attribute query of this function returned that one's scratch
    // size -- and a second renderer's counting module can do the same at load time, so
    // the scratch and LDS sizes come from this code object's kernel descriptor
    dev->jit_attr[0] = dev->jit_attr[1] = dev->jit_attr[2] = -1;
    (void)hipFuncGetAttribute(&dev->jit_attr[0], HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, fn);
    (void)hipFuncGetAttribute(&dev->jit_attr[1], HIP_FUNC_ATTRIBUTE_NUM_REGS, fn);
    (void)hipFuncGetAttribute(&dev->jit_attr[2], HIP_FUNC_ATTRIBUTE_SHARED_SIZE_BYTES, fn);
    {
        uint32_t group = 0, priv = 0;
        if (kd_segment_sizes(code, "wo_jit_pathtrace", &group, &priv)) {
            dev->jit_attr[0] = (int)priv;
            dev->jit_attr[2] = (int)group;
        }
    }
    dev->jit_src = src;
    {
        const char* m = strstr(src, "// wo_share_tiles ");
        const int v = m ? atoi(m + strlen("// wo_share_tiles ")) : 0;
        dev->jit_share_tiles = v >= 1 && v <= 64 ? (uint32_t)v : kShareTiles;
    }
    dev->jit_origin = origin;
    dev->jit_compile_sec = sec;
    return 0;
}

// ---- background compiles (wo_dev.h WoJitJob) ----
extern "C" int wo_dev_jit_cached(WoDev* dev, const char* src) {
    const std::string key = jit_key(src, dev->arch);
    {
        std::lock_guard<std::mutex> lock(g_jit_mu);
        if (jit_cache().count(key)) return 1;
    }
    void* buf = nullptr;
    size_t n = 0;
    if (wo_jit_disk_load(key.c_str(), &buf, &n) != 0) return 0;
    std::vector<char> code((char*)buf, (char*)buf + n);
    free(buf);
    std::lock_guard<std::mutex> lock(g_jit_mu);
    jit_cache_put(key, code);
    return 1;
}

struct WoJitJob {
    std::thread th;
    std::atomic<int> done{0};
    int rc = 0;
    std::string src, arch;
    char err[512] = {0};
};

extern "C" WoJitJob* wo_jit_job_start(WoDev* dev, const char* src) {
    WoJitJob* j = new (std::nothrow) WoJitJob();
    if (!j) return nullptr;
    j->src = src;
    j->arch = dev->arch;
    try {
        j->th = std::thread([j]() {
            std::vector<char> code;
            std::string key;
            int origin = -1;
            double sec = 0.0;
            j->rc = jit_code(j->src.c_str(), j->arch, false, code, key, origin, sec, j->err, sizeof j->err);
            j->done.store(1, std::memory_order_release);
        });
    } catch (...) {
        delete j;
        return nullptr;
    }
    return j;
}

extern "C" int wo_jit_job_done(WoJitJob* j) { return j->done.load(std::memory_order_acquire); }

extern "C" const char* wo_jit_job_source(WoJitJob* j) { return j->src.c_str(); }

extern "C" int wo_jit_job_finish(WoJitJob* j, char* err, size_t errlen) {
    if (j->th.joinable()) j->th.join();
    const int rc = j->rc;
    if (rc && err && errlen) snprintf(err, errlen, "%s", j->err);
    delete j;
    return rc;
}

extern "C" int wo_dev_jit_origin(WoDev* dev, double* seconds) {
    if (!dev || !dev->jit_fn) return -1;
    if (seconds) *seconds = dev->jit_compile_sec;
    return dev->jit_origin;
}

extern "C" int wo_dev_lanes_info(WoDev* dev, uint32_t* out) {
    if (!dev) return -1;
    out[0] = dev->lb_nodes;
    out[1] = dev->lb_depth;
    out[2] = dev->lb_top;
    out[3] = dev->lb_always;
    out[4] = dev->last_kind;
    return 0;
}

extern "C" int wo_jit_compile_check(const char* src, const char* arch, char* err, size_t errlen) {
    std::vector<char> code;
    return jit_compile(src, arch ? std::string(arch) : std::string("gfx950"), false, code, err, errlen);
}

extern "C" int wo_dev_jit_active(WoDev* dev) { return dev && dev->jit_fn ? 1 : 0; }
extern "C" int wo_dev_lanes_available(WoDev* dev) {
    return dev && (dev->union_only || dev->lb_terms || dev->lb_general) ? 1 : 0;
}
extern "C" void wo_dev_set_lanes(WoDev* dev, int on) {
    if (dev) dev->lanes_on = on != 0;
}
extern "C" double wo_dev_jit_compile_sec(WoDev* dev) { return dev ? dev->jit_compile_sec : 0.0; }

// Path-tracer launch grid (PathLaunch): big tiles first, then a tail of small
// 4x4 tiles sized to ~3 waves of resident workgroups, which fills the end of
// the frame while the last big tiles finish.  Measured (csg32 1080p64, slowest
// rank, tools/rank_share.py): no tail 5.57 / 2.87 / 1.60 / 1.09 ms at N = 1 / 2 /
// 4 / 8 (8x8 tiles throughout); 3-round tail 5.50 / 2.81 / 1.53 / 0.81 ms.  The big shape is 8x8
// while the frame holds >= 8 rounds of such tiles, else 8x4 (2-round tail), else 4x4
// (plan_tiles); `resident` = workgroups the device holds at once.  Env (measurements):
// WOLOLO_TILE=8x8|8x4|4x4 forces one shape everywhere, with no tail.
// "WxH" with W, H in {1, 2, 4, 8, 16} and W*H <= kTileMaxPix; 0 if not such a shape
static uint32_t shape_of(const char* f) {
    unsigned w = 0, h = 0;
    if (sscanf(f, "%ux%u", &w, &h) != 2) return 0u;
    auto lg = [](unsigned v) -> int { return v == 1u ? 0 : v == 2u ? 1 : v == 4u ? 2 : v == 8u ? 3 : v == 16u ? 4 : -1; };
    const int lw = lg(w), lh = lg(h);
    if (lw < 0 || lh < 0 || w * h > kTileMaxPix) return 0u;
    return (uint32_t)lw | ((uint32_t)lh << 4);
}
static uint32_t tiles_across(uint32_t width, uint32_t shape) { return (width + (1u << (shape & 15u)) - 1u) >> (shape & 15u); }

static PathLaunch plan_tiles(uint32_t width, uint32_t rows, uint32_t resident, uint32_t band_rows,
                             uint32_t want_per_wg) {
    const uint32_t s44 = 2u | (2u << 4);
    PathLaunch g = {};
    // the tail's tiles: 4x4 (2x2 / 4x2 for an 8-rank share's tail: within noise,
    // DESIGN.md §6)
    const uint32_t small = s44;
    g.small_log2 = small;
    g.tiles_x_small = tiles_across(width, small);
    const uint32_t sh = 1u << (small >> 4);
    double tail_rounds = 3.0;  // rounds of resident workgroups in the tail
    const char* f = getenv("WOLOLO_TILE");  // a forced tile shape ("8x4"): the whole frame in it
    uint32_t big = (f && *f) ? shape_of(f) : 0u;
    if (big) {
        tail_rounds = 0.0;
    } else {
        // The largest shape that gives every resident workgroup >= want_per_wg tiles
        // (kShareTiles = 3 for every kernel since round 5, see the end of this note): a
        // workgroup's tiles then average out the costly ones (glass, deep CSG),
        // which otherwise set the end of a short launch.  8x8 keeps a 3-round
        // tail of 4x4 tiles, 8x4 a 2-round one.  Measured (tools/rank_share.py,
        // 1080p64, slowest rank of 4 / 8, ms): csg32 8x8 1.454 / 0.770, 8x4 1.400 /
        // 0.762, 4x4 1.499 / 0.786; csg256 balanced 8x4 4.73 / 3.50, 4x4 4.23 / 2.34;
        // csg256 chain 8x4 7.34 / 5.02, 4x4 7.99 / 4.15; rtiow 8x4 8.47 / 4.30,
        // 4x4 8.27 / 4.37.  One GPU keeps 8x8 (csg32 5.18 vs 5.37 ms at 8x4).  Round 4
        // (tools/root_step.py, N = 8 projection): 3 tiles per resident workgroup instead
        // of 8 (8x4 at N = 8): csg32 6.37 -> 6.62x, csg256 balanced 6.79 -> 4.18x,
        // chain 6.83 -> 4.75x, csg32_nested 6.35 -> 5.83x, RTIOW 6.59 -> 6.63x; kept at 8.
        // Round 5 (camera-ray waves, tools/root_step.py at N = 8 without the present
        // map-back, band 5:1): small tiles now cost more -- a wave drains its last paths
        // at the end of every tile, and a 4x4 tile gives a wave 4 camera iterations (the
        // whole csg32 frame in 4x4 tiles: 2.77 -> 3.33 ms) -- so the specialised kernels
        // of trees up to depth 32 (the generator's `wo_share_tiles`) want 3 tiles per
        // resident workgroup: csg32 6.30 -> 6.87x, csg32_nested 7.09 -> 7.66x, csg256
        // balanced 6.88 -> 7.19x; the chain keeps 8 (6.96 -> 6.46x with 3: its costly tiles
        // set the end of a share); the lane tracer keeps 8.  Those runs put rank 0's five
        // streams on HIP's 4 hardware queues, so a render could queue behind a copy; with
        // bench.py's layout (two render streams + one gather stream, 8 queues) 3 wins for
        // every scene (want 3 / 8, N = 8 projection): csg32 6.86 / 6.40x, csg32_nested
        // 7.67 / 7.27x, balanced 7.17 / 6.78x, chain 6.99 / 6.88x, RTIOW 7.37 / 6.97x,
        // csg512 6.00 / 5.45x, C4 7.59 / 7.60x (profiles/r05_root_step_want_hwq8.log).
        // So every kernel passes kShareTiles (the lane tracer, the interpreter and a
        // specialised kernel without the generator's marker included).
        const char* tw = getenv("WOLOLO_TILE_WANT");  // (measurement) tiles per resident workgroup
        const char* ts = getenv("WOLOLO_TILE_SPAN");  // (measurement) 8x8 tiles may span two row bands
        const uint64_t want_tiles = (uint64_t)(tw && *tw ? (uint32_t)atoi(tw) : want_per_wg) * resident;
        const bool span = ts && *ts == '1';
        big = 3u | (3u << 4);
        if ((uint64_t)tiles_across(width, big) * (rows >> 3) < want_tiles || (band_rows < 8u && !span)) {
            big = 3u | (2u << 4);
            tail_rounds = 2.0;
        }
        if ((uint64_t)tiles_across(width, big) * (rows >> 2) < want_tiles) big = s44;
    }
    g.big_log2 = big;
    g.tiles_x_big = tiles_across(width, big);
    const uint32_t bh = 1u << (big >> 4);
    uint32_t rows_small = 0;
    if (tail_rounds > 0.0 && big != small) {
        uint64_t want = (uint64_t)(tail_rounds * resident + 0.5);
        rows_small = (uint32_t)(((want + g.tiles_x_small - 1u) / g.tiles_x_small) * sh);
    }
    uint32_t rows_big = rows > rows_small ? ((rows - rows_small) / bh) * bh : 0u;
    if (big == small) rows_big = ((rows + bh - 1u) / bh) * bh;  // one shape: the big grid covers everything
    g.rows_big = rows_big;
    g.n_big = g.tiles_x_big * (rows_big / bh);
    return g;
}

static const size_t kLdsBudget = 64u * 1024u;
// Lane-traversal nodes in LDS: up to ~1200 nodes keeps 6 workgroups per CU

extern "C" int wo_dev_launch(WoDev* dev, WoFrame const* frame_in, void* d_out, void* stream_v,
                             unsigned long long* d_segments, char* err, size_t errlen) {
    return wo_dev_launch_ex(dev, frame_in, d_out, stream_v, d_segments, nullptr, 0u, err, errlen);
}

// the numbers are wo_renderer_lanes_info's "kind" (the lane tracer's forms, LaneTracer)
enum PathKind { kLanesBvh = 2, kLanesBvhSpheres = 3, kLanesTerms = 6, kLanesGeneral = 7, kLanesDynWideTerms = 14,
                kJit = 16, kInterpLds = 17, kInterpGlobal = 18 };

template <bool kCount>
static hipError_t static_occupancy(PathKind kind, size_t dyn_lds, int* per_cu) {
    switch (kind) {
    case kLanesBvh:
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, pathtrace_lanes_kernel<2, kCount>, kBlock, dyn_lds);
    case kLanesBvhSpheres:
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, pathtrace_lanes_kernel<3, kCount>, kBlock, dyn_lds);
    case kLanesTerms:
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, pathtrace_lanes_kernel<6, kCount>, kBlock, dyn_lds);
    case kLanesGeneral:
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, pathtrace_lanes_kernel<7, kCount>, kBlock, dyn_lds);
    case kLanesDynWideTerms:
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, pathtrace_lanes_kernel<14, kCount>, kBlock, dyn_lds);
    case kInterpLds:
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, pathtrace_kernel<true, kCount>, kBlock, dyn_lds);
    default:
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, pathtrace_kernel<false, kCount>, kBlock, dyn_lds);
    }
}

// Resources of one path kernel as the runtime loaded it (hipFuncGetAttributes):
// private (scratch) bytes per lane, VGPRs, static LDS.
template <bool kCount>
static hipError_t static_attrs(PathKind kind, hipFuncAttributes* a) {
    switch (kind) {
    case kLanesBvh: return hipFuncGetAttributes(a, (const void*)pathtrace_lanes_kernel<2, kCount>);
    case kLanesBvhSpheres: return hipFuncGetAttributes(a, (const void*)pathtrace_lanes_kernel<3, kCount>);
    case kLanesTerms: return hipFuncGetAttributes(a, (const void*)pathtrace_lanes_kernel<6, kCount>);
    case kLanesGeneral: return hipFuncGetAttributes(a, (const void*)pathtrace_lanes_kernel<7, kCount>);
    case kLanesDynWideTerms: return hipFuncGetAttributes(a, (const void*)pathtrace_lanes_kernel<14, kCount>);
    case kInterpLds: return hipFuncGetAttributes(a, (const void*)pathtrace_kernel<true, kCount>);
    default: return hipFuncGetAttributes(a, (const void*)pathtrace_kernel<false, kCount>);
    }
}

// The path kernel of the last launch: key_hex (65 bytes) gets the specialised
// kernel's code-object key (jit_key) or "static:<kind>:<source hash>"; out[0] = kind (PathKind),
// out[1] = private bytes per lane, out[2] = registers (VGPRs), out[3] = static LDS
// bytes.  A profile session records these beside its counters, so a summary says
// which code object it measured.
extern "C" int wo_dev_kernel_info(WoDev* dev, char* key_hex, uint32_t* out) {
    if (!dev || !out || dev->last_kind == 0u) return -1;
    const PathKind kind = (PathKind)dev->last_kind;
    if (hipSetDevice(dev->device) != hipSuccess) return -1;
    out[0] = (uint32_t)kind;
    if (kind == kJit) {
        if (!dev->jit_fn || dev->jit_attr[0] < 0 || dev->jit_attr[1] < 0 || dev->jit_attr[2] < 0) return -1;
        out[1] = (uint32_t)dev->jit_attr[0];  // read when the module was loaded (wo_dev_set_jit)
        out[2] = (uint32_t)dev->jit_attr[1];
        out[3] = (uint32_t)dev->jit_attr[2];
        if (key_hex) snprintf(key_hex, 65, "%s", dev->jit_key.c_str());
    } else {
        // "static:<kind>:" + the first 40 hex digits of the library kernels' source hash
        hipFuncAttributes a;
        if (static_attrs<false>(kind, &a) != hipSuccess) return -1;
        out[1] = (uint32_t)a.localSizeBytes;
        out[2] = (uint32_t)a.numRegs;
        out[3] = (uint32_t)a.sharedSizeBytes;
        if (key_hex) snprintf(key_hex, 65, "static:%u:%.40s", (unsigned)kind, WO_STATIC_SRC_SHA);
    }
    return 0;
}

template <int kMode, bool kCount>
static void lanes_launch(dim3 grid, size_t dyn_lds, hipStream_t stream, WoDev* dev, const WoFrame& fr,
                         uint32_t local_rows, float4* out, unsigned long long* slots, const PathLaunch& tg) {
    hipLaunchKernelGGL((pathtrace_lanes_kernel<kMode, kCount>), grid, dim3(kBlock), dyn_lds, stream, dev->d_prog,
                       dev->d_ordpc, dev->d_mats, fr, local_rows, out, slots, tg, lane_bvh(dev));
}

template <bool kCount>
static void static_launch(PathKind kind, dim3 grid, size_t dyn_lds, hipStream_t stream, WoDev* dev, const WoFrame& fr,
                          const KLayout& lay, uint32_t local_rows, float4* out, unsigned long long* slots,
                          const PathLaunch& tg) {
    switch (kind) {
    case kLanesBvh:
        lanes_launch<2, kCount>(grid, dyn_lds, stream, dev, fr, local_rows, out, slots, tg);
        break;
    case kLanesBvhSpheres:
        lanes_launch<3, kCount>(grid, dyn_lds, stream, dev, fr, local_rows, out, slots, tg);
        break;
    case kLanesTerms:
        lanes_launch<6, kCount>(grid, dyn_lds, stream, dev, fr, local_rows, out, slots, tg);
        break;
    case kLanesGeneral:
        lanes_launch<7, kCount>(grid, dyn_lds, stream, dev, fr, local_rows, out, slots, tg);
        break;
    case kLanesDynWideTerms:
        lanes_launch<14, kCount>(grid, dyn_lds, stream, dev, fr, local_rows, out, slots, tg);
        break;
    case kInterpLds:
        hipLaunchKernelGGL((pathtrace_kernel<true, kCount>), grid, dim3(kBlock), dyn_lds, stream, dev->d_prog,
                           dev->d_mats, fr, lay, local_rows, out, slots, tg);
        break;
    default:
        hipLaunchKernelGGL((pathtrace_kernel<false, kCount>), grid, dim3(kBlock), dyn_lds, stream, dev->d_prog,
                           dev->d_mats, fr, lay, local_rows, out, slots, tg);
        break;
    }
}

static int launch_impl(WoDev* dev, WoFrame const* frame_in, void* d_out, void* stream_v,
                       unsigned long long* d_segments, long long* d_accum, uint32_t accum_spp, bool count, char* err,
                       size_t errlen);

extern "C" int wo_dev_launch_ex(WoDev* dev, WoFrame const* frame_in, void* d_out, void* stream_v,
                                unsigned long long* d_segments, long long* d_accum, uint32_t accum_spp, char* err,
                                size_t errlen) {
    return launch_impl(dev, frame_in, d_out, stream_v, d_segments, d_accum, accum_spp, false, err, errlen);
}

// `count`: the counting variant of the chosen path kernel (work counters in the
// segment slots; wo_dev_count_work collects them).
static int launch_impl(WoDev* dev, WoFrame const* frame_in, void* d_out, void* stream_v,
                       unsigned long long* d_segments, long long* d_accum, uint32_t accum_spp, bool count, char* err,
                       size_t errlen) {
    hipStream_t stream = (hipStream_t)stream_v;  // NULL = the null stream (HIP convention)
    WoFrame fr = *frame_in;
    if (fr.width == 0 || fr.height == 0) return 0;
    if (fr.tile_rows == 0 || fr.nranks == 0 || fr.rank >= fr.nranks) {
        snprintf(err, errlen, "bad row tiling (tile_rows=%u rank=%u nranks=%u)", fr.tile_rows, fr.rank, fr.nranks);
        return -1;
    }
    if (fr.n_recs != dev->n_recs || fr.n_prims != dev->n_prims) {
        snprintf(err, errlen, "frame/scene mismatch (recs %u vs %u)", fr.n_recs, dev->n_recs);
        return -1;
    }
    hipError_t e = hipSetDevice(dev->device);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipSetDevice", e);
        return -1;
    }
    uint32_t local_rows = wo_rank_local_rows_ex(fr.height, fr.tile_rows, fr.nranks, fr.band_cycle, fr.band_skip);
    float4* out = (float4*)d_out;

    if (fr.mode == WO_MODE_UBERSHADER_RT1 || fr.mode == WO_MODE_DEBUG_ST) {
        dim3 grid((fr.width + kBlock - 1) / kBlock, local_rows);
        hipLaunchKernelGGL(ubershader_kernel, grid, dim3(kBlock), 0, stream, fr, local_rows, out);
    } else if (fr.mode == WO_MODE_PATHTRACE || fr.mode == WO_MODE_NORMALS) {
        if (fr.n_prims >= (1u << 20)) {
            snprintf(err, errlen, "scene has %u primitives (max %u)", fr.n_prims, (1u << 20) - 1u);
            return -1;
        }
        // the kernels count segments into the per-device slots; seg_collect_kernel
        // then moves the sum into the caller's counter
        unsigned long long* slots = nullptr;
        if (d_segments) {
            if (!dev->d_segslots) {
                e = hipMalloc((void**)&dev->d_segslots, kSegSlots * kSegStride * sizeof(unsigned long long));
                if (e == hipSuccess)
                    e = zero_now(dev->d_segslots, kSegSlots * kSegStride * sizeof(unsigned long long));
                if (e != hipSuccess) {
                    dev->d_segslots = nullptr;
                    set_err(err, errlen, "hipMalloc(segment slots)", e);
                    return -1;
                }
            }
            slots = dev->d_segslots;
        }
        // which kernel, with how much dynamic LDS; then the workgroups one CU holds
        PathKind kind;
        size_t dyn_lds = 0;
        KLayout lay = {};
        if (dev->lanes_on && (dev->union_only || dev->lb_terms || dev->lb_general) && !dev->jit_fn) {
            // the ordered BVH, its lane stacks and top nodes in LDS.  Term mode over more
            // than 256 terms: the 4-wide tree with the resumable walk (dynamic ray fetch;
            // csg512_balanced 84.3 -> 44.7 ms; slower where walks are short or alike: the
            // RTIOW cover 11.7 -> 12.9-15.5 ms, csg256 balanced's 65 terms 16.5 -> 18.2;
            // DESIGN.md §3.6c)
            kind = dev->lb_wide      ? kLanesDynWideTerms
                   : dev->lb_terms   ? kLanesTerms
                   : dev->lb_general ? kLanesGeneral
                   : (dev->lb_spheres_only ? kLanesBvhSpheres : kLanesBvh);
            const size_t stacks = ((size_t)dev->lb_depth * kBlock * (dev->lb_stack16 ? 2u : 4u) + 15u) & ~(size_t)15u;
            dyn_lds = stacks + (size_t)dev->lb_top * lb_node_f4(dev) * sizeof(float4);
            if (dev->lb_general) dyn_lds += (size_t)dev->lb_gwords * kBlock * sizeof(uint32_t);  // the tree's bits
        } else if (dev->jit_fn) {
            kind = kJit;
        } else {
            lay.codes_words = (fr.n_recs + 7u) / 8u + 1u;
            lay.ordpc_off = lay.codes_words;
            uint32_t hib_words = fr.n_prims > 64u ? (fr.n_prims - 64u + 31u) / 32u : 0u;
            lay.hib_off = lay.ordpc_off + fr.n_prims;
            lay.wave_words = (lay.hib_off + hib_words * 64u + 3u) & ~3u;
            size_t scratch = (size_t)(kBlock / 64u) * lay.wave_words * 4u;
            size_t prog_bytes = (size_t)fr.n_recs * sizeof(WoRec);
            if (prog_bytes + scratch <= kLdsBudget) {
                kind = kInterpLds;
                dyn_lds = prog_bytes + scratch;
            } else if (scratch <= kLdsBudget) {
                kind = kInterpGlobal;
                dyn_lds = scratch;
            } else {
                snprintf(err, errlen, "scene too large for the LDS scratch (%zu bytes per workgroup)", scratch);
                return -1;
            }
        }
        dev->last_kind = (uint32_t)kind;
        int per_cu = 0;
        hipFunction_t jfn = count ? dev->count_fn : dev->jit_fn;
        if (kind == kJit)
            e = hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, jfn, kBlock, 0);
        else
            e = count ? static_occupancy<true>(kind, dyn_lds, &per_cu) : static_occupancy<false>(kind, dyn_lds, &per_cu);
        if (e != hipSuccess || per_cu < 1) per_cu = 1;
        // a rank's local rows are bands of tile_rows consecutive frame rows: a tile
        // taller than a band would join rows far apart (incoherent primary rays)
        PathLaunch tg = plan_tiles(fr.width, local_rows, (uint32_t)dev->cus * (uint32_t)per_cu,
                                   fr.nranks > 1u ? fr.tile_rows : ~0u, kind == kJit ? dev->jit_share_tiles : kShareTiles);
        if (d_accum && fr.mode == WO_MODE_PATHTRACE) {
            tg.acc = d_accum;
            tg.acc_spp = accum_spp;
        }
        const uint64_t n_small =
            local_rows > tg.rows_big
                ? (uint64_t)tg.tiles_x_small * ((local_rows - tg.rows_big + (1u << (tg.small_log2 >> 4)) - 1u) >>
                                                (tg.small_log2 >> 4))
                : 0u;
        const uint64_t n_wg = (uint64_t)tg.n_big + n_small;
        if (n_wg >= (1ull << 31)) {
            snprintf(err, errlen, "frame too large (%llu workgroups)", (unsigned long long)n_wg);
            return -1;
        }
        dim3 grid((uint32_t)n_wg);
        if (kind == kJit) {
            const WoRec* p = dev->d_prog;
            const WoMaterial* m = dev->d_mats;
            unsigned long long* sl = slots;
            PathLaunch plv = tg;
            void* args[] = {&p, &m, &fr, &local_rows, &out, &sl, &plv};
            e = hipModuleLaunchKernel(jfn, grid.x, 1, 1, kBlock, 1, 1, 0, stream, args, nullptr);
            if (e != hipSuccess) {
                set_err(err, errlen, "hipModuleLaunchKernel", e);
                return -1;
            }
        } else if (count) {
            static_launch<true>(kind, grid, dyn_lds, stream, dev, fr, lay, local_rows, out, slots, tg);
        } else {
            static_launch<false>(kind, grid, dyn_lds, stream, dev, fr, lay, local_rows, out, slots, tg);
        }
        if (slots) hipLaunchKernelGGL(seg_collect_kernel, dim3(1), dim3(kBlock), 0, stream, slots, d_segments);
    } else {
        snprintf(err, errlen, "unknown shading mode %u", fr.mode);
        return -1;
    }
    e = hipGetLastError();
    if (e != hipSuccess) {
        set_err(err, errlen, "kernel launch", e);
        return -1;
    }
    return 0;
}

// One frame of this rank with the counting variant of its path kernel:
// counts[WO_WORK_*] are lane counts of what ran (synchronous; the image goes to
// the device's scratch frame and equals the normal kernel's).
extern "C" int wo_dev_count_work(WoDev* dev, WoFrame const* frame, unsigned long long* counts, char* err,
                                 size_t errlen) {
    WoFrame fr = *frame;
    if (fr.mode != WO_MODE_PATHTRACE && fr.mode != WO_MODE_NORMALS) {
        snprintf(err, errlen, "work counters need a path-traced frame");
        return -1;
    }
    hipError_t e = hipSetDevice(dev->device);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipSetDevice", e);
        return -1;
    }
    if (dev->jit_fn && !dev->count_fn) {
        std::vector<char> code;
        std::string key;
        int origin = -1;
        double sec = 0.0;
        if (jit_code(dev->jit_src.c_str(), dev->arch, true, code, key, origin, sec, err, errlen)) return -1;
        if (load_jit_module(code, &dev->count_module, &dev->count_fn, err, errlen)) return -1;
    }
    const size_t local_rows = wo_rank_local_rows_ex(fr.height, fr.tile_rows, fr.nranks, fr.band_cycle, fr.band_skip);
    if (ensure_buffer(&dev->d_frame, &dev->frame_cap, local_rows * fr.width * sizeof(float4), err, errlen)) return -1;
    if (!dev->d_work) {
        e = hipMalloc((void**)&dev->d_work, WO_WORK_KINDS * sizeof(unsigned long long));
        if (e != hipSuccess) {
            dev->d_work = nullptr;
            set_err(err, errlen, "hipMalloc(work counters)", e);
            return -1;
        }
    }
    e = hipMemsetAsync(dev->d_work, 0, WO_WORK_KINDS * sizeof(unsigned long long), dev->stream);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipMemsetAsync(work counters)", e);
        return -1;
    }
    if (launch_impl(dev, &fr, dev->d_frame, dev->stream, dev->d_work, nullptr, 0u, true, err, errlen)) return -1;
    hipLaunchKernelGGL(work_collect_kernel, dim3(1), dim3(kBlock), 0, dev->stream, dev->d_segslots, dev->d_work);
    e = hipGetLastError();
    if (e == hipSuccess)
        e = hipMemcpyAsync(counts, dev->d_work, WO_WORK_KINDS * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                           dev->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(dev->stream);
    if (e != hipSuccess) {
        set_err(err, errlen, "work counters", e);
        return -1;
    }
    return 0;
}

extern "C" int wo_dev_render_host(WoDev* dev, WoFrame const* frame, float* host_rgba, char* err, size_t errlen) {
    WoFrame fr = *frame;
    fr.tile_rows = 16;
    fr.rank = 0;
    fr.nranks = 1;
    size_t local_rows = wo_rank_local_rows(fr.height, fr.tile_rows, 1);
    size_t bytes = local_rows * fr.width * sizeof(float4);
    hipError_t e = hipSetDevice(dev->device);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipSetDevice", e);
        return -1;
    }
    if (ensure_buffer(&dev->d_frame, &dev->frame_cap, bytes, err, errlen)) return -1;
    if (wo_dev_launch(dev, &fr, dev->d_frame, dev->stream, nullptr, err, errlen)) return -1;
    e = hipMemcpyAsync(host_rgba, dev->d_frame, (size_t)fr.width * fr.height * sizeof(float4), hipMemcpyDeviceToHost,
                       dev->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(dev->stream);
    if (e != hipSuccess) {
        set_err(err, errlen, "render (device->host)", e);
        return -1;
    }
    return 0;
}

// ---- progressive accumulation and the draw_frame pipeline (renderer.c) ----

// Frames of the pipeline are whole frames (one rank, 4-row tiles).
static WoFrame whole_frame(WoFrame const* f) {
    WoFrame fr = *f;
    fr.tile_rows = 4;
    fr.rank = 0;
    fr.nranks = 1;
    return fr;
}

extern "C" int wo_dev_accum_prepare(WoDev* dev, uint32_t width, uint32_t height, uint32_t tile_rows,
                                    uint32_t nranks, int reset, long long** d_accum, char* err, size_t errlen) {
    hipError_t e = hipSetDevice(dev->device);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipSetDevice", e);
        return -1;
    }
    const size_t bytes = (size_t)width * wo_rank_local_rows(height, tile_rows, nranks) * 3u * sizeof(long long);
    const long long* old = dev->d_accum;
    if (ensure_buffer(&dev->d_accum, &dev->accum_cap, bytes, err, errlen)) return -1;
    if (reset || dev->d_accum != old) {
        e = hipMemsetAsync(dev->d_accum, 0, bytes, dev->stream);
        if (e != hipSuccess) {
            set_err(err, errlen, "hipMemsetAsync(accumulation)", e);
            return -1;
        }
    }
    *d_accum = dev->d_accum;
    return 0;
}

static int ensure_event(hipEvent_t* ev, char* err, size_t errlen) {
    if (*ev) return 0;
    hipError_t e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    if (e != hipSuccess) {
        *ev = nullptr;
        set_err(err, errlen, "hipEventCreate", e);
        return -1;
    }
    return 0;
}

static int ensure_pinned(void** p, size_t* cap, size_t bytes, char* err, size_t errlen) {
    if (bytes <= *cap && *p) return 0;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipHostMalloc(p, bytes ? bytes : 64, hipHostMallocDefault);
    if (e != hipSuccess) {
        *p = nullptr;
        set_err(err, errlen, "hipHostMalloc(frame slot)", e);
        return -1;
    }
    *cap = bytes;
    return 0;
}

// The slot's buffers on the device that presents (current device = dev's):
// the device frame (`frame_rows` rows), its pinned host copy, the present
// encode on both sides and the slot event.
static int prep_slot(WoDev* dev, int slot, uint32_t width, uint32_t height, uint32_t frame_rows, char* err,
                     size_t errlen) {
    const size_t pixels = (size_t)width * height;
    if (ensure_buffer(&dev->d_slot[slot], &dev->dslot_cap[slot], (size_t)width * frame_rows * sizeof(float4), err,
                      errlen))
        return -1;
    if (ensure_pinned((void**)&dev->h_slot[slot], &dev->hslot_cap[slot], pixels * sizeof(float4), err, errlen))
        return -1;
    if (ensure_pinned((void**)&dev->h_bgra[slot], &dev->hbgra_cap[slot], pixels * sizeof(uint32_t), err, errlen))
        return -1;
    if (ensure_buffer(&dev->d_bgra[slot], &dev->dbgra_cap[slot], pixels * sizeof(uint32_t), err, errlen)) return -1;
    if (ensure_event(&dev->rend_ev[slot], err, errlen)) return -1;
    return ensure_event(&dev->slot_ev[slot], err, errlen);
}

// Before a frame is rendered into d_slot: the render stream waits for the
// slot's previous map-back (it reads d_slot / d_bgra on the copy stream), and
// the render-begin stamp.
static int open_slot(WoDev* dev, int slot, char* err, size_t errlen) {
    hipError_t e = dev->slot_recorded[slot] ? hipStreamWaitEvent(dev->stream, dev->slot_ev[slot], 0) : hipSuccess;
    if (e == hipSuccess && dev->stamps) e = hipEventRecord(dev->st_ev[slot][0], dev->stream);
    if (e != hipSuccess) {
        set_err(err, errlen, "frame slot gate", e);
        return -1;
    }
    return 0;
}

// After the frame is in d_slot (on the render stream): the map-back on the copy
// stream -- the present encode, its copy to pinned host memory and, when
// `map_float`, the float frame's copy -- then the slot event.  The render stream
// does not wait for any of it: the next frame's kernel starts at once.
// `encoded`: the ranks have already written the present encode into h_bgra (the
// split present, wo_dev_frame_submit_ranks); only the float frame is left.
static int present_slot(WoDev* dev, int slot, size_t pixels, bool map_float, char* err, size_t errlen,
                        bool encoded = false) {
    hipError_t e = dev->stamps ? hipEventRecord(dev->st_ev[slot][1], dev->stream) : hipSuccess;
    if (e == hipSuccess) e = hipEventRecord(dev->rend_ev[slot], dev->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(dev->copy_stream, dev->rend_ev[slot], 0);
    if (e != hipSuccess) {
        set_err(err, errlen, "map-back gate", e);
        return -1;
    }
    dev->slot_float[slot] = map_float || !pixels;
    dev->slot_pixels[slot] = pixels;
    if (pixels) {
        // the present encode (wo_renderer_last_frame_bgra8) and, eagerly or on
        // demand (wo_dev_frame_map_float), the float frame (wo_renderer_last_frame)
        if (!encoded) {
            if (wo_dev_srgb8(dev->d_slot[slot], dev->d_bgra[slot], pixels, dev->copy_stream, err, errlen)) return -1;
            e = hipMemcpyAsync(dev->h_bgra[slot], dev->d_bgra[slot], pixels * sizeof(uint32_t), hipMemcpyDeviceToHost,
                               dev->copy_stream);
        }
        if (e == hipSuccess && map_float)
            e = hipMemcpyAsync(dev->h_slot[slot], dev->d_slot[slot], pixels * sizeof(float4), hipMemcpyDeviceToHost,
                               dev->copy_stream);
        if (e != hipSuccess) {
            set_err(err, errlen, "hipMemcpyAsync(frame slot)", e);
            return -1;
        }
    }
    e = dev->stamps ? hipEventRecord(dev->st_ev[slot][2], dev->copy_stream) : hipSuccess;
    if (e == hipSuccess) e = hipEventRecord(dev->slot_ev[slot], dev->copy_stream);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipEventRecord", e);
        return -1;
    }
    dev->slot_recorded[slot] = true;
    dev->st_valid[slot] = dev->stamps;
    return 0;
}

static bool present_slot_ok(int slot) { return slot >= 0 && slot <= WO_SLOT_SYNC; }

extern "C" int wo_dev_frame_submit(WoDev* dev, WoFrame const* frame, int slot, long long* d_accum,
                                   uint32_t accum_spp, int map_float, char* err, size_t errlen) {
    if (!present_slot_ok(slot)) {
        snprintf(err, errlen, "bad frame slot %d", slot);
        return -1;
    }
    WoFrame fr = whole_frame(frame);
    hipError_t e = hipSetDevice(dev->device);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipSetDevice", e);
        return -1;
    }
    if (prep_slot(dev, slot, fr.width, fr.height, wo_rank_local_rows(fr.height, fr.tile_rows, 1u), err, errlen))
        return -1;
    if (open_slot(dev, slot, err, errlen)) return -1;
    if (wo_dev_launch_ex(dev, &fr, dev->d_slot[slot], dev->stream, nullptr, d_accum, accum_spp, err, errlen))
        return -1;
    // whole frame, one rank: the local rows are the frame rows
    return present_slot(dev, slot, (size_t)fr.width * fr.height, map_float != 0, err, errlen);
}

// The float frame of a presented slot whose map-back left it on the device
// (lazy map-back): copied now, synchronously.  The slot must have been waited
// for and not submitted again since.
extern "C" int wo_dev_frame_map_float(WoDev* dev, int slot, float const** host, char* err, size_t errlen) {
    if (!present_slot_ok(slot) || !dev->slot_ev[slot] || !dev->d_slot[slot] || !dev->h_slot[slot]) {
        snprintf(err, errlen, "frame slot %d holds no frame", slot);
        return -1;
    }
    if (!dev->slot_float[slot]) {
        // The presented slot's frame is complete (its slot_ev was waited for when it
        // was presented); the copy runs on map_stream, after slot_ev, so it does not
        // wait for the frame in flight behind it on copy_stream.
        hipError_t e = hipSetDevice(dev->device);
        const size_t bytes = dev->slot_pixels[slot] * sizeof(float4);
        if (e == hipSuccess && !dev->map_stream) e = hipStreamCreateWithFlags(&dev->map_stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamWaitEvent(dev->map_stream, dev->slot_ev[slot], 0);
        if (e == hipSuccess) e = hipMemcpyAsync(dev->h_slot[slot], dev->d_slot[slot], bytes, hipMemcpyDeviceToHost,
                                                dev->map_stream);
        if (e == hipSuccess) e = hipStreamSynchronize(dev->map_stream);
        if (e != hipSuccess) {
            set_err(err, errlen, "float frame map-back", e);
            return -1;
        }
        dev->slot_float[slot] = true;
    }
    *host = dev->h_slot[slot];
    return 0;
}

// Pipeline timestamps: while on, every frame submitted to a present slot records
// three timing events (render begin and end on the render stream, map-back end
// on the copy stream); wo_dev_slot_stamps reads them, in ms after the moment
// stamps were turned on.
extern "C" int wo_dev_set_stamps(WoDev* dev, int on, char* err, size_t errlen) {
    hipError_t e = hipSetDevice(dev->device);
    auto mk = [&](hipEvent_t* ev) {
        if (e == hipSuccess && !*ev) e = hipEventCreate(ev);
    };
    if (on) {
        mk(&dev->st_base);
        for (int i = 0; i < WO_SLOTS; ++i)
            for (int k = 0; k < 3; ++k) mk(&dev->st_ev[i][k]);
        if (e == hipSuccess) e = hipEventRecord(dev->st_base, dev->stream);
    }
    if (e != hipSuccess) {
        set_err(err, errlen, "pipeline stamps", e);
        return -1;
    }
    dev->stamps = on != 0;
    for (int i = 0; i < WO_SLOTS; ++i) dev->st_valid[i] = false;
    return 0;
}

extern "C" int wo_dev_slot_stamps(WoDev* dev, int slot, double out[3]) {
    if (!present_slot_ok(slot) || !dev->st_valid[slot]) return -1;
    for (int k = 0; k < 3; ++k) {
        float ms = 0.0f;
        if (hipEventSynchronize(dev->st_ev[slot][k]) != hipSuccess ||
            hipEventElapsedTime(&ms, dev->st_base, dev->st_ev[slot][k]) != hipSuccess)
            return -1;
        out[k] = ms;
    }
    dev->st_valid[slot] = false;
    return 0;
}

// The caller's view of the device: every stream of it drained (set_devices /
// del before releasing ranks whose buffers the root's streams may still read).
extern "C" int wo_dev_sync(WoDev* dev) {
    if (!dev) return 0;
    return hipSetDevice(dev->device) == hipSuccess && hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

extern "C" int wo_dev_peer_mode(WoDev* dev) { return dev ? dev->peer_mode : -1; }

extern "C" int wo_dev_enable_peer(WoDev* from, WoDev* to, char* err, size_t errlen) {
    const char* pv = getenv("WOLOLO_PEER");
    if (pv && strcmp(pv, "staged") == 0) {
        from->peer_mode = WO_PEER_STAGED;
        return 0;
    }
    if (from->device == to->device) {
        from->peer_mode = WO_PEER_SAME;
        return 0;
    }
    int can = 0;
    hipError_t e = hipDeviceCanAccessPeer(&can, from->device, to->device);
    if (e != hipSuccess || !can) {
        (void)hipGetLastError();
        from->peer_mode = WO_PEER_STAGED;  // no peer path: through pinned host memory
        return 0;
    }
    e = hipSetDevice(from->device);
    if (e == hipSuccess) e = hipDeviceEnablePeerAccess(to->device, 0);
    if (e == hipErrorPeerAccessAlreadyEnabled) {
        (void)hipGetLastError();
        e = hipSuccess;
    }
    if (e != hipSuccess) {
        set_err(err, errlen, "hipDeviceEnablePeerAccess", e);
        return -1;
    }
    from->peer_mode = WO_PEER_DMA;
    return 0;
}

// A frame over n ranks into the root's device buffer `dst`,
// assembled on the root-device stream `s_out`: rank i renders its row-cyclic
// 4-row tiles on its own device and stream once the slot is free (gate: recorded
// on s_out after the slot's previous assembly, so frame k+1 in the other slot
// renders while frame k is still being gathered); ranks 1..n-1 deliver their share into the root's rank-major gather
// buffer (peer DMA over xGMI, a device copy when stacked on the root's device, or
// through pinned host memory without a peer path) and record part_ev; s_out waits
// for every part, then un-interleaves the gathered shares into dst.  The root's
// own share renders on root->stream, straight into its slice of the gather buffer
// (an event orders it when s_out is another stream).  Asynchronous throughout.
// The split present (wo_dev_frame_submit_ranks, WOLOLO_PRESENT_SPLIT=1): rank `rank`
// encodes its own rows for present (srgb8_kernel, the same code per pixel as the
// whole frame's encode) on its copy stream, after its render, and copies them
// straight into the root's pinned frame `h_frame`: its full 4-row bands in one 2D
// copy (band lb is frame band lb * n + rank), a partial last band on its own.  So
// each rank's D2H is 1/n of the frame, over its own link, instead of the root
// copying the whole encoded frame.  Current device: the rank's.
static int present_rows(WoDev* dv, int slot, uint32_t rank, uint32_t n, const WoFrame& fr, const float4* d_rows,
                        hipStream_t src_stream, uint32_t* h_frame, char* err, size_t errlen) {
    const uint32_t T = fr.tile_rows, W = fr.width, H = fr.height;
    const uint32_t lr = wo_rank_local_rows(H, T, n);
    if (ensure_buffer(&dv->d_pbgra[slot], &dv->dpbgra_cap[slot], (size_t)lr * W * sizeof(uint32_t), err, errlen))
        return -1;
    if (ensure_event(&dv->psrc_ev[slot], err, errlen) || ensure_event(&dv->penc_ev[slot], err, errlen) ||
        ensure_event(&dv->pmap_ev[slot], err, errlen))
        return -1;
    const uint32_t cnt = wo_rank_tile_count(H, T, rank, n);
    hipError_t e = hipEventRecord(dv->psrc_ev[slot], src_stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(dv->copy_stream, dv->psrc_ev[slot], 0);
    if (e != hipSuccess) {
        set_err(err, errlen, "split present gate", e);
        return -1;
    }
    if (cnt && wo_dev_srgb8(d_rows, dv->d_pbgra[slot], (size_t)cnt * T * W, dv->copy_stream, err, errlen)) return -1;
    e = hipEventRecord(dv->penc_ev[slot], dv->copy_stream);
    if (e == hipSuccess && cnt) {
        const uint32_t g_last = (cnt - 1u) * n + rank;
        const bool partial = (g_last + 1u) * T > H;
        const uint32_t full = cnt - (partial ? 1u : 0u);
        const size_t band = (size_t)T * W * sizeof(uint32_t);
        if (full)
            e = hipMemcpy2DAsync(h_frame + (size_t)rank * T * W, band * n, dv->d_pbgra[slot], band, band, full,
                                 hipMemcpyDeviceToHost, dv->copy_stream);
        if (e == hipSuccess && partial)
            e = hipMemcpyAsync(h_frame + (size_t)g_last * T * W, dv->d_pbgra[slot] + (size_t)(cnt - 1u) * T * W,
                               (size_t)(H - g_last * T) * W * sizeof(uint32_t), hipMemcpyDeviceToHost,
                               dv->copy_stream);
    }
    if (e == hipSuccess) e = hipEventRecord(dv->pmap_ev[slot], dv->copy_stream);
    if (e != hipSuccess) {
        set_err(err, errlen, "split present copy", e);
        return -1;
    }
    return 0;
}

// Off by default: in tools/root_step.py's N = 8 model (csg32, band 2:1) the other
// ranks' shares took 0.447 ms with their encode + D2H against 0.384 without, and
// rank 0's step stayed between 0.30 and 0.55 ms either way (profiles/r06_split_present.log)
static bool present_split_on() {
    static const bool on = [] {
        const char* v = getenv("WOLOLO_PRESENT_SPLIT");
        return v && *v == '1';
    }();
    return on;
}

// `h_present` (the split present): every rank also encodes its rows into the root's
// pinned frame (present_rows); nullptr: the frame is only assembled.
static int ranks_render_assemble(WoDev* const* devs, uint32_t n, WoFrame fr, int slot, long long* const* d_accum,
                                 uint32_t accum_spp, hipStream_t s_out, float4* dst, bool count_segments, char* err,
                                 size_t errlen, uint32_t* h_present = nullptr) {
    WoDev* root = devs[0];
    fr.tile_rows = 4;
    fr.nranks = n;
    fr.band_cycle = fr.band_skip = 0u;  // the C API's device ranks: one band per rank and round
    const uint32_t lr = wo_rank_local_rows(fr.height, fr.tile_rows, n);
    const size_t share = (size_t)lr * fr.width;  // float4s per rank
    hipError_t e = hipSetDevice(root->device);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipSetDevice", e);
        return -1;
    }
    if (ensure_buffer(&root->d_gather[slot], &root->dgather_cap[slot], share * n * sizeof(float4), err, errlen))
        return -1;
    if (!root->gate_ev[slot]) {  // first use of the slot: nothing to wait for beyond what s_out holds
        if (ensure_event(&root->gate_ev[slot], err, errlen)) return -1;
        e = hipEventRecord(root->gate_ev[slot], s_out);
        if (e != hipSuccess) {
            set_err(err, errlen, "hipEventRecord(gate)", e);
            return -1;
        }
    }
    auto seg_counter = [&](WoDev* dv) -> unsigned long long* {
        if (!count_segments) return nullptr;
        if (!dv->d_segacc) {
            hipError_t m = hipMalloc((void**)&dv->d_segacc, sizeof(unsigned long long));
            if (m == hipSuccess) m = zero_now(dv->d_segacc, sizeof(unsigned long long));
            if (m != hipSuccess) {
                dv->d_segacc = nullptr;
                set_err(err, errlen, "hipMalloc(segment counter)", m);
            }
        }
        return dv->d_segacc;
    };
    // rank 0 renders straight into its slice of the gather buffer
    fr.rank = 0;
    unsigned long long* seg0 = seg_counter(root);
    if (count_segments && !seg0) return -1;
    const bool own_stream = s_out != root->stream;
    if (own_stream) {
        if (ensure_event(&root->part_ev[slot], err, errlen)) return -1;
        e = hipStreamWaitEvent(root->stream, root->gate_ev[slot], 0);
        if (e != hipSuccess) {
            set_err(err, errlen, "hipStreamWaitEvent(gate)", e);
            return -1;
        }
    }
    if (wo_dev_launch_ex(root, &fr, root->d_gather[slot], root->stream, seg0, d_accum ? d_accum[0] : nullptr,
                         accum_spp, err, errlen))
        return -1;
    if (h_present && present_rows(root, slot, 0u, n, fr, root->d_gather[slot], root->stream, h_present, err, errlen))
        return -1;
    if (own_stream) {
        e = hipEventRecord(root->part_ev[slot], root->stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(s_out, root->part_ev[slot], 0);
        if (e != hipSuccess) {
            set_err(err, errlen, "rank 0 share event", e);
            return -1;
        }
    }
    for (uint32_t i = 1; i < n; ++i) {
        WoDev* dv = devs[i];
        fr.rank = i;
        e = hipSetDevice(dv->device);
        if (e != hipSuccess) {
            set_err(err, errlen, "hipSetDevice", e);
            return -1;
        }
        unsigned long long* seg = seg_counter(dv);
        if (count_segments && !seg) return -1;
        if (ensure_buffer(&dv->d_part[slot], &dv->dpart_cap[slot], share * sizeof(float4), err, errlen)) return -1;
        if (ensure_event(&dv->part_ev[slot], err, errlen)) return -1;
        const bool staged = dv->peer_mode == WO_PEER_STAGED;
        if (staged && ensure_pinned((void**)&dv->h_part[slot], &dv->hpart_cap[slot], share * sizeof(float4), err,
                                    errlen))
            return -1;
        e = hipStreamWaitEvent(dv->stream, root->gate_ev[slot], 0);
        if (e != hipSuccess) {
            set_err(err, errlen, "hipStreamWaitEvent(gate)", e);
            return -1;
        }
        if (wo_dev_launch_ex(dv, &fr, dv->d_part[slot], dv->stream, seg, d_accum ? d_accum[i] : nullptr, accum_spp,
                             err, errlen))
            return -1;
        if (h_present && present_rows(dv, slot, i, n, fr, dv->d_part[slot], dv->stream, h_present, err, errlen))
            return -1;
        float4* slice = root->d_gather[slot] + share * i;
        if (staged)  // device -> pinned host on the rank, host -> root below
            e = hipMemcpyAsync(dv->h_part[slot], dv->d_part[slot], share * sizeof(float4), hipMemcpyDeviceToHost,
                               dv->stream);
        else if (dv->device == root->device)
            e = hipMemcpyAsync(slice, dv->d_part[slot], share * sizeof(float4), hipMemcpyDeviceToDevice, dv->stream);
        else
            e = hipMemcpyPeerAsync(slice, root->device, dv->d_part[slot], dv->device, share * sizeof(float4),
                                   dv->stream);
        if (e == hipSuccess) e = hipEventRecord(dv->part_ev[slot], dv->stream);
        if (e == hipSuccess) e = hipSetDevice(root->device);
        if (e == hipSuccess) e = hipStreamWaitEvent(s_out, dv->part_ev[slot], 0);
        if (e == hipSuccess && staged)
            e = hipMemcpyAsync(slice, dv->h_part[slot], share * sizeof(float4), hipMemcpyHostToDevice, s_out);
        if (e != hipSuccess) {
            set_err(err, errlen, staged ? "gather copy (host-staged)" : "gather copy", e);
            return -1;
        }
    }
    if (wo_dev_assemble(root->d_gather[slot], dst, fr.width, fr.height, fr.tile_rows, n, 0u, 0u, s_out, err, errlen))
        return -1;
    // the slot's buffers are free once the assembly (and the split present's
    // encodes) have read them
    for (uint32_t i = 0; h_present && i < n && e == hipSuccess; ++i) e = hipStreamWaitEvent(s_out, devs[i]->penc_ev[slot], 0);
    if (e == hipSuccess) e = hipEventRecord(root->gate_ev[slot], s_out);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipEventRecord(gate)", e);
        return -1;
    }
    return 0;
}

// The draw_frame pipeline over n ranks: the frame is assembled into the slot's
// device frame on the root's stream and then presented as for one device.
extern "C" int wo_dev_frame_submit_ranks(WoDev* const* devs, uint32_t n, WoFrame const* frame, int slot,
                                         long long* const* d_accum, uint32_t accum_spp, int map_float, char* err,
                                         size_t errlen) {
    if (n <= 1u)
        return wo_dev_frame_submit(devs[0], frame, slot, d_accum ? d_accum[0] : nullptr, accum_spp, map_float, err,
                                   errlen);
    if (!present_slot_ok(slot)) {
        snprintf(err, errlen, "bad frame slot %d", slot);
        return -1;
    }
    WoDev* root = devs[0];
    hipError_t e = hipSetDevice(root->device);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipSetDevice", e);
        return -1;
    }
    if (prep_slot(root, slot, frame->width, frame->height, frame->height, err, errlen)) return -1;
    if (open_slot(root, slot, err, errlen)) return -1;
    const size_t pixels = (size_t)frame->width * frame->height;
    const bool split = present_split_on() && pixels;
    if (ranks_render_assemble(devs, n, *frame, slot, d_accum, accum_spp, root->stream, root->d_slot[slot], false, err,
                              errlen, split ? root->h_bgra[slot] : nullptr))
        return -1;
    if (!split) return present_slot(root, slot, pixels, map_float != 0, err, errlen);
    // the split present: the encoded frame is already on its way to h_bgra from
    // every rank; the slot's map-back ends when all of those copies have (and the
    // float frame's, when it is mapped eagerly, after the assembly)
    e = hipSetDevice(root->device);
    for (uint32_t i = 0; i < n && e == hipSuccess; ++i) e = hipStreamWaitEvent(root->copy_stream, devs[i]->pmap_ev[slot], 0);
    if (e != hipSuccess) {
        set_err(err, errlen, "split present wait", e);
        return -1;
    }
    return present_slot(root, slot, pixels, map_float != 0, err, errlen, /*encoded=*/true);
}

extern "C" int wo_dev_frame_ranks_device(WoDev* const* devs, uint32_t n, WoFrame const* frame, int slot, void* d_frame,
                                         void* stream, char* err, size_t errlen) {
    if (slot != WO_SLOT_DEV0 && slot != WO_SLOT_DEV1) {
        snprintf(err, errlen, "bad device-frame slot %d", slot);
        return -1;
    }
    if (!d_frame) {
        snprintf(err, errlen, "no device frame");
        return -1;
    }
    WoDev* root = devs[0];
    if (n <= 1u) {  // one rank: straight into the caller's frame (rows >= height are not written)
        WoFrame fr = whole_frame(frame);
        hipError_t e = hipSetDevice(root->device);
        if (e != hipSuccess) {
            set_err(err, errlen, "hipSetDevice", e);
            return -1;
        }
        if (!root->d_segacc) {
            e = hipMalloc((void**)&root->d_segacc, sizeof(unsigned long long));
            if (e == hipSuccess) e = zero_now(root->d_segacc, sizeof(unsigned long long));
            if (e != hipSuccess) {
                root->d_segacc = nullptr;
                set_err(err, errlen, "hipMalloc(segment counter)", e);
                return -1;
            }
        }
        const bool path = fr.mode == WO_MODE_PATHTRACE || fr.mode == WO_MODE_NORMALS;
        return wo_dev_launch(root, &fr, d_frame, stream, path ? root->d_segacc : nullptr, err, errlen);
    }
    const bool path = frame->mode == WO_MODE_PATHTRACE || frame->mode == WO_MODE_NORMALS;
    return ranks_render_assemble(devs, n, *frame, slot, nullptr, 0u, (hipStream_t)stream, (float4*)d_frame, path, err,
                                 errlen);
}

extern "C" int wo_dev_take_segments(WoDev* dev, unsigned long long* total, char* err, size_t errlen) {
    *total = 0;
    if (!dev->d_segacc) return 0;
    hipError_t e = hipSetDevice(dev->device);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(total, dev->d_segacc, sizeof(unsigned long long), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = zero_now(dev->d_segacc, sizeof(unsigned long long));
    if (e != hipSuccess) {
        set_err(err, errlen, "segment counter", e);
        return -1;
    }
    return 0;
}

extern "C" int wo_dev_frame_wait(WoDev* dev, int slot, float const** host, uint32_t const** host_bgra8, char* err,
                                 size_t errlen) {
    if (!present_slot_ok(slot) || !dev->slot_ev[slot]) {
        snprintf(err, errlen, "frame slot %d was never submitted", slot);
        return -1;
    }
    hipError_t e = hipEventSynchronize(dev->slot_ev[slot]);
    if (e != hipSuccess) {
        set_err(err, errlen, "frame wait", e);
        return -1;
    }
    *host = dev->slot_float[slot] ? dev->h_slot[slot] : nullptr;  // NULL: wo_dev_frame_map_float on demand
    if (host_bgra8) *host_bgra8 = dev->h_bgra[slot];
    return 0;
}

// The present encode's threshold table, one copy per device (built once).
static std::mutex g_srgb_mu;
static float* g_srgb_tab[64];

extern "C" int wo_dev_srgb8(void const* d_rgba, void* d_bgra8, size_t pixels, void* stream, char* err,
                            size_t errlen) {
    if (pixels == 0) return 0;
    int d = -1;
    hipError_t e = hipGetDevice(&d);
    if (e != hipSuccess || d < 0 || d >= 64) {
        set_err(err, errlen, "hipGetDevice", e);
        return -1;
    }
    float* tab = nullptr;
    {
        std::lock_guard<std::mutex> lock(g_srgb_mu);
        if (!g_srgb_tab[d]) {
            float host[255];
            wo_srgb8_thresholds(host);
            float* p = nullptr;
            e = hipMalloc((void**)&p, sizeof host);
            if (e == hipSuccess) e = hipMemcpy(p, host, sizeof host, hipMemcpyHostToDevice);
            if (e != hipSuccess) {
                if (p) (void)hipFree(p);
                set_err(err, errlen, "sRGB table upload", e);
                return -1;
            }
            g_srgb_tab[d] = p;
        }
        tab = g_srgb_tab[d];
    }
    size_t blocks = (pixels + kBlock - 1) / kBlock;
    if (blocks > 16384u) blocks = 16384u;
    hipLaunchKernelGGL(srgb8_kernel, dim3((uint32_t)blocks), dim3(kBlock), 0, (hipStream_t)stream,
                       (const float4*)d_rgba, (uint32_t*)d_bgra8, pixels, (const float*)tab);
    e = hipGetLastError();
    if (e != hipSuccess) {
        set_err(err, errlen, "sRGB encode launch", e);
        return -1;
    }
    return 0;
}

extern "C" int wo_dev_assemble(void const* d_gathered, void* d_frame, uint32_t width, uint32_t height,
                               uint32_t tile_rows, uint32_t nranks, uint32_t cycle, uint32_t skip, void* stream,
                               char* err, size_t errlen) {
    if (tile_rows == 0 || nranks == 0) {
        snprintf(err, errlen, "bad tiling");
        return -1;
    }
    uint32_t local_rows = wo_rank_local_rows_ex(height, tile_rows, nranks, cycle, skip);
    size_t total = (size_t)width * height;
    uint32_t blocks = (uint32_t)((total + kBlock - 1) / kBlock);
    if (blocks > 8192u) blocks = 8192u;
    if (blocks == 0) return 0;
    hipLaunchKernelGGL(assemble_kernel, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream,
                       (const float4*)d_gathered, (float4*)d_frame, width, height, tile_rows, nranks, cycle, skip,
                       local_rows);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_err(err, errlen, "assemble launch", e);
        return -1;
    }
    return 0;
}
