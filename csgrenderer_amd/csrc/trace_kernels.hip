// trace_kernels.hip -- the per-pixel hot path of the wololo renderer, written for
// gfx950 (MI355X, CDNA4, wave64).  Replaces the reference's fragment stage:
//   src/wololo/renderer/ubershader1.frag:19-163 (ray generation, hit_sphere,
//   ray_color, ep_rt1_1 / ep_debug_view_1), launched by the reference as one
//   fragment invocation per pixel from draw_frame_with_renderer
//   (renderer.c:2085-2219).
//
// Kernels
//   ubershader_kernel  -- the reference shader, restated bit-for-bit in IEEE fp32
//                         (sin hoisted to the host).  HBM-store bound: 16 B/pixel.
//   pathtrace_kernel   -- north-star path: CSG program evaluation (stackless,
//                         bit-stack over a postfix program), spheres + half-spaces,
//                         lambertian / metal / dielectric, spp x bounces with
//                         path regeneration.  FP32-VALU bound.
//   assemble_kernel    -- un-interleaves row-cyclic rank tiles after the gather.
//
// Numerics: the whole file is compiled with contraction off, and hipcc lowers
// fp32 '/' and sqrtf to correctly rounded sequences on gfx950
// (v_div_scale/fmas/fixup, v_sqrt + ulp fix-up), so every result is reproducible
// bit-for-bit by the C oracle (oracle/oracle.c) compiled with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "wo_dev.h"
#include "wololo/wo_scene.h"

#pragma clang fp contract(off)

namespace {

constexpr uint32_t kBlock = 256;       // 4 waves
constexpr uint32_t kPtTile = 16;       // pathtrace block = 16x16 pixels, waves = 8x8
constexpr int kWindow = 8;             // sorted event window per lane (registers)
constexpr uint32_t kEmptyKey32 = 0xFFFFFFFFu;
constexpr uint64_t kEmptyKey = ~0ull;
constexpr float kInf = __builtin_inff();

// 4-bit op codes of the per-wave compacted program (8 per dword).
constexpr uint32_t kCodePrim = 1, kCodeUnion = 2, kCodeInter = 3, kCodeDiff = 4, kCodeRdiff = 5,
                   kCodeConst0 = 6;

struct F3 {
    float x, y, z;
};

__device__ __forceinline__ F3 f3(float x, float y, float z) {
    F3 r;
    r.x = x;
    r.y = y;
    r.z = z;
    return r;
}
__device__ __forceinline__ float dot3(F3 a, F3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ F3 unit3(F3 v) {
    float inv = 1.0f / sqrtf(dot3(v, v));
    return f3(v.x * inv, v.y * inv, v.z * inv);
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// ---------------------------------------------------------------------------
// Counter-based RNG (PCG-RXS-M-XS 32), identical to oracle.c.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t pcg_hash(uint32_t v) {
    uint32_t s = v * 747796405u + 2891336453u;
    uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    return (w >> 22u) ^ w;
}
struct Rng {
    uint32_t s;
    __device__ __forceinline__ uint32_t next() {
        s = s * 747796405u + 2891336453u;
        uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
        return (w >> 22u) ^ w;
    }
    __device__ __forceinline__ float uniform() { return (float)(next() >> 8) * 0x1p-24f; }
};

__device__ __forceinline__ F3 random_in_unit_sphere(Rng& rng) {
    for (int i = 0; i < 64; ++i) {
        float x = 2.0f * rng.uniform() - 1.0f;
        float y = 2.0f * rng.uniform() - 1.0f;
        float z = 2.0f * rng.uniform() - 1.0f;
        F3 p = f3(x, y, z);
        float l2 = dot3(p, p);
        if (l2 < 1.0f && l2 > 1e-12f) return p;
    }
    return f3(0.0f, 0.0f, 1.0f);
}

// ---------------------------------------------------------------------------
// Leaf intersections.  Intervals [a, b]; empty = (+inf, -inf).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void leaf_interval(const WoRec& L, uint32_t kind, F3 o, F3 d, float& la, float& lb) {
    if (kind == WO_LEAF_SPHERE) {
        float fx = o.x - L.f[0], fy = o.y - L.f[1], fz = o.z - L.f[2];
        float b = (fx * d.x + fy * d.y) + fz * d.z;
        float lx = fx - b * d.x, ly = fy - b * d.y, lz = fz - b * d.z;
        float ll = (lx * lx + ly * ly) + lz * lz;
        float disc = L.f[3] - ll;
        if (disc < 0.0f) {
            la = kInf;
            lb = -kInf;
        } else {
            float s = sqrtf(disc);
            float nb = -b;
            la = nb - s;
            lb = nb + s;
        }
    } else {
        float den = (L.f[0] * d.x + L.f[1] * d.y) + L.f[2] * d.z;
        float no = (L.f[0] * o.x + L.f[1] * o.y) + L.f[2] * o.z;
        float dist = L.f[3] - no;
        if (den == 0.0f) {
            if (dist >= 0.0f) {
                la = -kInf;
                lb = kInf;
            } else {
                la = kInf;
                lb = -kInf;
            }
        } else {
            float t = dist / den;
            if (den > 0.0f) {
                la = -kInf;
                lb = t;
            } else {
                la = t;
                lb = kInf;
            }
        }
    }
}

struct Ivl {
    float a, b;
    uint32_t ma, mb;
};

// Convex primitive = intersection of its member leaves.  Ties keep the first member.
template <class Prog>
__device__ __forceinline__ Ivl prim_interval(Prog prog, uint32_t pc, uint32_t count, F3 o, F3 d) {
    Ivl iv;
    iv.a = -kInf;
    iv.b = kInf;
    iv.ma = 0;
    iv.mb = 0;
    for (uint32_t m = 0; m < count; ++m) {
        WoRec L = prog[pc + 1u + m];
        uint32_t kind = uni(L.op);
        float la, lb;
        leaf_interval(L, kind, o, d, la, lb);
        if (la > iv.a) {
            iv.a = la;
            iv.ma = m;
        }
        if (lb < iv.b) {
            iv.b = lb;
            iv.mb = m;
        }
    }
    return iv;
}

// Conservative "may the ray [0, inf) touch this bounding sphere" test.  The
// 4e-6*tca^2 slack covers fp32 rounding of the perpendicular distance.
__device__ __forceinline__ bool bound_may_hit(const WoRec& B, F3 o, F3 d) {
    float ox = B.f[0] - o.x, oy = B.f[1] - o.y, oz = B.f[2] - o.z;
    float tca = (ox * d.x + oy * d.y) + oz * d.z;
    float lx = ox - tca * d.x, ly = oy - tca * d.y, lz = oz - tca * d.z;
    float d2 = (lx * lx + ly * ly) + lz * lz;
    bool miss = (d2 > B.f[3] + 4e-6f * (tca * tca)) || (tca + B.f[4] < 0.0f);
    return !miss;
}

// Event key: (t, primitive ordinal, type) lexicographic == one u64 compare,
// because t > WO_T_MIN > 0 makes the float bits monotone.  The low 11 bits
// carry the member leaf that produced the event (for the normal).
__device__ __forceinline__ uint64_t event_key(float t, uint32_t ord, uint32_t type, uint32_t member) {
    return ((uint64_t)__float_as_uint(t) << 32) | (uint64_t)((ord << 12) | (type << 11) | member);
}

// Sorted insertion into the register window (drops the largest on overflow).
struct Window {
    uint64_t k[kWindow];
    bool dropped;
    __device__ __forceinline__ void clear() {
#pragma unroll
        for (int i = 0; i < kWindow; ++i) k[i] = kEmptyKey;
        dropped = false;
    }
    __device__ __forceinline__ void insert(uint64_t key) {
        dropped |= (k[kWindow - 1] != kEmptyKey);
#pragma unroll
        for (int i = kWindow - 1; i > 0; --i) {
            uint64_t prev = k[i - 1];
            uint64_t cur = k[i];
            k[i] = key < prev ? prev : (key < cur ? key : cur);
        }
        k[0] = key < k[0] ? key : k[0];
    }
    __device__ __forceinline__ uint64_t pop() {
        uint64_t r = k[0];
#pragma unroll
        for (int i = 0; i < kWindow - 1; ++i) k[i] = k[i + 1];
        k[kWindow - 1] = kEmptyKey;
        return r;
    }
};

// Per-wave LDS scratch layout (dwords), computed on the host.
struct KLayout {
    uint32_t codes_words;  // packed 4-bit codes of the compacted program
    uint32_t ordpc_off;    // primitive ordinal -> program counter
    uint32_t hib_off;      // membership bits of ordinals >= 64: [word][64 lanes]
    uint32_t wave_words;   // stride between waves
};

struct Trace {
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
    // Evaluate the root over the compacted program with a 32-deep bit stack.
    __device__ __forceinline__ uint32_t eval_root() const {
        uint32_t st = 0, ord = 0;
        uint32_t nwords = (ncodes + 7u) >> 3;
        for (uint32_t w = 0; w < nwords; ++w) {
            uint32_t word = uni(codes[w]);
            uint32_t n = ncodes - w * 8u;
            n = n < 8u ? n : 8u;
            for (uint32_t j = 0; j < n; ++j) {
                uint32_t c = (word >> (4u * j)) & 15u;
                if (c == kCodePrim) {
                    st = (st << 1) | bit(ord);
                    ++ord;
                } else if (c == kCodeConst0) {
                    st = st << 1;
                } else {
                    uint32_t r;
                    if (c == kCodeUnion)
                        r = (st | (st >> 1)) & 1u;
                    else if (c == kCodeInter)
                        r = (st & (st >> 1)) & 1u;
                    else if (c == kCodeDiff)
                        r = (st >> 1) & ~st & 1u;
                    else
                        r = st & ~(st >> 1) & 1u;
                    st = ((st >> 1) & ~1u) | r;
                }
            }
        }
        return st & 1u;
    }
};

struct Hit {
    float t;
    uint32_t ord, type, member;
    uint32_t root_after;  // 1: the ray enters the solid here
};

// Nearest boundary crossing of the CSG root after WO_T_MIN along o + t d
// (|d| = 1).  Must be called by every lane that wants a result; lanes that are
// not tracing must be masked off by the caller.
template <class Prog>
__device__ __forceinline__ bool trace(Prog prog, uint32_t nrec, Trace& tr, F3 o, F3 d, Hit& hit) {
    const float tmin = WO_T_MIN;
    Window win;
    win.clear();
    tr.bits = 0;
    tr.ncodes = 0;
    tr.nprims = 0;
    uint32_t code_acc = 0;
    uint32_t hib_acc = 0;

    // ---- pass 1: walk the program (wave-uniform pc), cull, intersect, collect.
    uint32_t pc = 0;
    while (pc < nrec) {
        WoRec rec = prog[pc];
        uint32_t op = uni(rec.op);
        uint32_t code;
        if (op == WO_OP_BOUND) {
            bool may = bound_may_hit(rec, o, d);
            if (__ballot(may) != 0ull) {
                ++pc;
                continue;
            }
            code = kCodeConst0;
            pc = uni(rec.u0);
        } else if (op == WO_OP_PRIM) {
            uint32_t count = uni(rec.u0);
            uint32_t ord = tr.nprims;
            Ivl iv = prim_interval(prog, pc, count, o, d);
            uint32_t inside = 0;
            if (!(iv.a > iv.b)) {
                inside = (iv.a <= tmin && iv.b > tmin) ? 1u : 0u;
                if (iv.a > tmin) win.insert(event_key(iv.a, ord, 0u, iv.ma));
                if (iv.b > tmin && iv.b < kInf) win.insert(event_key(iv.b, ord, 1u, iv.mb));
            }
            if (ord < 64u) {
                tr.bits |= (uint64_t)inside << ord;
            } else {
                uint32_t sh = (ord - 64u) & 31u;
                hib_acc |= inside << sh;
                if (sh == 31u) {
                    tr.hib[((ord - 64u) >> 5) * 64u + tr.lane] = hib_acc;
                    hib_acc = 0;
                }
            }
            tr.ordpc[ord] = pc;
            tr.nprims = ord + 1u;
            code = kCodePrim;
            pc += 1u + count;
        } else {
            code = op;  // WO_OP_UNION..RDIFF share values with the codes
            ++pc;
        }
        uint32_t slot = tr.ncodes & 7u;
        code_acc |= code << (4u * slot);
        if (slot == 7u) {
            tr.codes[tr.ncodes >> 3] = code_acc;
            code_acc = 0;
        }
        ++tr.ncodes;
    }
    if (tr.ncodes & 7u) tr.codes[tr.ncodes >> 3] = code_acc;
    if (tr.nprims > 64u && ((tr.nprims - 64u) & 31u)) tr.hib[((tr.nprims - 64u) >> 5) * 64u + tr.lane] = hib_acc;

    // ---- pass 2: sweep events in key order; first root flip is the hit.
    bool found = false;
    if (win.k[0] == kEmptyKey) return false;
    uint32_t root = tr.eval_root();
    for (;;) {
        while (win.k[0] != kEmptyKey) {
            uint64_t key = win.pop();
            uint32_t lo = (uint32_t)key;
            uint32_t ord = lo >> 12;
            tr.toggle(ord);
            uint32_t r = tr.eval_root();
            if (r != root) {
                hit.t = __uint_as_float((uint32_t)(key >> 32));
                hit.ord = ord;
                hit.type = (lo >> 11) & 1u;
                hit.member = lo & 2047u;
                hit.root_after = r;
                found = true;
                win.dropped = false;
                break;
            }
            root = r;
            if (win.k[0] == kEmptyKey && win.dropped) {
                // Window exhausted but events were dropped: re-collect the
                // events strictly after `key` (membership state carries on).
                win.clear();
                uint32_t ordc = 0;
                uint32_t nwords = (tr.ncodes + 7u) >> 3;
                for (uint32_t w = 0; w < nwords; ++w) {
                    uint32_t word = uni(tr.codes[w]);
                    uint32_t n = tr.ncodes - w * 8u;
                    n = n < 8u ? n : 8u;
                    for (uint32_t j = 0; j < n; ++j) {
                        if (((word >> (4u * j)) & 15u) != kCodePrim) continue;
                        uint32_t ppc = uni(tr.ordpc[ordc]);
                        uint32_t count = uni(prog[ppc].u0);
                        Ivl iv = prim_interval(prog, ppc, count, o, d);
                        if (!(iv.a > iv.b)) {
                            if (iv.a > tmin) {
                                uint64_t k2 = event_key(iv.a, ordc, 0u, iv.ma);
                                if (k2 > key) win.insert(k2);
                            }
                            if (iv.b > tmin && iv.b < kInf) {
                                uint64_t k2 = event_key(iv.b, ordc, 1u, iv.mb);
                                if (k2 > key) win.insert(k2);
                            }
                        }
                        ++ordc;
                    }
                }
            }
        }
        break;
    }
    return found;
}

__device__ __forceinline__ F3 sky(F3 d) {
    float t = 0.5f * (d.y + 1.0f);
    float s = 1.0f - t;
    return f3(s + t * 0.5f, s + t * 0.7f, s + t * 1.0f);
}

// Pixel -> (local row) mapping for row-cyclic rank tiles.
__device__ __forceinline__ uint32_t local_to_global_row(const WoFrame& fr, uint32_t lrow) {
    uint32_t lt = lrow / fr.tile_rows;
    uint32_t g = lt * fr.nranks + fr.rank;
    return g * fr.tile_rows + (lrow - lt * fr.tile_rows);
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
    float aspect = resx / resy;                   // frag:20
    float fx = (float)lx + 0.5f;                  // gl_FragCoord at the pixel centre,
    float fy = (float)y + 0.5f;                   // OriginUpperLeft (row 0 = top)
    float stx = fx / resx;                        // frag:26-29
    float sty = 1.0f - fy / resy;
    float4 res;
    if (fr.mode == WO_MODE_DEBUG_ST) {            // frag:133-138
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

// ---------------------------------------------------------------------------
// CSG path tracer.
// ---------------------------------------------------------------------------
struct ProgPtr {
    const WoRec* p;
    __device__ __forceinline__ WoRec operator[](uint32_t i) const { return p[i]; }
};

template <bool kProgInLds>
__global__ __launch_bounds__(kBlock) void pathtrace_kernel(const WoRec* __restrict__ gprog,
                                                           const WoMaterial* __restrict__ mats, WoFrame fr,
                                                           KLayout lay, uint32_t local_rows,
                                                           float4* __restrict__ out,
                                                           unsigned long long* __restrict__ seg_out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t nrec = fr.n_recs;

    uint32_t* scratch = smem;
    ProgPtr prog;
    if constexpr (kProgInLds) {
        const uint4* src = reinterpret_cast<const uint4*>(gprog);
        uint4* dst = reinterpret_cast<uint4*>(smem);
        for (uint32_t i = tid; i < nrec * 2u; i += kBlock) dst[i] = src[i];
        __syncthreads();
        prog.p = reinterpret_cast<const WoRec*>(smem);
        scratch = smem + nrec * 8u;
    } else {
        prog.p = gprog;
    }
    uint32_t* ws = scratch + wave * lay.wave_words;
    Trace tr;
    tr.codes = ws;
    tr.ordpc = ws + lay.ordpc_off;
    tr.hib = ws + lay.hib_off;
    tr.lane = lane;

    // 16x16 block; each wave an 8x8 pixel tile for ray coherence.
    uint32_t lx = blockIdx.x * kPtTile + (wave & 1u) * 8u + (lane & 7u);
    uint32_t lrow = blockIdx.y * kPtTile + (wave >> 1) * 8u + (lane >> 3);
    uint32_t y = lrow < local_rows ? local_to_global_row(fr, lrow) : fr.height;
    bool active = lx < fr.width && y < fr.height;

    const WoCamera& cam = fr.cam;
    const uint32_t W = fr.width, H = fr.height;
    const uint32_t pix = y * W + lx;
    const uint32_t spp = fr.mode == WO_MODE_NORMALS ? 1u : fr.spp;
    const uint32_t max_depth = fr.mode == WO_MODE_NORMALS ? 1u : fr.max_depth;
    const uint32_t seed_hash = pcg_hash(fr.seed);

    F3 acc = f3(0.0f, 0.0f, 0.0f);
    F3 o = f3(0.0f, 0.0f, 0.0f), d = f3(0.0f, 0.0f, -1.0f), thr = f3(1.0f, 1.0f, 1.0f);
    Rng rng;
    rng.s = 0;
    uint32_t sample = 0, depth = 0;
    uint32_t segs = 0;
    bool done = !active || spp == 0u || max_depth == 0u;

    // Camera ray for (pix, sample); RTIOW camera.get_ray with defocus.
    auto start_sample = [&]() {
        rng.s = pcg_hash(pix ^ pcg_hash((fr.sample_offset + sample) ^ seed_hash));
        float sx, ty;
        if (fr.mode == WO_MODE_NORMALS) {
            sx = ((float)lx + 0.5f) / (float)W;
            ty = ((float)(H - 1u - y) + 0.5f) / (float)H;
        } else {
            float r1 = rng.uniform();
            float r2 = rng.uniform();
            sx = ((float)lx + r1) / (float)W;
            ty = ((float)(H - 1u - y) + r2) / (float)H;
        }
        float offx = 0.0f, offy = 0.0f, offz = 0.0f;
        if (cam.lens_radius > 0.0f && fr.mode != WO_MODE_NORMALS) {
            float px = 0.0f, py = 0.0f;
            for (int i = 0; i < 64; ++i) {
                px = 2.0f * rng.uniform() - 1.0f;
                py = 2.0f * rng.uniform() - 1.0f;
                if (px * px + py * py < 1.0f) break;
            }
            float rx = cam.lens_radius * px, ry = cam.lens_radius * py;
            offx = cam.u[0] * rx + cam.v[0] * ry;
            offy = cam.u[1] * rx + cam.v[1] * ry;
            offz = cam.u[2] * rx + cam.v[2] * ry;
        }
        o = f3(cam.origin[0] + offx, cam.origin[1] + offy, cam.origin[2] + offz);
        F3 dir = f3(((cam.lower_left[0] + sx * cam.horizontal[0]) + ty * cam.vertical[0]) - cam.origin[0] - offx,
                    ((cam.lower_left[1] + sx * cam.horizontal[1]) + ty * cam.vertical[1]) - cam.origin[1] - offy,
                    ((cam.lower_left[2] + sx * cam.horizontal[2]) + ty * cam.vertical[2]) - cam.origin[2] - offz);
        d = unit3(dir);
        thr = f3(1.0f, 1.0f, 1.0f);
        depth = 0;
    };
    if (!done) start_sample();

    while (__any(!done)) {
        if (!done) {
            Hit h;
            bool found = trace(prog, nrec, tr, o, d, h);
            ++segs;
            bool end = false;
            F3 radiance = f3(0.0f, 0.0f, 0.0f);
            if (!found) {
                F3 s = sky(d);
                radiance = f3(thr.x * s.x, thr.y * s.y, thr.z * s.z);
                end = true;
            } else {
                uint32_t ppc = tr.ordpc[h.ord];
                WoRec L = prog[ppc + 1u + h.member];
                F3 P = f3(o.x + h.t * d.x, o.y + h.t * d.y, o.z + h.t * d.z);
                F3 n;
                if (L.op == WO_LEAF_SPHERE)
                    n = f3((P.x - L.f[0]) * L.f[4], (P.y - L.f[1]) * L.f[4], (P.z - L.f[2]) * L.f[4]);
                else
                    n = f3(L.f[0], L.f[1], L.f[2]);
                // Leaf entered (type 0): its outward normal faces the ray.
                F3 N = h.type == 0u ? n : f3(-n.x, -n.y, -n.z);
                bool front = h.root_after != 0u;
                if (fr.mode == WO_MODE_NORMALS) {
                    // outward normal of the solid
                    F3 ns = front ? N : f3(-N.x, -N.y, -N.z);
                    radiance = f3(0.5f * (ns.x + 1.0f), 0.5f * (ns.y + 1.0f), 0.5f * (ns.z + 1.0f));
                    end = true;
                } else {
                    const WoMaterial m = mats[L.u0];
                    F3 nd;
                    F3 att;
                    bool scatter = true;
                    if (m.kind == WO_MAT_LAMBERTIAN) {
                        F3 ru = unit3(random_in_unit_sphere(rng));
                        F3 sd = f3(N.x + ru.x, N.y + ru.y, N.z + ru.z);
                        if (fabsf(sd.x) < 1e-8f && fabsf(sd.y) < 1e-8f && fabsf(sd.z) < 1e-8f) sd = N;
                        nd = unit3(sd);
                        att = f3(m.albedo[0], m.albedo[1], m.albedo[2]);
                    } else if (m.kind == WO_MAT_METAL) {
                        float k = 2.0f * dot3(d, N);
                        F3 rs = random_in_unit_sphere(rng);
                        F3 sc = f3((d.x - k * N.x) + m.fuzz * rs.x, (d.y - k * N.y) + m.fuzz * rs.y,
                                   (d.z - k * N.z) + m.fuzz * rs.z);
                        scatter = dot3(sc, N) > 0.0f;
                        nd = unit3(sc);
                        att = f3(m.albedo[0], m.albedo[1], m.albedo[2]);
                    } else {
                        float ri = front ? (1.0f / m.ior) : m.ior;
                        float ct = dot3(f3(-d.x, -d.y, -d.z), N);
                        ct = ct < 1.0f ? ct : 1.0f;
                        float st = sqrtf(1.0f - ct * ct);
                        bool reflect = ri * st > 1.0f;
                        if (!reflect) {
                            float r0 = (1.0f - ri) / (1.0f + ri);
                            r0 = r0 * r0;
                            float x = 1.0f - ct;
                            float x5 = (((x * x) * x) * x) * x;
                            float refl = r0 + (1.0f - r0) * x5;
                            reflect = refl > rng.uniform();
                        }
                        F3 sc;
                        if (reflect) {
                            float k = 2.0f * dot3(d, N);
                            sc = f3(d.x - k * N.x, d.y - k * N.y, d.z - k * N.z);
                        } else {
                            F3 perp = f3(ri * (d.x + ct * N.x), ri * (d.y + ct * N.y), ri * (d.z + ct * N.z));
                            float par = -sqrtf(fabsf(1.0f - dot3(perp, perp)));
                            sc = f3(perp.x + par * N.x, perp.y + par * N.y, perp.z + par * N.z);
                        }
                        nd = unit3(sc);
                        att = f3(1.0f, 1.0f, 1.0f);
                    }
                    if (!scatter) {
                        end = true;
                    } else {
                        thr = f3(thr.x * att.x, thr.y * att.y, thr.z * att.z);
                        o = P;
                        d = nd;
                        ++depth;
                        if (depth >= max_depth) end = true;
                    }
                }
            }
            if (end) {
                acc = f3(acc.x + radiance.x, acc.y + radiance.y, acc.z + radiance.z);
                ++sample;
                if (sample >= spp)
                    done = true;
                else
                    start_sample();
            }
        }
    }

    if (active) {
        float fs = (float)spp;
        out[(size_t)lrow * W + lx] = make_float4(acc.x / fs, acc.y / fs, acc.z / fs, 1.0f);
    }
    if (seg_out != nullptr) {
        unsigned long long v = segs;
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (lane == 0u && v != 0ull) atomicAdd(seg_out, v);
    }
}

__global__ __launch_bounds__(kBlock) void assemble_kernel(const float4* __restrict__ gathered, float4* __restrict__ frame,
                                                          uint32_t W, uint32_t H, uint32_t T, uint32_t N,
                                                          uint32_t local_rows) {
    size_t total = (size_t)W * H;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < total; i += (size_t)gridDim.x * kBlock) {
        uint32_t y = (uint32_t)(i / W), x = (uint32_t)(i - (size_t)y * W);
        uint32_t g = y / T;
        uint32_t r = g % N;
        uint32_t lrow = (g / N) * T + (y - g * T);
        frame[i] = gathered[((size_t)r * local_rows + lrow) * W + x];
    }
}

}  // namespace

// ===========================================================================
// Host glue (C ABI declared in wo_dev.h)
// ===========================================================================
struct WoDev {
    int device;
    WoRec* d_prog;
    size_t prog_cap;
    WoMaterial* d_mats;
    size_t mats_cap;
    uint32_t n_recs, n_prims, n_mats;
    float4* d_frame;
    size_t frame_cap;
    hipStream_t stream;
};

static void set_err(char* err, size_t len, const char* what, hipError_t e) {
    if (err && len) snprintf(err, len, "%s: %s", what, hipGetErrorString(e));
}

extern "C" int wo_dev_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

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
    WoDev* dev = (WoDev*)calloc(1, sizeof(WoDev));
    if (!dev) {
        snprintf(err, errlen, "out of host memory");
        return -1;
    }
    dev->device = device;
    e = hipStreamCreateWithFlags(&dev->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipStreamCreate", e);
        free(dev);
        return -1;
    }
    *out = dev;
    return 0;
}

extern "C" void wo_dev_destroy(WoDev* dev) {
    if (!dev) return;
    (void)hipSetDevice(dev->device);
    (void)hipStreamSynchronize(dev->stream);
    if (dev->d_prog) (void)hipFree(dev->d_prog);
    if (dev->d_mats) (void)hipFree(dev->d_mats);
    if (dev->d_frame) (void)hipFree(dev->d_frame);
    (void)hipStreamDestroy(dev->stream);
    free(dev);
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

extern "C" int wo_dev_upload_scene(WoDev* dev, WoRec const* prog, uint32_t n_recs, uint32_t n_prims,
                                   WoMaterial const* mats, uint32_t n_mats, char* err, size_t errlen) {
    hipError_t e = hipSetDevice(dev->device);
    if (e != hipSuccess) {
        set_err(err, errlen, "hipSetDevice", e);
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
    return 0;
}

static const size_t kLdsBudget = 64u * 1024u;

extern "C" int wo_dev_launch(WoDev* dev, WoFrame const* frame_in, void* d_out, void* stream_v,
                             unsigned long long* d_segments, char* err, size_t errlen) {
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
    uint32_t local_rows = wo_rank_local_rows(fr.height, fr.tile_rows, fr.nranks);
    float4* out = (float4*)d_out;

    if (fr.mode == WO_MODE_UBERSHADER_RT1 || fr.mode == WO_MODE_DEBUG_ST) {
        dim3 grid((fr.width + kBlock - 1) / kBlock, local_rows);
        hipLaunchKernelGGL(ubershader_kernel, grid, dim3(kBlock), 0, stream, fr, local_rows, out);
    } else if (fr.mode == WO_MODE_PATHTRACE || fr.mode == WO_MODE_NORMALS) {
        if (fr.n_prims >= (1u << 20)) {
            snprintf(err, errlen, "scene has %u primitives (max %u)", fr.n_prims, (1u << 20) - 1u);
            return -1;
        }
        KLayout lay;
        lay.codes_words = (fr.n_recs + 7u) / 8u + 1u;
        lay.ordpc_off = lay.codes_words;
        uint32_t hib_words = fr.n_prims > 64u ? (fr.n_prims - 64u + 31u) / 32u : 0u;
        lay.hib_off = lay.ordpc_off + fr.n_prims;
        lay.wave_words = (lay.hib_off + hib_words * 64u + 3u) & ~3u;
        size_t scratch = (size_t)(kBlock / 64u) * lay.wave_words * 4u;
        size_t prog_bytes = (size_t)fr.n_recs * sizeof(WoRec);
        dim3 grid((fr.width + kPtTile - 1) / kPtTile, (local_rows + kPtTile - 1) / kPtTile);
        if (prog_bytes + scratch <= kLdsBudget) {
            hipLaunchKernelGGL(pathtrace_kernel<true>, grid, dim3(kBlock), prog_bytes + scratch, stream, dev->d_prog,
                               dev->d_mats, fr, lay, local_rows, out, d_segments);
        } else if (scratch <= kLdsBudget) {
            hipLaunchKernelGGL(pathtrace_kernel<false>, grid, dim3(kBlock), scratch, stream, dev->d_prog, dev->d_mats,
                               fr, lay, local_rows, out, d_segments);
        } else {
            snprintf(err, errlen, "scene too large for the LDS scratch (%zu bytes per workgroup)", scratch);
            return -1;
        }
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

extern "C" int wo_dev_assemble(void const* d_gathered, void* d_frame, uint32_t width, uint32_t height,
                               uint32_t tile_rows, uint32_t nranks, void* stream, char* err, size_t errlen) {
    if (tile_rows == 0 || nranks == 0) {
        snprintf(err, errlen, "bad tiling");
        return -1;
    }
    uint32_t local_rows = wo_rank_local_rows(height, tile_rows, nranks);
    size_t total = (size_t)width * height;
    uint32_t blocks = (uint32_t)((total + kBlock - 1) / kBlock);
    if (blocks > 8192u) blocks = 8192u;
    if (blocks == 0) return 0;
    hipLaunchKernelGGL(assemble_kernel, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream,
                       (const float4*)d_gathered, (float4*)d_frame, width, height, tile_rows, nranks, local_rows);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_err(err, errlen, "assemble launch", e);
        return -1;
    }
    return 0;
}
