/*
 * Analysis build of the oracle (not test infrastructure, not the product):
 * records every traced ray (origin, direction, depth) of a single-threaded
 * render, for tools/stats/wave_coherence.py.
 */
#include <stdint.h>

static float* g_rays;  /* 8 floats per ray: o[3], d[3], depth, unused */
static uint64_t g_cap, g_n;
static uint32_t t_depth;

static void dump_ray(const float* o, const float* d) {
    if (g_n < g_cap) {
        float* r = g_rays + 8 * g_n;
        r[0] = o[0]; r[1] = o[1]; r[2] = o[2];
        r[3] = d[0]; r[4] = d[1]; r[5] = d[2];
        r[6] = (float)t_depth;
        r[7] = 0.0f;
    }
    ++g_n;
}

#define ORACLE_TRACE_HOOK(s, nev, swept, hit) dump_ray(o, d)
#define ORACLE_DEPTH_HOOK(depth) (t_depth = (depth))
#include "../../oracle/oracle.c"

void dump_set(float* buf, uint64_t cap) {
    g_rays = buf;
    g_cap = cap;
    g_n = 0;
}
uint64_t dump_count(void) { return g_n; }
