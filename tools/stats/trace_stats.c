/*
 * Analysis build of the oracle (not test infrastructure, not the product):
 * oracle.c compiled with ORACLE_TRACE_HOOK counting, per trace, the events
 * collected and the events swept before the hit.  Used by tools/trace_stats.py
 * to size the event window and to see where the sweep spends its evaluations.
 */
#include <stdint.h>

static uint64_t g_stats[32];
static __thread uint32_t t_depth;

static void stats_hook(uint32_t nev, uint32_t swept, int hit) {
    if (t_depth > 0) {
#pragma omp atomic
        g_stats[16] += 1; /* secondary traces */
#pragma omp atomic
        g_stats[17] += (uint64_t)hit;
#pragma omp atomic
        g_stats[18] += nev;
#pragma omp atomic
        g_stats[19] += swept;
    }
    uint32_t bin = swept == 0 ? 0 : swept == 1 ? 1 : swept == 2 ? 2 : swept <= 4 ? 3 : swept <= 8 ? 4 : 5;
#pragma omp atomic
    g_stats[0] += 1; /* traces */
#pragma omp atomic
    g_stats[1] += (uint64_t)hit;
#pragma omp atomic
    g_stats[2] += nev;
#pragma omp atomic
    g_stats[3] += swept;
#pragma omp atomic
    g_stats[4 + bin] += 1; /* swept histogram: 0, 1, 2, 3-4, 5-8, 9+ */
#pragma omp atomic
    g_stats[10] += (uint64_t)(swept > 4u || (!hit && nev > 4u)); /* window-4 re-collects needed */
#pragma omp atomic
    g_stats[11] += (uint64_t)(nev > 4u);
}

#define ORACLE_TRACE_HOOK(s, nev, swept, hit) stats_hook((nev), (swept), (hit))
#define ORACLE_DEPTH_HOOK(depth) (t_depth = (depth))
#include "../../oracle/oracle.c"

void stats_get(uint64_t out[32]) {
    for (int i = 0; i < 32; ++i) out[i] = g_stats[i];
}
void stats_reset(void) {
    for (int i = 0; i < 32; ++i) g_stats[i] = 0;
}
