/*
 * present.c -- the headless present path: float framebuffer -> 8-bit sRGB.
 *
 * The reference presents through a swapchain whose format it picks as
 * B8G8R8A8_SRGB when available (renderer.c:813-832): the hardware clamps the
 * fragment output to [0, 1], applies the sRGB transfer function and quantises to
 * 8 bits.  Here the encode runs on the GPU (srgb8_kernel, trace_kernels.hip)
 * into the same B8G8R8A8 layout; this file holds its table and the PPM dump.
 *
 * Exactness: an 8-bit code is a count of thresholds.  Threshold j (0..254) is
 * the smallest float v with 255 * srgb(v) >= j + 0.5, srgb being the
 * IEC 61966-2-1 encode in double precision:
 *     srgb(v) = 12.92 v                    (v <= 0.0031308)
 *             = 1.055 v^(1/2.4) - 0.055    (otherwise)
 * so code(v) = round-half-up(255 * srgb(clamp(v, 0, 1))) for every float v,
 * with no per-pixel pow (NaN -> 0).  The table is found by bisection over the
 * float bit patterns, which are monotone for v >= 0.
 */
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "wo_internal.h"

static double srgb_encode_d(double v) {
    return v <= 0.0031308 ? 12.92 * v : 1.055 * pow(v, 1.0 / 2.4) - 0.055;
}

static float f_of_bits(uint32_t u) {
    float f;
    memcpy(&f, &u, sizeof f);
    return f;
}

static float g_srgb_table[255];
static pthread_once_t g_srgb_once = PTHREAD_ONCE_INIT;

static void build_srgb_table(void) {
    for (int j = 0; j < 255; ++j) {
        const double target = (j + 0.5) / 255.0;
        /* smallest bits b in (0, bits(1.0)] with srgb(f(b)) >= target */
        uint32_t lo = 0u, hi = 0x3f800000u; /* srgb(0) < target <= srgb(1) */
        while (hi - lo > 1u) {
            uint32_t mid = lo + (hi - lo) / 2u;
            if (srgb_encode_d((double)f_of_bits(mid)) >= target)
                hi = mid;
            else
                lo = mid;
        }
        g_srgb_table[j] = f_of_bits(hi);
    }
}

void wo_srgb8_thresholds(float out[255]) {
    (void)pthread_once(&g_srgb_once, build_srgb_table); /* built once, whatever thread asks first */
    memcpy(out, g_srgb_table, sizeof g_srgb_table);
}

/* Host form of the device encode (same table, same rule): used for the PPM
 * dump of frames rendered elsewhere and by tests. */
static uint8_t srgb8_code(float v, const float* t) {
    uint32_t k = 0;
    for (uint32_t s = 128u; s > 0u; s >>= 1)
        if (k + s <= 255u && t[k + s - 1u] <= v) k += s;
    return (uint8_t)k;
}

static uint8_t unorm8(float a) {
    if (!(a > 0.0f)) return 0;
    if (a >= 1.0f) return 255;
    return (uint8_t)((double)a * 255.0 + 0.5); /* exact in double: round-half-up */
}

void wo_srgb8_encode_host(float const* rgba, uint32_t* bgra8, size_t pixels) {
    float t[255];
    wo_srgb8_thresholds(t);
    for (size_t i = 0; i < pixels; ++i) {
        const float* p = rgba + 4 * i;
        bgra8[i] = (uint32_t)srgb8_code(p[2], t) | ((uint32_t)srgb8_code(p[1], t) << 8) |
                   ((uint32_t)srgb8_code(p[0], t) << 16) | ((uint32_t)unorm8(p[3]) << 24);
    }
}

int wo_write_ppm_bgra8(char const* path, uint32_t const* bgra8, uint32_t w, uint32_t h) {
    FILE* f = fopen(path, "wb");
    if (!f) {
        wo_set_error("cannot write %s", path);
        return -1;
    }
    int ok = fprintf(f, "P6\n%u %u\n255\n", w, h) > 0;
    unsigned char* row = (unsigned char*)malloc((size_t)w * 3 + 1);
    if (!row) ok = 0;
    for (uint32_t y = 0; ok && y < h; ++y) {
        for (uint32_t x = 0; x < w; ++x) {
            const uint32_t p = bgra8[(size_t)y * w + x];
            row[x * 3 + 0] = (unsigned char)(p >> 16); /* R */
            row[x * 3 + 1] = (unsigned char)(p >> 8);  /* G */
            row[x * 3 + 2] = (unsigned char)p;         /* B */
        }
        ok = fwrite(row, 1, (size_t)w * 3, f) == (size_t)w * 3;
    }
    free(row);
    if (fclose(f) != 0) ok = 0;
    if (!ok) {
        wo_set_error("short write to %s", path);
        return -1;
    }
    return 0;
}
