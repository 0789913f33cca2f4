/*
 * jit_cache.c -- persistent cache of the scene-specialised kernels' code objects.
 *
 * The reference compiles its shaders offline (top-shader-build.sh, glslc) and
 * loads the SPIR-V at startup (renderer.c:1811-1873).  Here the path tracer is
 * specialised per scene and compiled with hiprtc at scene upload (scene_jit.c),
 * which costs ~1 s for csg32 and 10+ s for csg256 on every process and every
 * rank.  This file keeps the code objects on disk, keyed by the SHA-256 of
 * everything that determines them (source, embedded headers, target, compile
 * options, hiprtc version: the key is computed in trace_kernels.hip), so a
 * second process or rank loads the object instead of compiling it.
 *
 * Location: $WOLOLO_JIT_CACHE (a directory; "0" or "" disables the cache), else
 * $XDG_CACHE_HOME/wololo/jit, else $HOME/.cache/wololo/jit; created 0700, and
 * not used unless it is owned by this user and writable by nobody else.
 * File: <key>.co = "WOJITCO1" | u64 size | SHA-256(code) | code.  Written to a
 * private temporary name and renamed into place, so concurrent writers (ranks
 * of one node) never expose a partial file; a reader checks the size and the
 * digest and treats any mismatch as a miss.
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include "wo_internal.h"

/* ---- SHA-256 (FIPS 180-4) ---- */
static const uint32_t kK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u,
};

static uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static void sha_block(WoSha256* s, const uint8_t* p) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
        w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
        uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = s->h[0], b = s->h[1], c = s->h[2], d = s->h[3], e = s->h[4], f = s->h[5], g = s->h[6], h = s->h[7];
    for (int i = 0; i < 64; ++i) {
        uint32_t t1 = h + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + kK[i] + w[i];
        uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + t2;
    }
    s->h[0] += a;
    s->h[1] += b;
    s->h[2] += c;
    s->h[3] += d;
    s->h[4] += e;
    s->h[5] += f;
    s->h[6] += g;
    s->h[7] += h;
}

void wo_sha256_init(WoSha256* s) {
    static const uint32_t h0[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    memcpy(s->h, h0, sizeof h0);
    s->len = 0;
    s->fill = 0;
}

void wo_sha256_update(WoSha256* s, const void* data, size_t n) {
    const uint8_t* p = (const uint8_t*)data;
    s->len += n;
    while (n > 0) {
        size_t k = 64u - s->fill;
        if (k > n) k = n;
        memcpy(s->buf + s->fill, p, k);
        s->fill += (uint32_t)k;
        p += k;
        n -= k;
        if (s->fill == 64u) {
            sha_block(s, s->buf);
            s->fill = 0;
        }
    }
}

void wo_sha256_final(WoSha256* s, uint8_t out[32]) {
    const uint64_t bits = s->len * 8u;
    const uint8_t one = 0x80u, zero = 0u;
    wo_sha256_update(s, &one, 1);
    while (s->fill != 56u) wo_sha256_update(s, &zero, 1);
    uint8_t lenb[8];
    for (int i = 0; i < 8; ++i) lenb[i] = (uint8_t)(bits >> (56 - 8 * i));
    wo_sha256_update(s, lenb, 8);
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(s->h[i] >> 24);
        out[4 * i + 1] = (uint8_t)(s->h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(s->h[i] >> 8);
        out[4 * i + 3] = (uint8_t)s->h[i];
    }
}

void wo_sha256_hex(const uint8_t d[32], char out[65]) {
    static const char hx[] = "0123456789abcdef";
    for (int i = 0; i < 32; ++i) {
        out[2 * i] = hx[d[i] >> 4];
        out[2 * i + 1] = hx[d[i] & 15];
    }
    out[64] = '\0';
}

/* ---- the cache directory ---- */
static int mkdir_p(const char* path) {
    char buf[1024];
    size_t n = strlen(path);
    if (n == 0 || n >= sizeof buf) return -1;
    memcpy(buf, path, n + 1);
    for (size_t i = 1; i <= n; ++i) {
        if (buf[i] == '/' || buf[i] == '\0') {
            char c = buf[i];
            buf[i] = '\0';
            if (mkdir(buf, 0700) != 0 && errno != EEXIST) return -1;
            buf[i] = c;
        }
    }
    return 0;
}

int wo_jit_cache_dir(char* out, size_t len) {
    const char* env = getenv("WOLOLO_JIT_CACHE");
    int n;
    if (env) {
        if (!*env || strcmp(env, "0") == 0) return -1;
        n = snprintf(out, len, "%s", env);
    } else {
        const char* xdg = getenv("XDG_CACHE_HOME");
        const char* home = getenv("HOME");
        if (xdg && *xdg)
            n = snprintf(out, len, "%s/wololo/jit", xdg);
        else if (home && *home)
            n = snprintf(out, len, "%s/.cache/wololo/jit", home);
        else
            return -1;
    }
    if (n <= 0 || (size_t)n >= len) return -1;
    if (mkdir_p(out)) return -1;
    /* Every object in the directory is loaded and run as GPU code: refuse one
     * that another user owns or that others can write to (an existing private
     * cache created with 0755 is fine; new directories are created 0700). */
    struct stat st;
    if (stat(out, &st) != 0 || !S_ISDIR(st.st_mode) || st.st_uid != geteuid() || (st.st_mode & 022)) {
        static int warned;
        if (!__atomic_exchange_n(&warned, 1, __ATOMIC_RELAXED))
            fprintf(stderr, WO_LOG_PREFIX " code-object cache %s is not a private directory of this user; "
                            "cache off\n", out);
        return -1;
    }
    return 0;
}

static const char kMagic[8] = {'W', 'O', 'J', 'I', 'T', 'C', 'O', '1'};

int wo_jit_disk_load(const char* key_hex, void** code, size_t* size) {
    char dir[900], path[1024];
    *code = NULL;
    *size = 0;
    if (wo_jit_cache_dir(dir, sizeof dir)) return -1;
    snprintf(path, sizeof path, "%s/%s.co", dir, key_hex);
    FILE* f = fopen(path, "rb");
    if (!f) return -1;
    char magic[8];
    uint64_t n = 0;
    uint8_t want[32], got[32];
    void* buf = NULL;
    int ok = fread(magic, 1, 8, f) == 8 && memcmp(magic, kMagic, 8) == 0 && fread(&n, sizeof n, 1, f) == 1 &&
             n > 0 && n < (1ull << 30) && fread(want, 1, 32, f) == 32;
    if (ok) {
        buf = malloc((size_t)n);
        ok = buf && fread(buf, 1, (size_t)n, f) == (size_t)n && fgetc(f) == EOF;
    }
    fclose(f);
    if (ok) {
        WoSha256 s;
        wo_sha256_init(&s);
        wo_sha256_update(&s, buf, (size_t)n);
        wo_sha256_final(&s, got);
        ok = memcmp(got, want, 32) == 0;
    }
    if (!ok) {
        free(buf);
        return -1;
    }
    *code = buf;
    *size = (size_t)n;
    return 0;
}

int wo_jit_disk_store(const char* key_hex, const void* code, size_t size) {
    char dir[900], path[1024], tmp[1100];
    if (wo_jit_cache_dir(dir, sizeof dir)) return -1;
    snprintf(path, sizeof path, "%s/%s.co", dir, key_hex);
    static unsigned counter;
    snprintf(tmp, sizeof tmp, "%s.tmp.%ld.%u", path, (long)getpid(), __atomic_fetch_add(&counter, 1u, __ATOMIC_RELAXED));
    FILE* f = fopen(tmp, "wb");
    if (!f) return -1;
    uint8_t dg[32];
    WoSha256 s;
    wo_sha256_init(&s);
    wo_sha256_update(&s, code, size);
    wo_sha256_final(&s, dg);
    const uint64_t n = size;
    int ok = fwrite(kMagic, 1, 8, f) == 8 && fwrite(&n, sizeof n, 1, f) == 1 && fwrite(dg, 1, 32, f) == 32 &&
             fwrite(code, 1, size, f) == size;
    if (fclose(f) != 0) ok = 0;
    if (!ok || rename(tmp, path) != 0) {
        (void)unlink(tmp);
        return -1;
    }
    return 0;
}
