/*
 * app.c -- the wololo application loop, headless.
 *
 * Reference: src/wololo/app.c.  Same singleton (app.c:43-56), same callback
 * order (init -> loop {fixed-step updates, stats, draw_frame} -> de-init),
 * same fixed-timestep accumulator (app.c:140-155) and 1 Hz frame-time report
 * (app.c:156-194).  Differences:
 *   - no window system: the loop runs WOLOLO_FRAMES frames (default 60)
 *     instead of "until the window closes" (app.c:136);
 *   - a second wo_app_new() returns NULL instead of asserting;
 *   - the report uses the real mean (ref truncates the sum to size_t, app.c:171)
 *     and a real standard deviation (ref prints the variance, app.c:178-181).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "wo_internal.h"
#include "wololo/app.h"

struct Wo_App {
    Wo_InitCallbackPtr init_cb;
    Wo_UpdateCallbackPtr update_cb;
    Wo_DeInitCallbackPtr deinit_cb;
    Wo_Renderer* renderer;
    double updates_per_sec;
    double update_time_sec;
    uint32_t width, height;
    char* caption;
    double t_start;
    int running;
};

static int g_app_in_use = 0;
static struct Wo_App g_app;

Wo_App* wo_app_new(double target_updates_per_sec, uint32_t window_width, uint32_t window_height,
                   char const* window_caption, Wo_InitCallbackPtr opt_init_cb, Wo_UpdateCallbackPtr opt_update_cb,
                   Wo_DeInitCallbackPtr opt_de_init_cb) {
    if (g_app_in_use) {
        fprintf(stderr, WO_LOG_PREFIX " wo_app_new: the app is a singleton and is already in use.\n");
        return NULL;
    }
    g_app_in_use = 1;
    memset(&g_app, 0, sizeof g_app);
    g_app.init_cb = opt_init_cb;
    g_app.update_cb = opt_update_cb;
    g_app.deinit_cb = opt_de_init_cb;
    g_app.width = window_width;
    g_app.height = window_height;
    if (window_caption) {
        size_t n = strlen(window_caption);
        g_app.caption = (char*)malloc(n + 1);
        if (g_app.caption) memcpy(g_app.caption, window_caption, n + 1);
    }
    g_app.updates_per_sec = target_updates_per_sec > 0.0 ? target_updates_per_sec : 60.0;
    g_app.update_time_sec = 1.0 / g_app.updates_per_sec;
    g_app.t_start = wo_monotonic_sec();
    return &g_app;
}

double wo_app_time_sec(Wo_App* app) { return app ? wo_monotonic_sec() - app->t_start : 0.0; }
uint32_t wo_app_window_width(Wo_App* app) { return app ? app->width : 0u; }
uint32_t wo_app_window_height(Wo_App* app) { return app ? app->height : 0u; }
GLFWwindow* wo_app_glfw_window(Wo_App* app) {
    (void)app;
    return NULL;
}
void wo_app_swap_scene(Wo_App* app_ref, Wo_Renderer* new_scene_renderer) {
    if (app_ref) app_ref->renderer = new_scene_renderer;
}

static long frames_to_run(void) {
    const char* v = getenv("WOLOLO_FRAMES");
    if (v && *v) {
        long n = strtol(v, NULL, 10);
        if (n >= 0) return n;
    }
    return 60;
}

bool wo_app_run(Wo_App* app) {
    if (!app) return false;
    app->t_start = wo_monotonic_sec();
    if (app->init_cb) {
        if (!app->init_cb(app, app->width, app->height, app->caption ? app->caption : "", app->update_time_sec)) {
            printf("- Extension init failed.\n");
            return false;
        }
        printf("Initializing '%s' {w=%u, h=%u} @ %lf updates per second\n", app->caption ? app->caption : "",
               app->width, app->height, app->updates_per_sec);
    }
    const long frames = frames_to_run();
    const double report_every = 1.0;
    double last = wo_monotonic_sec() - app->t_start;
    double behind = 0.0;
    long reports = 1;
    /* Welford running statistics of the frame time */
    long n = 0;
    double mean = 0.0, m2 = 0.0;
    app->running = 1;
    for (long f = 0; f < frames; ++f) {
        double now = wo_monotonic_sec() - app->t_start;
        double dt = now - last;
        last = now;
        behind += dt;
        while (app->update_cb && behind >= app->update_time_sec) {
            behind -= app->update_time_sec;
            app->update_cb(app, app->update_time_sec);
        }
        ++n;
        double delta = dt - mean;
        mean += delta / (double)n;
        m2 += delta * (dt - mean);
        if (now > (double)reports * report_every) {
            ++reports;
            double sd = n > 1 ? sqrt(m2 / (double)(n - 1)) : 0.0;
            printf("[Wololo][Stats] | %ld frames / %.3lf sec = %.3lf fps | Avg. Frame-Time: %.6lf sec | Stddev. "
                   "Frame-Time: %.6lf |\n",
                   n, report_every, (double)n / report_every, mean, sd);
            n = 0;
            mean = m2 = 0.0;
        }
        if (app->renderer) wo_renderer_draw_frame(app->renderer);
    }
    app->running = 0;
    if (app->deinit_cb) app->deinit_cb(app);
    return true;
}
