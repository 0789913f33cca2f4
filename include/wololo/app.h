/*
 * wololo/app.h -- the application loop that drives the renderer.
 *
 * Same types and entry points as the reference (src/wololo/app.h:14-34).  The
 * app is a process-wide singleton (ref app.c:43-56): a second wo_app_new()
 * returns NULL here instead of asserting.
 *
 * Headless behaviour (this build has no window system by default): wo_app_run()
 * calls the init callback, then runs `WOLOLO_FRAMES` frames (environment
 * variable, default 60) through wo_renderer_draw_frame() of the scene installed
 * with wo_app_swap_scene(), printing the same 1 Hz frame-time report as the
 * reference (with the ref's integer-truncated mean and variance-as-stddev bugs,
 * app.c:171 / 178-181, fixed), then calls the de-init callback.
 */
#ifndef WOLOLO_APP_H
#define WOLOLO_APP_H

#include <stdbool.h>
#include <stdint.h>

#include "platform.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct Wo_Renderer Wo_Renderer;
typedef struct Wo_App Wo_App;

/* ref app.h:16-18 */
typedef bool (*Wo_InitCallbackPtr)(Wo_App* app, uint32_t window_width, uint32_t window_height,
                                   char const* window_caption, double target_frame_time_sec);
typedef void (*Wo_UpdateCallbackPtr)(Wo_App* app, double elapsed_time_in_sec);
typedef void (*Wo_DeInitCallbackPtr)(Wo_App* app);

/* ref app.h:20-27 / app.c:228-241 */
Wo_App* wo_app_new(double target_updates_per_sec, uint32_t window_width, uint32_t window_height,
                   char const* window_caption, Wo_InitCallbackPtr opt_init_cb,
                   Wo_UpdateCallbackPtr opt_update_cb, Wo_DeInitCallbackPtr opt_de_init_cb);
/* ref app.h:28 / app.c:243-245 */
bool wo_app_run(Wo_App* app_ref);
/* ref app.h:29 / app.c:247-249: borrows the renderer pointer. */
void wo_app_swap_scene(Wo_App* app_ref, Wo_Renderer* new_scene_renderer);
/* ref app.h:30 / app.c:251-253: NULL when running headless. */
GLFWwindow* wo_app_glfw_window(Wo_App* app);

/* ---- extensions (new names only) ---- */
/* Window size the app was created with (the renderer's default frame size). */
uint32_t wo_app_window_width(Wo_App* app);
uint32_t wo_app_window_height(Wo_App* app);
/* Seconds since wo_app_run() started (the reference uses glfwGetTime(), renderer.c:2136). */
double wo_app_time_sec(Wo_App* app);

#ifdef __cplusplus
}
#endif

#endif /* WOLOLO_APP_H */
