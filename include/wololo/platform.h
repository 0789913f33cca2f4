/*
 * wololo/platform.h -- window-system glue.
 *
 * The reference pulls in <vulkan/vulkan.h> and <GLFW/glfw3.h> here
 * (src/wololo/platform.h:3-5).  This build has no Vulkan at all (the renderer
 * runs on HIP), and GLFW is optional: define WOLOLO_WITH_GLFW to include the
 * real header, otherwise `GLFWwindow` stays an opaque forward declaration so
 * `app.h` (which exposes `GLFWwindow*`, ref app.h:34) still compiles headless.
 */
#ifndef WOLOLO_PLATFORM_H
#define WOLOLO_PLATFORM_H

#if defined(WOLOLO_WITH_GLFW)
#include <GLFW/glfw3.h>
#else
typedef struct GLFWwindow GLFWwindow;
#endif

#endif /* WOLOLO_PLATFORM_H */
