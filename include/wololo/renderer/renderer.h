/*
 * wololo/renderer/renderer.h -- the renderer + CSG scene C API.
 *
 * Drop-in replacement for the reference header src/wololo/renderer/renderer.h:14-33:
 * every type, name and signature below is the reference's, so code written
 * against the reference (src/wololo_demo/main.c) compiles and links unchanged.
 * Behind it, the Vulkan backend (renderer.c:394-2219) is replaced by HIP
 * kernels for gfx950.  Extensions live in renderer_ext.h.
 *
 * Node semantics (ref renderer.c:2220-2313):
 *   - handles are sequential uint32 indices starting at 0;
 *   - a binop marks both operands non-root; wo_renderer_isroot() reports the
 *     complement of that bitset;
 *   - the scene that gets rendered is the union of all root nodes.
 * Failure behaviour: wo_renderer_new() returns NULL (the reference intends
 * this but dereferences NULL first, renderer.c:334-335); adding a node past
 * max_node_count logs and returns WO_NODE_INVALID instead of aborting.
 */
#ifndef WOLOLO_RENDERER_RENDERER_H
#define WOLOLO_RENDERER_RENDERER_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#include "wololo/app.h"
#include "wololo/wmath.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct Wo_Renderer Wo_Renderer;
typedef uint32_t Wo_Node;      /* ref renderer.h:15 */
typedef uint32_t Wo_Material;  /* ref renderer.h:16 */

/* A placed operand of a CSG binop: the child node, rotated by `orientation`
 * and then translated by `offset` into the parent's frame (ref renderer.h:22-27).
 * 64 bytes, passed by value. */
typedef struct Wo_Node_Argument Wo_Node_Argument;
struct Wo_Node_Argument {
    Wo_Quaternion orientation;
    Wo_Vec3 offset;
    Wo_Node node;
};

/* ref renderer.h:18-20 */
Wo_Renderer* wo_renderer_new(Wo_App* app, char const* name, size_t max_node_count);
void wo_renderer_del(Wo_Renderer* renderer);
void wo_renderer_draw_frame(Wo_Renderer* renderer);

/* ref renderer.h:28-33 */
Wo_Node wo_renderer_add_sphere_node(Wo_Renderer* renderer, Wo_Scalar radius);
Wo_Node wo_renderer_add_infinite_planar_partition_node(Wo_Renderer* renderer, Wo_Vec3 outward_facing_normal);
Wo_Node wo_renderer_add_union_of_node(Wo_Renderer* renderer, Wo_Node_Argument left, Wo_Node_Argument right);
Wo_Node wo_renderer_add_intersection_of_node(Wo_Renderer* renderer, Wo_Node_Argument left, Wo_Node_Argument right);
Wo_Node wo_renderer_add_difference_of_node(Wo_Renderer* renderer, Wo_Node_Argument left, Wo_Node_Argument right);
bool wo_renderer_isroot(Wo_Renderer* renderer, Wo_Node node);

#ifdef __cplusplus
}
#endif

#endif /* WOLOLO_RENDERER_RENDERER_H */
