/* Compatibility shim: the reference splits its math header into decl/impl
 * (src/wololo/wmath.decl.h, src/wololo/wmath.impl.h).  Both names resolve to
 * the single header here so either include keeps compiling. */
#ifndef WOLOLO_WMATH_DECL_H
#define WOLOLO_WMATH_DECL_H
#include "wmath.h"
#endif
