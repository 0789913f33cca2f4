/* Compatibility shim for src/wololo/wmath.impl.h; see wmath.decl.h. */
#ifndef WOLOLO_WMATH_IMPL_H
#define WOLOLO_WMATH_IMPL_H
#include "wmath.h"
#endif
