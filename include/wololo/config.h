/*
 * wololo/config.h -- compile-time configuration.
 *
 * The reference keeps WO_DEBUG and the CWD-relative SPIR-V paths here
 * (src/wololo/config.h:3-6).  There are no shader files any more: the per-pixel
 * programs are HIP kernels linked into libwololo.so, so only the debug switch and
 * the runtime knobs remain.
 */
#ifndef WOLOLO_CONFIG_H
#define WOLOLO_CONFIG_H

#ifndef WO_DEBUG
#define WO_DEBUG (1)
#endif

/* Log prefix used by every library message (ref: renderer.c "[Wololo] ..."). */
#define WO_LOG_PREFIX "[Wololo]"

#endif /* WOLOLO_CONFIG_H */
