/* wololo/wololo.h -- umbrella include (ref: src/wololo/wololo.h:1-6). */
#ifndef WOLOLO_WOLOLO_H
#define WOLOLO_WOLOLO_H

#include <stdbool.h>
#include <stdint.h>

#include "app.h"

#endif /* WOLOLO_WOLOLO_H */
