#!/usr/bin/env bash
# Round-2 knob re-check: balanced BOUND subtree size, csg32 tail rounds (pairs on one box).
bash tools/env_ab.sh \
 "csg256_balanced|WOLOLO_JIT_BOUND_MIN_LEAVES=6" \
 "csg256_balanced|WOLOLO_JIT_BOUND_MIN_LEAVES=4" \
 "csg256_balanced|WOLOLO_JIT_BOUND_MIN_LEAVES=3" \
 "csg256_balanced|WOLOLO_JIT_BOUND_MIN_LEAVES=5" \
 "csg256_balanced|WOLOLO_JIT_BOUND_MIN_LEAVES=6" \
 "csg256_balanced|WOLOLO_JIT_BOUND_MIN_LEAVES=4" \
 "csg32|WOLOLO_JIT_SPATIAL_LEAF=8" \
 "csg32|WOLOLO_TILE_TAIL=4" \
 "csg32|WOLOLO_TILE_TAIL=3" \
 "csg32|WOLOLO_JIT_SPATIAL_LEAF=8" \
 "csg32|WOLOLO_TILE_TAIL=4" \
 "csg32|WOLOLO_JIT_UNION_COUNT=0" \
 "csg32|WOLOLO_JIT_SPATIAL_LEAF=8"
