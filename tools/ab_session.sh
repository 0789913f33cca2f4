#!/usr/bin/env bash
# Round-2 knob check: operator-aware term units in the spatial collect (WOLOLO_JIT_SPATIAL_UNITS).
bash tools/env_ab.sh \
 "csg256_balanced|WOLOLO_JIT_SPATIAL=0" \
 "csg256_balanced|WOLOLO_JIT_SPATIAL=1 WOLOLO_JIT_SPATIAL_UNITS=1" \
 "csg256_balanced|WOLOLO_JIT_SPATIAL=1 WOLOLO_JIT_SPATIAL_UNITS=1 WOLOLO_JIT_SPATIAL_LEAF=4" \
 "csg256_balanced|WOLOLO_JIT_SPATIAL=0" \
 "csg256_balanced|WOLOLO_JIT_SPATIAL=1 WOLOLO_JIT_SPATIAL_UNITS=1" \
 "csg32|WOLOLO_JIT_SPATIAL=1" \
 "csg32|WOLOLO_JIT_SPATIAL=1 WOLOLO_JIT_SPATIAL_UNITS=1"
timeout -k 10 400 env WOLOLO_JIT_SPATIAL=1 WOLOLO_JIT_SPATIAL_UNITS=1 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "balanced or csg32" > gpurun_out/par_units.log 2>&1
echo "parity rc=$?"
tail -3 gpurun_out/par_units.log
