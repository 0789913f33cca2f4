#!/usr/bin/env bash
# Round-2 session: full GPU suite with the current kernels, csg32 with the union count forced.
S=tools/gpu_session.sh
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-count-work"
bash $S \
 "gt:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "c32:200:$B > gpurun_out/ab_c32.json" \
 "c32_uc:200:WOLOLO_JIT_UNION_COUNT=2 $B > gpurun_out/ab_c32_uc.json" \
 "c32b:200:$B > gpurun_out/ab_c32b.json" \
 "c32_ucb:200:WOLOLO_JIT_UNION_COUNT=2 $B > gpurun_out/ab_c32_ucb.json"
