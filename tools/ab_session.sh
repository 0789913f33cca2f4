#!/usr/bin/env bash
# Round-2 A/B session: spatial collect (surface-area splits) on csg32.
S=tools/gpu_session.sh
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-count-work"
bash $S \
 "c32:200:WOLOLO_JIT_SPATIAL=0 $B > gpurun_out/ab_c32.json" \
 "c32_sp:200:WOLOLO_JIT_SPATIAL=1 $B > gpurun_out/ab_c32_sp.json" \
 "c32_sp4:200:WOLOLO_JIT_SPATIAL=1 WOLOLO_JIT_SPATIAL_LEAF=4 $B > gpurun_out/ab_c32_sp4.json" \
 "c32_sp6:200:WOLOLO_JIT_SPATIAL=1 WOLOLO_JIT_SPATIAL_LEAF=6 $B > gpurun_out/ab_c32_sp6.json" \
 "c32_sp3:200:WOLOLO_JIT_SPATIAL=1 WOLOLO_JIT_SPATIAL_LEAF=3 $B > gpurun_out/ab_c32_sp3.json" \
 "c32b:200:WOLOLO_JIT_SPATIAL=0 $B > gpurun_out/ab_c32b.json" \
 "c32_spb:200:WOLOLO_JIT_SPATIAL=1 $B > gpurun_out/ab_c32_spb.json" \
 "c4:300:WOLOLO_JIT_SPATIAL=0 python bench.py --width 3840 --height 2160 --spp 256 --steps 3 --warmup 1 --no-cpu-baseline --no-count-work > gpurun_out/ab_c4.json" \
 "c4_sp:300:WOLOLO_JIT_SPATIAL=1 python bench.py --width 3840 --height 2160 --spp 256 --steps 3 --warmup 1 --no-cpu-baseline --no-count-work > gpurun_out/ab_c4_sp.json" \
 "par:500:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k 'knobs or chain'"
