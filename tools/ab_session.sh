#!/usr/bin/env bash
# Round-2 A/B session: spatial collect leaf size and event window on the chain.
S=tools/gpu_session.sh
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-count-work"
bash $S \
 "ch8:200:$B --scene csg256_chain > gpurun_out/ab_ch8.json" \
 "ch12:200:WOLOLO_JIT_SPATIAL_LEAF=12 $B --scene csg256_chain > gpurun_out/ab_ch12.json" \
 "ch16:200:WOLOLO_JIT_SPATIAL_LEAF=16 $B --scene csg256_chain > gpurun_out/ab_ch16.json" \
 "ch6:200:WOLOLO_JIT_SPATIAL_LEAF=6 $B --scene csg256_chain > gpurun_out/ab_ch6.json" \
 "ch8lds:200:WOLOLO_JIT_LDS_EVENTS=1 WOLOLO_JIT_SPATIAL=1 $B --scene csg256_chain > gpurun_out/ab_ch8lds.json" \
 "ch8w6:200:WOLOLO_JIT_FLAGS=-DWO_WINDOW=6 $B --scene csg256_chain > gpurun_out/ab_ch8w6.json" \
 "ch8w4:200:WOLOLO_JIT_FLAGS=-DWO_WINDOW=4 $B --scene csg256_chain > gpurun_out/ab_ch8w4.json" \
 "ch8b:200:$B --scene csg256_chain > gpurun_out/ab_ch8b.json"
