#!/usr/bin/env bash
# Round-2 A/B session: spatial collect (WOLOLO_JIT_SPATIAL, WOLOLO_JIT_SPATIAL_LEAF).
S=tools/gpu_session.sh
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-count-work"
bash $S \
 "ch_sp:200:$B --scene csg256_chain > gpurun_out/ab_ch_sp.json" \
 "ch_nosp:200:WOLOLO_JIT_SPATIAL=0 $B --scene csg256_chain > gpurun_out/ab_ch_nosp.json" \
 "ch_sp2:200:WOLOLO_JIT_SPATIAL_LEAF=2 $B --scene csg256_chain > gpurun_out/ab_ch_sp2.json" \
 "ch_sp8:200:WOLOLO_JIT_SPATIAL_LEAF=8 $B --scene csg256_chain > gpurun_out/ab_ch_sp8.json" \
 "bal_sp:200:WOLOLO_JIT_SPATIAL=1 $B --scene csg256_balanced > gpurun_out/ab_bal_sp.json" \
 "bal:200:$B --scene csg256_balanced > gpurun_out/ab_bal.json" \
 "c32_sp:200:WOLOLO_JIT_SPATIAL=1 $B > gpurun_out/ab_c32_sp.json" \
 "c32:200:$B > gpurun_out/ab_c32.json" \
 "par:500:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k 'chain or knobs'"
