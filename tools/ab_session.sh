#!/usr/bin/env bash
# Round-2 A/B session: union count with popcounted single-primitive terms (no spills).
S=tools/gpu_session.sh
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-count-work"
bash $S \
 "bal_uc:200:$B --scene csg256_balanced > gpurun_out/ab_bal_uc.json" \
 "bal_nouc:200:WOLOLO_JIT_UNION_COUNT=0 $B --scene csg256_balanced > gpurun_out/ab_bal_nouc.json" \
 "bal_uc2:200:$B --scene csg256_balanced > gpurun_out/ab_bal_uc2.json" \
 "c32:200:$B > gpurun_out/ab_c32.json" \
 "c32_nouc:200:WOLOLO_JIT_UNION_COUNT=0 $B > gpurun_out/ab_c32_nouc.json" \
 "c32b:200:$B > gpurun_out/ab_c32b.json" \
 "c32_noucb:200:WOLOLO_JIT_UNION_COUNT=0 $B > gpurun_out/ab_c32_noucb.json" \
 "pw:200:bash tools/profile_session.sh csg256b_jit --scene csg256_balanced --steps 5 --warmup 1" \
 "par:400:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k 'balanced or csg32 or knobs'"
