#!/usr/bin/env bash
# Round-2 A/B session: the union count's term table in LDS (csg32).
S=tools/gpu_session.sh
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-count-work"
bash $S \
 "c32:200:$B > gpurun_out/ab_c32.json" \
 "c32_g:200:WOLOLO_JIT_LDS_UTERM=0 $B > gpurun_out/ab_c32_g.json" \
 "c32b:200:$B > gpurun_out/ab_c32b.json" \
 "c32_gb:200:WOLOLO_JIT_LDS_UTERM=0 $B > gpurun_out/ab_c32_gb.json" \
 "bal_l:200:WOLOLO_JIT_LDS_UTERM=1 python bench.py --scene csg256_balanced --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/ab_bal_l.json" \
 "bal:200:python bench.py --scene csg256_balanced --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/ab_bal.json" \
 "par:500:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k 'csg32 or knobs'"
