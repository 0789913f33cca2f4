#!/usr/bin/env bash
# Round-2 session: full GPU suite, then evidence for the kernels the spatial collect changed.
S=tools/gpu_session.sh
bash $S \
 "gt:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "p32:400:bash tools/profile_session.sh csg32_jit --steps 10 --warmup 2" \
 "pc4:500:bash tools/profile_session.sh c4_jit --width 3840 --height 2160 --spp 256 --steps 3 --warmup 1" \
 "rs32:200:python tools/rank_share.py --scene csg32 --worlds 1 2 4 8 --reps 5 > gpurun_out/r02_share32.log 2>&1" \
 "rs4k:300:python tools/rank_share.py --scene csg32 --width 3840 --height 2160 --spp 256 --worlds 1 8 --reps 3 > gpurun_out/r02_share4k.log 2>&1" \
 "bal_sp4:200:WOLOLO_JIT_SPATIAL=1 WOLOLO_JIT_SPATIAL_LEAF=4 python bench.py --scene csg256_balanced --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/ab_bal_sp4.json" \
 "bal_sp16:200:WOLOLO_JIT_SPATIAL=1 WOLOLO_JIT_SPATIAL_LEAF=16 python bench.py --scene csg256_balanced --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/ab_bal_sp16.json" \
 "bal:200:python bench.py --scene csg256_balanced --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/ab_bal.json"
