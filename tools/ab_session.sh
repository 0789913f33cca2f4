#!/usr/bin/env bash
# Round-2 final session: full GPU suite, smoke, csg256 balanced evidence (BOUNDs from 4 leaves).
S=tools/gpu_session.sh
bash $S \
 "gt:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:300:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "b256b:200:python bench.py --scene csg256_balanced --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02_bench_256b.json" \
 "p256b:400:bash tools/profile_session.sh csg256b_jit --scene csg256_balanced --steps 5 --warmup 1" \
 "rs256b:300:python tools/rank_share.py --scene csg256_balanced --worlds 1 8 --reps 3 > gpurun_out/r02_share256b.log 2>&1"
