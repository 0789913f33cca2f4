cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_session.sh \
 "bc4:300:python bench.py --width 3840 --height 2160 --spp 256 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ev_bench_c4.json" \
 "rs4k:300:python tools/rank_share.py --scene csg32 --width 3840 --height 2160 --spp 256 --worlds 1 8 --reps 3 > gpurun_out/ev_share4k.log 2>&1" \
 "ab:600:bash tools/env_ab.sh 'csg32|WOLOLO_JIT_BOUND_MIN_LEAVES=6' 'csg32|WOLOLO_JIT_BOUND_MIN_LEAVES=4' 'csg32|WOLOLO_JIT_BOUND_MIN_LEAVES=5' 'csg32|WOLOLO_JIT_BOUND_MIN_LEAVES=7' 'csg32|WOLOLO_JIT_BOUND_MIN_LEAVES=8' 'csg32|WOLOLO_JIT_FLAGS=-DWO_LDS_EVENTS=6' 'csg32|WOLOLO_JIT_FLAGS=-DWO_LDS_EVENTS=8' 'csg32|WOLOLO_BOUND_MIN_LEAVES=3' 'csg256_balanced|WOLOLO_JIT_BOUND_MIN_LEAVES=6' 'csg256_balanced|WOLOLO_JIT_BOUND_MIN_LEAVES=4' 'csg256_balanced|WOLOLO_JIT_BOUND_MIN_LEAVES=8' 'csg32|WOLOLO_JIT_BOUND_MIN_LEAVES=6'"
