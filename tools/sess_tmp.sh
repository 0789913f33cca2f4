tools/gpu_session.sh \
"rtg05:150:WOLOLO_LANES_GRID=1 WOLOLO_LANES_GRID_DENSITY=0.5 python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/rtg05.json" \
"rs_def:300:python tools/root_step.py --scene csg32 --worlds 8 > gpurun_out/rs_def.log 2>&1" \
"rs_84:300:WOLOLO_TILE=8x4 python tools/root_step.py --scene csg32 --worlds 8 > gpurun_out/rs_84.log 2>&1" \
"rs_88:300:WOLOLO_TILE=8x8 python tools/root_step.py --scene csg32 --worlds 8 > gpurun_out/rs_88.log 2>&1" \
"rs_tail2:300:WOLOLO_TILE_TAIL=1 python tools/root_step.py --scene csg32 --worlds 8 > gpurun_out/rs_tail1.log 2>&1"
