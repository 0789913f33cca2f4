tools/gpu_session.sh \
"rt_base:150:python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/rt_base.json" \
"rt_s16:150:WOLOLO_LANES_STACK16=1 python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/rt_s16.json" \
"rt_s16_t200:150:WOLOLO_LANES_STACK16=1 WOLOLO_LANES_TOP=200 python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/rt_s16_t200.json" \
"rt_s16_tall:150:WOLOLO_LANES_STACK16=1 WOLOLO_LANES_TOP=600 python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/rt_s16_tall.json" \
"rt_tall:150:WOLOLO_LANES_TOP=600 python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/rt_tall.json" \
"rt_d0:150:WOLOLO_LANES_DEPTH=0 python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/rt_d0.json" \
"rt_w_tall:150:WOLOLO_LANES_WIDE=1 WOLOLO_LANES_TOP=600 python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/rt_w_tall.json"
