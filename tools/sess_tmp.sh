tools/gpu_session.sh \
"b32:150:python bench.py --scene csg32 --steps 20 --warmup 3 --no-cpu-baseline --no-count-work > gpurun_out/b32.json" \
"b32_nofc:150:WOLOLO_JIT_FLAGS=-DWO_FRAME_SCALAR_COPIES=0 python bench.py --scene csg32 --steps 20 --warmup 3 --no-cpu-baseline --no-count-work > gpurun_out/b32_nofc.json" \
"b32_kv:150:WOLOLO_JIT_KEY_VMOV=1 python bench.py --scene csg32 --steps 20 --warmup 3 --no-cpu-baseline --no-count-work > gpurun_out/b32_kv.json" \
"b32b:150:python bench.py --scene csg32 --steps 20 --warmup 3 --no-cpu-baseline --no-count-work > gpurun_out/b32b.json" \
"bch:150:python bench.py --scene csg256_chain --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/bch.json" \
"bch_lds:150:WOLOLO_JIT_LDS_EVENTS=1 python bench.py --scene csg256_chain --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/bch_lds.json" \
"bbal:150:python bench.py --scene csg256_balanced --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/bbal.json" \
"rt_base:150:python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/rt_base.json" \
"rt_s16:150:WOLOLO_LANES_STACK16=1 python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/rt_s16.json" \
"rt_s16_tall:150:WOLOLO_LANES_STACK16=1 WOLOLO_LANES_TOP=600 python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/rt_s16_tall.json" \
"rt_tall:150:WOLOLO_LANES_TOP=600 python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/rt_tall.json" \
"rt_d0:150:WOLOLO_LANES_DEPTH=0 python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/rt_d0.json"
