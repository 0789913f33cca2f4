tools/gpu_session.sh \
"twide:300:python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 150 --timeout-method thread --maxfail=3 -k wide" \
"brt:150:python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/brt.json" \
"brt_w:150:WOLOLO_LANES_WIDE=1 python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/brt_w.json" \
"b32:150:python bench.py --scene csg32 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b32.json" \
"b32_dc:150:WOLOLO_JIT_DIST_CULL=1 python bench.py --scene csg32 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b32_dc.json" \
"bbal_dc:150:WOLOLO_JIT_DIST_CULL=1 python bench.py --scene csg256_balanced --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bbal_dc.json" \
"b32_ev:150:WOLOLO_JIT_TERMS=0 python bench.py --scene csg32 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b32_ev.json" \
"bbal:150:python bench.py --scene csg256_balanced --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bbal.json" \
"bbal_ev:150:WOLOLO_JIT_TERMS=0 python bench.py --scene csg256_balanced --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bbal_ev.json" \
"b512:150:python bench.py --scene csg512_balanced --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b512.json" \
"b512_w:150:WOLOLO_LANES_WIDE=1 python bench.py --scene csg512_balanced --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b512_w.json" \
"tpar:700:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frame.py -m gpu -v --timeout 150 --timeout-method thread --maxfail=4"
