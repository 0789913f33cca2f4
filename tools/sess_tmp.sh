tools/gpu_session.sh \
"tpar:600:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frame.py -m gpu -v --timeout 150 --timeout-method thread --maxfail=4" \
"b32:150:python bench.py --scene csg32 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b32.json" \
"b32_ev:150:WOLOLO_JIT_TERMS=0 python bench.py --scene csg32 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b32_ev.json" \
"bbal:150:python bench.py --scene csg256_balanced --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bbal.json" \
"bbal_ev:150:WOLOLO_JIT_TERMS=0 python bench.py --scene csg256_balanced --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bbal_ev.json" \
"b32_l:150:python bench.py --scene csg32 --tracer lanes --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b32_l.json" \
"b4k:200:python bench.py --scene csg32 --width 3840 --height 2160 --spp 256 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b4k.json"
