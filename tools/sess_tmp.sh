tools/gpu_session.sh \
"diag:200:python tools/diag_async.py" \
"tlanes:500:python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 150 --timeout-method thread --maxfail=6 -k \"lanes or small_frame or full_size or auto\"" \
"b512l:200:python bench.py --scene csg512_balanced --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b512l.json" \
"brt:150:python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline --no-count-work > gpurun_out/brt.json" \
"bbal_l:150:python bench.py --scene csg256_balanced --tracer lanes --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bbal_l.json" \
"b32_l:150:python bench.py --scene csg32 --tracer lanes --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b32_l.json"
