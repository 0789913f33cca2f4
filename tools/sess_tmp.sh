tools/gpu_session.sh \
"p32:500:bash tools/profile_session.sh csg32_jit --steps 20 --warmup 5" \
"b32p:200:python bench.py --steps 20 --warmup 5 > gpurun_out/r03_bench_csg32.json" \
"tdist:400:python -u -m pytest tests/test_gpu_dist.py -m gpu -v --timeout 200 --timeout-method thread --maxfail=2"
