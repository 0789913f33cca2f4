cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_session.sh \
 "tests:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "b32:200:python bench.py > gpurun_out/ev_bench_csg32.json" \
 "b256b:200:python bench.py --scene csg256_balanced --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ev_bench_256b.json" \
 "b256c:200:python bench.py --scene csg256_chain --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ev_bench_256c.json" \
 "p32:400:bash tools/profile_session.sh csg32_jit --steps 10 --warmup 2" \
 "rs32:200:python tools/rank_share.py --scene csg32 --worlds 1 2 4 8 --reps 5 > gpurun_out/ev_share32.log 2>&1"
