cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_session.sh \
 "tests:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "b32:200:python bench.py > gpurun_out/ev_bench_csg32.json" \
 "b256b:200:python bench.py --scene csg256_balanced --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ev_bench_256b.json" \
 "b256c:200:python bench.py --scene csg256_chain --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ev_bench_256c.json" \
 "bc4:300:python bench.py --width 3840 --height 2160 --spp 256 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ev_bench_c4.json" \
 "p32:400:bash tools/profile_session.sh csg32_jit --steps 10 --warmup 2" \
 "p256:400:bash tools/profile_session.sh csg256_jit --scene csg256_balanced --steps 5 --warmup 1" \
 "rs32:200:python tools/rank_share.py --scene csg32 --worlds 1 2 4 8 --reps 5 > gpurun_out/ev_share32.log 2>&1" \
 "rs4k:300:python tools/rank_share.py --scene csg32 --width 3840 --height 2160 --spp 256 --worlds 1 8 --reps 3 > gpurun_out/ev_share4k.log 2>&1" \
 "gloo2:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --verify --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ev_gloo2.json 2> gpurun_out/ev_gloo2.err"
