cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_session.sh \
 "gloo8:400:python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 8 --dist-backend gloo --verify --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ev_gloo8.json 2> gpurun_out/ev_gloo8.err" \
 "gloo3:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 3 --dist-backend gloo --verify --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ev_gloo3.json 2> gpurun_out/ev_gloo3.err"
