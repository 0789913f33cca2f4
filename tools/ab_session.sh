#!/usr/bin/env bash
# Round-2 session: N>1 rehearsals (frames in flight), chain evidence with the spatial collect,
# and per-rank shares with back-to-back frames on two streams.
S=tools/gpu_session.sh
bash $S \
 "dist:400:python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread" \
 "b256c:200:python bench.py --scene csg256_chain --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02_bench_256c.json" \
 "p256c:400:bash tools/profile_session.sh csg256c_jit --scene csg256_chain --steps 5 --warmup 1" \
 "rs256c:300:python tools/rank_share.py --scene csg256_chain --worlds 1 8 --reps 3 > gpurun_out/r02_share256c.log 2>&1" \
 "rs32s:300:python tools/rank_share.py --scene csg32 --worlds 8 --reps 3 --stream-frames 20 > gpurun_out/r02_share32_stream.log 2>&1" \
 "par:500:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k 'chain'"
