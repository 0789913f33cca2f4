#!/usr/bin/env bash
# Round-2 evidence on one GPU: bench lines for every config, rocprofv3 passes
# (kernel stats, HBM bytes, instruction mix) and per-rank shares.  Results under
# gpurun_out/; tools/pmc_summary.py turns the profiles into profiles/ summaries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
# groups (one gpurun call each keeps a call short): bench | prof | share | all
S=tools/gpu_session.sh
group="${1:-all}"
if [ "$group" = bench ] || [ "$group" = all ]; then
bash $S \
 "b32:200:python bench.py > gpurun_out/r02_bench_csg32.json" \
 "b256b:200:python bench.py --scene csg256_balanced --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02_bench_256b.json" \
 "b256c:200:python bench.py --scene csg256_chain --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02_bench_256c.json" \
 "brt:300:python bench.py --scene rtiow_cover --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r02_bench_rtiow.json" \
 "bs256:300:python bench.py --scene sphere256 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r02_bench_sphere256.json" \
 "bc4:300:python bench.py --width 3840 --height 2160 --spp 256 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02_bench_c4.json" || exit $?
fi
if [ "$group" = prof ] || [ "$group" = all ]; then
bash $S \
 "p32:400:bash tools/profile_session.sh csg32_jit --steps 10 --warmup 2" \
 "p256b:400:bash tools/profile_session.sh csg256b_jit --scene csg256_balanced --steps 5 --warmup 1" \
 "p256c:400:bash tools/profile_session.sh csg256c_jit --scene csg256_chain --steps 5 --warmup 1" \
 "prt:500:bash tools/profile_session.sh rtiow_lanes --scene rtiow_cover --steps 3 --warmup 1" || exit $?
fi
if [ "$group" = share ] || [ "$group" = all ]; then
bash $S \
 "rs32:200:python tools/rank_share.py --scene csg32 --worlds 1 2 4 8 --reps 5 > gpurun_out/r02_share32.log 2>&1" \
 "rs256b:300:python tools/rank_share.py --scene csg256_balanced --worlds 1 8 --reps 3 > gpurun_out/r02_share256b.log 2>&1" \
 "rs256c:300:python tools/rank_share.py --scene csg256_chain --worlds 1 8 --reps 3 > gpurun_out/r02_share256c.log 2>&1" \
 "rsrt:300:python tools/rank_share.py --scene rtiow_cover --worlds 1 8 --reps 3 > gpurun_out/r02_sharert.log 2>&1" \
 "rs4k:300:python tools/rank_share.py --scene csg32 --width 3840 --height 2160 --spp 256 --worlds 1 8 --reps 3 > gpurun_out/r02_share4k.log 2>&1"
fi
