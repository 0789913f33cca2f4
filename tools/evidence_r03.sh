#!/usr/bin/env bash
# Round-3 evidence on one GPU: bench lines for every config, the headline's
# rocprofv3 passes (kernel stats, HBM bytes, instruction mix), rank 0's N-GPU
# step and the section profile.  Results under gpurun_out/; tools/pmc_summary.py
# turns the profiles into profiles/ summaries.
#   tools/evidence_r03.sh bench|prof|all
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S=tools/gpu_session.sh
group="${1:-all}"
if [ "$group" = bench ] || [ "$group" = all ]; then
bash $S \
 "b32:200:python bench.py > gpurun_out/r03_bench_csg32.json" \
 "b32n:200:python bench.py --scene csg32_nested --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03_bench_csg32_nested.json" \
 "b256b:200:python bench.py --scene csg256_balanced --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03_bench_256b.json" \
 "b256c:200:python bench.py --scene csg256_chain --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03_bench_256c.json" \
 "brt:300:python bench.py --scene rtiow_cover --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r03_bench_rtiow.json" \
 "bs256:300:python bench.py --scene sphere256 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r03_bench_sphere256.json" \
 "b512:300:python bench.py --scene csg512_balanced --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r03_bench_512b.json" \
 "bc4:300:python bench.py --width 3840 --height 2160 --spp 256 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03_bench_c4.json" || exit $?
fi
if [ "$group" = prof ] || [ "$group" = all ]; then
bash $S \
 "p32:500:bash tools/profile_session.sh csg32_jit --steps 20 --warmup 3" \
 "b32p:200:python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r03_bench_csg32_profbox.json" \
 "rs32:300:python tools/root_step.py --scene csg32 --worlds 2 4 8 > gpurun_out/r03_root_step_csg32.log 2>&1" \
 "wp:300:python tools/work_profile.py csg32 csg256_balanced csg256_chain > gpurun_out/r03_work_profile.log 2>&1" || exit $?
fi
