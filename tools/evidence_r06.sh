#!/usr/bin/env bash
# Round-6 evidence on one GPU: rocprofv3 passes (kernel stats, HBM bytes,
# instruction mix; every pass records the code object it ran) for every kernel the
# bench runs, then bench lines for every config.  Results under gpurun_out/;
# tools/pmc_summary.py turns the profiles into profiles/ summaries.
#   tools/evidence_r06.sh prof1|prof2|bench
# (a heartbeat line every 50 s: csg360_nested's kernel compiles for a minute or two)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S=tools/gpu_session.sh
B="--no-cpu-baseline --no-draw-frame --side-scenes ''"
(while sleep 50; do echo "tick $(date +%s)"; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
case "${1:-bench}" in
prof1)
    bash $S \
        "p32:400:bash tools/profile_session.sh r06_csg32 --steps 20 --warmup 3" \
        "p32n:400:bash tools/profile_session.sh r06_csg32_nested --scene csg32_nested --steps 10 --warmup 2" \
        "p256c:400:bash tools/profile_session.sh r06_csg256_chain --scene csg256_chain --steps 10 --warmup 2" \
        "p256b:400:bash tools/profile_session.sh r06_csg256_balanced --scene csg256_balanced --steps 10 --warmup 2"
    ;;
prof2)
    bash $S \
        "p512:500:bash tools/profile_session.sh r06_csg512 --scene csg512_balanced --steps 5 --warmup 1" \
        "prt:500:bash tools/profile_session.sh r06_rtiow --scene rtiow_cover --steps 5 --warmup 1" \
        "p360:900:bash tools/profile_session.sh r06_csg360 --scene csg360_nested --steps 3 --warmup 1" \
        "pc4:600:bash tools/profile_session.sh r06_c4 --width 3840 --height 2160 --spp 256 --steps 3 --warmup 1"
    ;;
bench)
    bash $S \
        "b32:300:python bench.py > gpurun_out/r06_bench_csg32.json" \
        "b256b:200:python bench.py --scene csg256_balanced --steps 10 --warmup 2 $B > gpurun_out/r06_bench_256b.json" \
        "b256c:200:python bench.py --scene csg256_chain --steps 10 --warmup 2 $B > gpurun_out/r06_bench_256c.json" \
        "brt:300:python bench.py --scene rtiow_cover --steps 5 --warmup 1 $B > gpurun_out/r06_bench_rtiow.json" \
        "b512:300:python bench.py --scene csg512_balanced --steps 5 --warmup 1 $B > gpurun_out/r06_bench_512b.json" \
        "b360:900:python bench.py --scene csg360_nested --steps 3 --warmup 1 $B > gpurun_out/r06_bench_csg360.json" \
        "bc4:300:python bench.py --width 3840 --height 2160 --spp 256 --steps 3 --warmup 1 $B > gpurun_out/r06_bench_c4.json"
    ;;
esac
