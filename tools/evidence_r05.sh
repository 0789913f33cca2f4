#!/usr/bin/env bash
# Round-5 evidence on one GPU: bench lines for every config, rocprofv3 passes
# (kernel stats, HBM bytes, instruction mix) for every kernel the bench runs, and
# rank 0's N-GPU step with the present map-back for every config.  Results under
# gpurun_out/; tools/pmc_summary.py turns the profiles into profiles/ summaries.
#   tools/evidence_r05.sh bench|prof1|prof2|rs|rsnomap|final
# (a heartbeat line every 50 s: the specialised kernel of csg360_nested compiles for a
# minute or two, which the box's silence watchdog would take for a hang)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S=tools/gpu_session.sh
B="--no-cpu-baseline --no-draw-frame --side-scenes ''"
(while sleep 50; do echo "tick $(date +%s)"; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
case "${1:-bench}" in
bench)
    bash $S \
        "b32:300:python bench.py > gpurun_out/r05_bench_csg32.json" \
        "b32n:200:python bench.py --scene csg32_nested --steps 10 --warmup 2 $B > gpurun_out/r05_bench_csg32_nested.json" \
        "b256b:200:python bench.py --scene csg256_balanced --steps 10 --warmup 2 $B > gpurun_out/r05_bench_256b.json" \
        "b256c:200:python bench.py --scene csg256_chain --steps 10 --warmup 2 $B > gpurun_out/r05_bench_256c.json" \
        "brt:300:python bench.py --scene rtiow_cover --steps 5 --warmup 1 $B > gpurun_out/r05_bench_rtiow.json" \
        "b512:300:python bench.py --scene csg512_balanced --steps 5 --warmup 1 $B > gpurun_out/r05_bench_512b.json" \
        "b360:600:python bench.py --scene csg360_nested --steps 3 --warmup 1 $B > gpurun_out/r05_bench_csg360.json" \
        "bc4:300:python bench.py --width 3840 --height 2160 --spp 256 --steps 3 --warmup 1 $B > gpurun_out/r05_bench_c4.json"
    ;;
prof1)
    bash $S \
        "p32:400:bash tools/profile_session.sh r05_csg32 --steps 20 --warmup 3" \
        "p32n:400:bash tools/profile_session.sh r05_csg32_nested --scene csg32_nested --steps 10 --warmup 2" \
        "p256c:400:bash tools/profile_session.sh r05_csg256_chain --scene csg256_chain --steps 10 --warmup 2" \
        "p256b:400:bash tools/profile_session.sh r05_csg256_balanced --scene csg256_balanced --steps 10 --warmup 2"
    ;;
prof2)
    bash $S \
        "p512:500:bash tools/profile_session.sh r05_csg512 --scene csg512_balanced --steps 5 --warmup 1" \
        "prt:500:bash tools/profile_session.sh r05_rtiow --scene rtiow_cover --steps 5 --warmup 1" \
        "p360:600:bash tools/profile_session.sh r05_csg360 --scene csg360_nested --steps 2 --warmup 1"
    ;;
rs)
    bash $S \
        "rs32:300:python tools/root_step.py --scene csg32 --worlds 2 4 8 --map-back bgra > gpurun_out/r05_root_step_csg32.log 2>&1" \
        "rs32n:300:python tools/root_step.py --scene csg32_nested --worlds 2 4 8 --map-back bgra > gpurun_out/r05_root_step_csg32_nested.log 2>&1" \
        "rs256b:300:python tools/root_step.py --scene csg256_balanced --worlds 2 4 8 --map-back bgra > gpurun_out/r05_root_step_256b.log 2>&1" \
        "rs256c:300:python tools/root_step.py --scene csg256_chain --worlds 2 4 8 --map-back bgra > gpurun_out/r05_root_step_256c.log 2>&1" \
        "rsrt:300:python tools/root_step.py --scene rtiow_cover --worlds 2 4 8 --map-back bgra > gpurun_out/r05_root_step_rtiow.log 2>&1" \
        "rs512:300:python tools/root_step.py --scene csg512_balanced --worlds 2 4 8 --map-back bgra > gpurun_out/r05_root_step_512b.log 2>&1" \
        "rsc4:400:python tools/root_step.py --scene csg32 --width 3840 --height 2160 --spp 256 --worlds 2 4 8 --map-back bgra > gpurun_out/r05_root_step_c4.log 2>&1"
    ;;
final)
    # the round's last build: the nested tree's, csg360's and the headline's profiles
    # first (on a fresh box: two sessions that profiled the nested tree after other
    # scenes' runs measured ~1 GB of writes per launch that no fresh session repeats),
    # then every bench line
    bash $S \
        "p32n:400:bash tools/profile_session.sh r05j_csg32_nested --scene csg32_nested --steps 10 --warmup 2" \
        "p360:900:bash tools/profile_session.sh r05j_csg360 --scene csg360_nested --steps 3 --warmup 1" \
        "p32:400:bash tools/profile_session.sh r05j_csg32 --steps 20 --warmup 3" || exit $?
    bash "$0" bench
    ;;
rsnomap)
    # the same without the present map-back (bench.py's N-GPU frame is not presented)
    for sc in csg32 csg32_nested csg256_balanced csg256_chain rtiow_cover csg512_balanced; do
        bash $S "nm_$sc:300:python tools/root_step.py --scene $sc --worlds 2 4 8 --map-back none > gpurun_out/r05_root_step_nomap_$sc.log 2>&1" || exit $?
    done
    ;;
esac
