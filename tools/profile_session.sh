#!/usr/bin/env bash
# rocprofv3 passes over one bench configuration, for the roofline and the
# counter analysis in DESIGN.md:
#   kstats  --kernel-trace --stats          per-kernel durations
#   fetch / write                            HBM bytes (separate --pmc passes)
#   pmc1 / pmc2                              instruction mix, wave cycles, lane use
# Outputs go to gpurun_out/prof_<tag>/; tools/pmc_summary.py reads them.
#   tools/profile_session.sh <tag> [bench.py args ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag="$1"
shift
out="gpurun_out/prof_$tag"
mkdir -p "$out"
run() {
    local name="$1"
    shift
    timeout -k 10 300 rocprofv3 "$@" -d "$out/$name" -o "$name" --output-format csv -- \
        python3 bench.py --no-cpu-baseline --no-count-work --no-draw-frame --side-scenes "" "${BENCH_ARGS[@]}" > "$out/$name.log" 2>&1
    local rc=$?
    # the code object this pass ran (key, scratch bytes per lane, VGPRs): the summary
    # checks that every pass ran the same one
    echo "[$tag/$name] rc=$rc kernel_object=$(python3 -c 'import json,sys
for l in open(sys.argv[1], errors="replace"):
    if l.startswith("{") and "\"roofline\"" in l: print(json.dumps(json.loads(l)["roofline"].get("kernel_object")))' "$out/$name.log" 2>/dev/null)"
    return $rc
}
BENCH_ARGS=("$@")
run kstats --kernel-trace --stats &&
    run fetch --pmc FETCH_SIZE &&
    run write --pmc WRITE_SIZE &&
    run pmc1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE &&
    run pmc2 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY
