#!/usr/bin/env bash
# Cache / LDS / instruction-fetch counters of one bench configuration (round 6:
# VERDICT r5 item 4 -- where a kernel's memory waits come from).  One rocprofv3
# pass per counter group, each under its own time limit:
#   c1  L2 hits and misses (TCC), vector-memory and LDS instructions, LDS conflicts
#   c2  vector L1 (TCP): accesses, misses to L2, their latency, pending stalls
#   c3  instruction cache (SQC): hits and misses
# Outputs under gpurun_out/cache_<tag>/; tools/cache_summary.py reads them.
#   tools/cache_profile.sh <tag> [bench.py args ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag="$1"
shift
out="gpurun_out/cache_$tag"
mkdir -p "$out"
run() {
    local name="$1"
    shift
    timeout -s KILL 240 rocprofv3 "$@" -d "$out/$name" -o "$name" --output-format csv -- \
        python3 bench.py --no-cpu-baseline --no-count-work --no-draw-frame --side-scenes "" "${BENCH_ARGS[@]}" > "$out/$name.log" 2>&1
    local rc=$?
    echo "[$tag/$name] rc=$rc"
    return $rc
}
BENCH_ARGS=("$@")
run c1 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_FLAT SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS &&
    run c2 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum &&
    run c3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES
