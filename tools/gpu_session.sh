#!/usr/bin/env bash
# Runs GPU steps on the gpurun box, each under its own time limit.  A step that
# exits 0 or 1 (test failures) lets the session go on; anything else (fault,
# abort, segfault, timeout, a pytest-timeout) stops the session immediately.
#   tools/gpu_session.sh "<name>:<seconds>:<command>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
    name="${spec%%:*}"
    rest="${spec#*:}"
    secs="${rest%%:*}"
    cmd="${rest#*:}"
    echo "=== [$name] ($secs s): $cmd" | tee -a gpurun_out/session.log
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    # a pytest-timeout hit means a kernel may still be running: stop as for a timeout
    if [ "$rc" -eq 1 ] && grep -q "+++ Timeout +++" "gpurun_out/$name.log"; then rc=124; fi
    echo "=== [$name] rc=$rc after $(( $(date +%s) - start )) s" | tee -a gpurun_out/session.log
    tail -n 15 "gpurun_out/$name.log"
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
        echo "=== stopping: [$name] ended with rc=$rc" | tee -a gpurun_out/session.log
        exit "$rc"
    fi
done
